"""cProfile of one drop-in API call (fit_transform_rank + aggregate_transform) at a config, after
a warm-up call: where the host-side time of the call goes beside the fit.

    python tools/api_profile.py [--config cfg4|cfg2]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from node2vec2rank_amd import synthetic  # noqa: E402
from node2vec2rank_amd.model import N2V2R  # noqa: E402

CONFIGS = {"cfg2": (100_000, 20.0, [64]), "cfg4": (1_000_000, 50.0, [8, 16, 32, 64, 128])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4", choices=sorted(CONFIGS))
    a = ap.parse_args()
    n, deg, dims = CONFIGS[a.config]
    layers = synthetic.er_layers(n, deg, 2, seed_base=1000)
    nodes = [f"n{i}" for i in range(n)]
    config = dict(embed_dimensions=dims, distance_metrics=["cosine", "euclidean"],
                  comp_strategy="sequential", seed=42, verbose=-1)
    m = N2V2R(layers, nodes, config)
    m.fit_transform_rank()
    m.aggregate_transform()
    del m
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    m = N2V2R(layers, nodes, config)
    m.fit_transform_rank()
    m.aggregate_transform()
    pr.disable()
    print(f"call {time.perf_counter() - t0:.4f} s  stages {m.stage_seconds}")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
