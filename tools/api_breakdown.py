"""Where the drop-in API's time goes at a config (GPU): layer conversion + upload + GPU ingest,
the first fit (column-block build included) vs a refit, ranking, frames, Borda of the frames.

    python tools/api_breakdown.py [--config cfg4|cfg2|cfg3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from node2vec2rank_amd import _lib, synthetic  # noqa: E402
from node2vec2rank_amd.model import N2V2R, _as_layer  # noqa: E402

CONFIGS = {
    "cfg2": dict(n=100_000, avg_deg=20.0, dims=[64]),
    "cfg4": dict(n=1_000_000, avg_deg=50.0, dims=[8, 16, 32, 64, 128]),
    "cfg3": dict(n=20_000, dense_layers=4, dims=[256]),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4", choices=sorted(CONFIGS))
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    if cfg.get("dense_layers"):
        layers = synthetic.corr_layers(cfg["n"], cfg["dense_layers"], seed_base=0)
    else:
        layers = synthetic.er_layers(cfg["n"], cfg["avg_deg"], 2, seed_base=1000)
    nodes = [f"n{i}" for i in range(cfg["n"])]
    config = dict(embed_dimensions=cfg["dims"], distance_metrics=["cosine", "euclidean"],
                  comp_strategy="sequential", seed=42, verbose=-1)
    out = {}
    for rep in range(2):
        t = {}
        t0 = time.perf_counter()
        conv = [_as_layer(g) for g in layers]
        t["as_layer"] = time.perf_counter() - t0
        if cfg.get("dense_layers"):
            t0 = time.perf_counter()
            _lib._denser_than_quarter(np.asarray(conv[0]))
            t["density_test_one_layer"] = time.perf_counter() - t0
        eng = _lib.Engine(0)
        t0 = time.perf_counter()
        eng.set_layers(conv)
        eng.synchronize()
        t["set_layers"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        eng.uase(max(cfg["dims"]), seed=42)
        t["uase_first"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        eng.uase(max(cfg["dims"]), seed=42)
        t["uase_again"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        eng.rank("sequential", cfg["dims"], ["cosine", "euclidean"], method=_lib.AGG_NONE)
        t["rank"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        D = eng.distances(0)
        t["distances_d2h"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        b = eng.borda_columns(D)
        t["borda_columns"] = time.perf_counter() - t0
        eng.close()
        del b
        # the whole API call
        t0 = time.perf_counter()
        m = N2V2R(layers, nodes, config)
        m.fit_transform_rank()
        t["api_fit_transform_rank"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        m.aggregate_transform()
        t["api_aggregate"] = time.perf_counter() - t1
        t["api_total"] = time.perf_counter() - t0
        t["api_stage_seconds"] = {k: round(v, 4) for k, v in m.stage_seconds.items()}
        out[f"rep{rep}"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()}
        del m
    print(json.dumps({"config": args.config, **out}))


if __name__ == "__main__":
    main()
