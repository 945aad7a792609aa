"""Flat tiled SpMM knobs A/B on a cfg4-sized ER graph (read per launch by the library):
N2V2R_FLAT_NT (non-temporal index / value loads, default on) and N2V2R_FLAT_BAR (the barrier
between column-block phases, default on).  (profiles/r04_flat_sync.jsonl came from a bounded-skew
variant, N2V2R_FLAT_SYNC=2, since dropped.)  One-layer launches, then whole fits, alternating in one
process.

    python tools/flat_knob_probe.py [--n 1000000] [--deg 50] [--reps 20] [--fits 1] [--d 128]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--deg", type=float, default=50.0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--fits", type=int, default=1)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--var", default="N2V2R_FLAT_NT")
    ap.add_argument("--modes", nargs="+", default=["1", "0"])
    a = ap.parse_args()
    layers = synthetic.er_layers(a.n, a.deg, 2, seed_base=1000)
    A = layers[0]
    eng = _lib.Engine(0)
    eng.set_layers(layers)
    rng = np.random.default_rng(5)
    X = rng.standard_normal((a.n, 8)).astype(np.float32)
    for rep in range(2):
        for mode in a.modes:
            os.environ[a.var] = mode
            Y, ms = eng.bench_spmm_tiled(0, X, nb=16, reps=a.reps, want_y=False)
            print(json.dumps(dict(var=a.var, value=mode, rep=rep, layer_launch_ms=round(ms, 4),
                                  G_entries_per_s=round(A.nnz / ms / 1e6, 1))), flush=True)
    for rep in range(a.fits):
        for mode in a.modes:
            os.environ[a.var] = mode
            t0 = time.time()
            st = eng.uase(a.d, seed=42)
            print(json.dumps(dict(var=a.var, value=mode, fit=rep, wall_ms=round((time.time() - t0) * 1e3, 1),
                                  ms_total=round(st["ms_total"], 1),
                                  apps=st["block_applications"],
                                  max_residual=st["max_residual"])), flush=True)


if __name__ == "__main__":
    main()
