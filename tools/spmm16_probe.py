"""Flat-window tiled SpMM at panel width 16 vs 8 (one layer, HIP events), cfg4-sized ER layer:
the per-entry line cost that decides whether b = 16 halves the SpMM per vector.

    python tools/spmm16_probe.py [--n 1000000] [--deg 50] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from node2vec2rank_amd import _lib, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--deg", type=float, default=50.0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--widths", type=int, nargs="+", default=[8, 16])
    a = ap.parse_args()
    layers = synthetic.er_layers(a.n, a.deg, 2, seed_base=1000)
    A = layers[0]
    eng = _lib.Engine(0)
    eng.set_layers(layers)
    rng = np.random.default_rng(5)
    rows = rng.choice(a.n, 2000, replace=False)
    plan = {8: (0, 16, 32), 16: (0, 16, 32, 64)}
    for b, nbs in ((w, plan[w]) for w in a.widths):
        X = rng.standard_normal((a.n, b)).astype(np.float32)
        ref = (A[rows] @ X.astype(np.float64))
        for nb in nbs:
            Y, ms = eng.bench_spmm_tiled(0, X, nb=nb, reps=a.reps)
            err = float(np.abs(Y[rows] - ref).max() / np.abs(ref).max())
            print(json.dumps(dict(b=b, nb=nb, ms=round(ms, 4), nnz=int(A.nnz),
                                  G_entries_per_s=round(A.nnz / ms / 1e6, 1),
                                  G_vector_entries_per_s=round(A.nnz * b / ms / 1e6, 1),
                                  rel_err=err,
                                  t16_rows=os.environ.get("N2V2R_T16_ROWS"),
                                  sched=os.environ.get("N2V2R_FLAT_SCHED"))), flush=True)


if __name__ == "__main__":
    main()
