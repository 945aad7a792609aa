"""Basis / keep sweep of the dense-layer fit at cfg3 (N = 20k |corrcoef|, K = 4, d = 256, b = 32):
block applications, restarts and fit time per (keep, max_basis), each setting fitted twice.

    python tools/sweep_cfg3.py [--n 20000] [--d 256]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from node2vec2rank_amd import _lib, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--keeps", type=int, nargs="+", default=[288, 320, 352])
    ap.add_argument("--bases", type=int, nargs="+", default=[576, 640, 704, 768])
    ap.add_argument("--pairs", nargs="*", default=None, help="keep:basis pairs instead of the grid")
    ap.add_argument("--seed-base", type=int, default=0, help="graph family member (synthetic)")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    layers = synthetic.corr_layers(a.n, 4, seed_base=a.seed_base)
    eng = _lib.Engine(0)
    eng.set_layers(layers)
    eng.uase(a.d, seed=42)  # warm-up (workspace, first-fit allocations)
    grid = ([tuple(int(v) for v in q.split(":")) for q in a.pairs] if a.pairs
            else list(itertools.product(a.keeps, a.bases)))
    for keep, basis in grid:
        if basis < keep + 64:
            continue
        for rep in range(a.reps):
            st = eng.uase(a.d, seed=42, keep=keep, max_basis=basis, raise_on_no_convergence=False)
            print(json.dumps(dict(seed_base=a.seed_base, keep=keep, basis=basis, rep=rep, ms=round(st["ms_total"], 1),
                                  apps=st["block_applications"], restarts=st["restarts"],
                                  converged=st["converged"], max_residual=st["max_residual"])),
                  flush=True)


if __name__ == "__main__":
    main()
