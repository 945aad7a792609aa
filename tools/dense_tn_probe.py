"""Dense GEMM forms A/B at cfg3 size (N = 20k |corrcoef| layers, b = 32, HIP events): the
B-operand streaming dense_tn_kernel (default) against the LDS-staged dense_gemm_kernel
(N2V2R_DENSE_TN=0, read per call): one-layer launches, then whole fits with the forms named by
--fit-forms.  (profiles/r04_dense_forms.jsonl also holds two dropped variants: dense_tn at
16 / 24 k pairs per stage and one workgroup per CU, and the LDS kernel with X prefetched.)

    python tools/dense_tn_probe.py [--n 20000] [--layers 4] [--reps 10] [--fits 1] [--d 256]
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
    ap.add_argument("--n", type=int, default=20_000)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--fits", type=int, default=1)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--fit-forms", nargs="+", default=["tn", "lds"])
    a = ap.parse_args()
    layers = synthetic.corr_layers(a.n, a.layers, seed_base=0)
    eng = _lib.Engine(0)
    eng.set_layers(layers)
    rng = np.random.default_rng(5)
    X = rng.standard_normal((a.n, 32)).astype(np.float32)
    rows = rng.choice(a.n, 500, replace=False)
    ref = layers[0][rows].astype(np.float64) @ X.astype(np.float64)
    forms = {"tn": "1", "lds": "0"}
    for rep in range(2):
        for form, tn in forms.items():
            os.environ["N2V2R_DENSE_TN"] = tn
            Y, ms, by = eng.bench_spmm(0, X, reps=a.reps)
            err = float(np.abs(Y[rows] - ref).max() / np.abs(ref).max())
            print(json.dumps(dict(form=form, rep=rep,
                                  launch_ms=round(ms, 4), TB_per_s=round(by / ms / 1e9, 2),
                                  TFLOP_per_s=round(2.0 * a.n * a.n * 32 / ms / 1e9, 1),
                                  rel_err=err)), flush=True)
    for rep in range(a.fits):
        for form in a.fit_forms:
            os.environ["N2V2R_DENSE_TN"] = forms[form]
            t0 = time.time()
            st = eng.uase(a.d, seed=42)
            print(json.dumps(dict(form=form, fit=rep,
                                  wall_ms=round((time.time() - t0) * 1e3, 1),
                                  ms_total=round(st["ms_total"], 1),
                                  apps=st["block_applications"],
                                  max_residual=st["max_residual"])), flush=True)


if __name__ == "__main__":
    main()
