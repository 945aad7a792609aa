"""Probe: the flat tiled SpMM at panel width 16 against width 8 on one cfg4-shaped ER layer
(N = 1M, degree 50): HIP-event ms per launch over column-block counts, and the b = 16 result
against scipy (fp64) on the same panel."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
deg = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
A = synthetic.er_layer_rows(n, deg, 1000)
eng = _lib.Engine(0)
eng.set_layers([A])
rng = np.random.default_rng(0)
X16 = rng.standard_normal((n, 16)).astype(np.float32)
X8 = np.ascontiguousarray(X16[:, :8])
ref = None
for rnd in range(2):
    combos = [(8, 16, 0), (16, 16, 0)]
    if len(sys.argv) > 3:  # "b:nb:cap,..."
        combos = [tuple(int(v) for v in c.split(":")) for c in sys.argv[3].split(",")]
    for b, nb, cap in combos:
        if cap:
            os.environ["N2V2R_SPMM_TILE_CAP"] = str(cap)
        else:
            os.environ.pop("N2V2R_SPMM_TILE_CAP", None)
        X = X16 if b == 16 else X8
        Y, ms = eng.bench_spmm_tiled(0, X, nb=nb, reps=20, want_y=(rnd == 0))
        err = None
        if rnd == 0:
            if ref is None:
                ref = A.astype(np.float64) @ X16.astype(np.float64)
            r = ref[:, :b]
            err = float(np.max(np.abs(Y - r)) / np.max(np.abs(r)))
        print(json.dumps({"b": b, "nb": nb, "cap": cap, "round": rnd, "ms": round(ms, 4),
                          "G_entries_per_s": round(A.nnz / ms / 1e6, 1),
                          "ms_per_vector": round(ms / b, 5), "rel_err": err}), flush=True)
