"""Tiled-SpMM column-block count probe: one ER layer (N, degree from argv; cfg5 by default),
the flat-window tiled SpMM of layer 0 at 8..64 column blocks (argv[3]) and window bits 5..7
(argv[4], "auto": the library's rule), HIP-event ms per launch."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
deg = float(sys.argv[2]) if len(sys.argv) > 2 else 30.0
blocks = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [8, 16, 32, 64]
wbs = sys.argv[4].split(",") if len(sys.argv) > 4 else ["auto"]
t0 = time.time()
A = synthetic.er_layer_rows(n, deg, 1000)
print(f"layer built {time.time() - t0:.1f}s nnz {A.nnz}", flush=True)
eng = _lib.Engine(0)
eng.set_layers([A])
X = np.random.default_rng(0).standard_normal((n, 8)).astype(np.float32)
Y0 = None
for rnd in range(2):
    for nb in blocks:
        for wb in wbs:
            if wb == "auto":
                os.environ.pop("N2V2R_SPMM_WBITS", None)
            else:
                os.environ["N2V2R_SPMM_WBITS"] = wb
            Y, ms = eng.bench_spmm_tiled(0, X, nb=nb, reps=10, want_y=(rnd == 0))
            same = None
            if rnd == 0:
                if Y0 is None:
                    Y0 = Y
                same = float(np.max(np.abs(Y - Y0)))
            print(json.dumps({"n": n, "deg": deg, "nb": nb, "wbits": wb, "round": rnd,
                              "ms": round(ms, 4), "G_entries_per_s": round(A.nnz / ms / 1e6, 1),
                              "max_diff_vs_first": same}), flush=True)
