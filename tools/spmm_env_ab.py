"""A/B probe of a tiled-SpMM switch read per launch: one ER layer (N, degree from argv), the
fit's column-block rule, HIP-event ms per layer launch, alternating the values of one
environment variable over rounds; every value's output compared bit for bit with the first's.
Usage: python tools/spmm_env_ab.py N DEG VAR v1,v2,... [rounds]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n, deg, var = int(sys.argv[1]), float(sys.argv[2]), sys.argv[3]
vals = sys.argv[4].split(",")
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 3
A = synthetic.er_layer_rows(n, deg, 1000)
eng = _lib.Engine(0)
eng.set_layers([A])
X = np.random.default_rng(0).standard_normal((n, 8)).astype(np.float32)
ys = {}
for r in range(rounds):
    for v in vals:
        os.environ[var] = v
        Y, ms = eng.bench_spmm_tiled(0, X, nb=0, reps=10, want_y=(r == 0))
        if r == 0:
            ys[v] = Y
        print(json.dumps({"n": n, "deg": deg, var: v, "round": r, "ms": round(ms, 4),
                          "G_entries_per_s": round(A.nnz / ms / 1e6, 1)}), flush=True)
print(json.dumps({"bit_identical_to_" + vals[0]: {v: bool(np.array_equal(ys[vals[0]], ys[v]))
                                                   for v in vals}}), flush=True)
eng.close()
