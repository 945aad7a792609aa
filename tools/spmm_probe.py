"""SpMM-only probe for rocprofv3 PMC passes: cfg2 layer 0, panel widths 8 and 32."""
import sys

import numpy as np

sys.path.insert(0, ".")
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
deg = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
eng = _lib.Engine(0)
eng.set_layers(synthetic.er_layers(n, deg, 2))
for b in (8, 32):
    X = np.random.default_rng(0).standard_normal((n, b)).astype(np.float32)
    _, ms, by = eng.bench_spmm(0, X, reps=20, want_y=False)
    print(f"b={b} avg_ms={ms:.5f} algo_bytes={by:.0f} GBps={by / ms / 1e6:.1f}", flush=True)
