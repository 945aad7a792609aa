"""SpMM A/B: row kernel vs XCD-local column blocks (bench_spmm, HIP events) over graph sizes.
Usage: python tools/cb_probe.py [n:deg ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

sizes = sys.argv[1:] or ["100000:20", "300000:30", "1000000:50"]
eng = _lib.Engine(0)
for spec in sizes:
    n, deg = spec.split(":")
    n, deg = int(n), float(deg)
    t0 = time.time()
    if n > 3_000_000:
        A = synthetic.er_layer_rows(n, deg, 2000, 0, n)
    else:
        A = synthetic.er_layer(n, deg, 2000)
    eng.set_layers([A], symmetric=1)
    X = np.random.default_rng(0).standard_normal((n, 8)).astype(np.float32)
    out = {}
    for cb in ("0", "1"):
        os.environ["N2V2R_SPMM_CB"] = cb
        _, ms, by = eng.bench_spmm(0, X, reps=20, want_y=False)
        out[cb] = ms
    print(f"n={n} deg={deg} nnz={A.nnz} row={out['0']*1e3:.1f}us cb={out['1']*1e3:.1f}us "
          f"ratio={out['0']/out['1']:.2f} (setup {time.time()-t0:.1f}s)", flush=True)
    del A, X
