"""Probe: BASELINE cfg3 (dense |corr| layers, N = 20k, d = 256) and the CSR lowrank_exact fit under
the library named by N2V2R_LIB; prints the solver statistics (N2V2R_TRACE=1 for per-cycle lines).
Usage: python tools/probe_cfg3.py [cfg3] [lowrank]"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from node2vec2rank_amd import _lib, synthetic  # noqa: E402

what = sys.argv[1:] or ["cfg3", "lowrank"]
eng = _lib.Engine(0)
print("lib", _lib.LIB_PATH, flush=True)
if "cfg3" in what:
    layers = synthetic.corr_layers(20_000, 4)
    eng.set_layers(layers, storage="dense", symmetric=1)
    for seed in (42,):
        t = time.time()
        st = eng.uase(256, seed=seed, raise_on_no_convergence=False)
        print(f"cfg3 seed {seed}: {time.time() - t:.2f} s", st, flush=True)
    del layers
for kind in ("lowrank", "lowrank_dense"):
    if kind not in what:
        continue
    from conftest import load_fixture
    from test_oracle_golden import lowrank_exact_layers
    fx = load_fixture("lowrank_exact")
    if kind == "lowrank":
        eng.set_layers([sp.csr_matrix(a) for a in lowrank_exact_layers(fx)])
    else:
        eng.set_layers(lowrank_exact_layers(fx), storage="dense")
    print(kind, flush=True)
    st = eng.uase(8, seed=int(fx["seed"]), raise_on_no_convergence=False)
    print(kind, st, eng._err(), flush=True)
    if st["converged"]:
        print("sigma err", np.max(np.abs(eng.singular_values() / fx["sigma"] - 1)), flush=True)
eng.close()
