"""Probe: the lowrank_exact fixture (rank-8 dense layers) through the CSR path (b = 8) under
several solver settings; prints the eig stats of each (N2V2R_TRACE=1 logs the cycles)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

CASES = [("default", {}), ("no_lean", {"N2V2R_LEAN_W": "0"}), ("band", {"N2V2R_RR": "band"}),
         ("no_defer", {"N2V2R_REORTH_DEFER": "0"}), ("reorth0", {"N2V2R_REORTH_TOL": "0"})]

if len(sys.argv) == 1:
    for name, env in CASES:
        e = dict(os.environ, N2V2R_TRACE="1", **env)
        print(f"==== {name} {env}", flush=True)
        subprocess.run([sys.executable, __file__, name], env=e, timeout=120)
    sys.exit(0)

import numpy as np
import scipy.sparse as sp
from conftest import load_fixture
from test_oracle_golden import lowrank_exact_layers
from node2vec2rank_amd import _lib

fx = load_fixture("lowrank_exact")
layers = [sp.csr_matrix(a) for a in lowrank_exact_layers(fx)]
eng = _lib.Engine(0)
eng.set_layers(layers)
st = eng.uase(8, seed=42, raise_on_no_convergence=False)
print({k: st[k] for k in ("restarts", "block_applications", "converged", "max_residual",
                          "stagnated", "basis", "rr_fallbacks", "est_scale", "lean_checks")})
s = eng.singular_values()
print("sigma", s, "ref", fx["sigma"])
