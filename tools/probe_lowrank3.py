"""Probe 3: the lowrank_exact CSR fit (b = 8) with N2V2R_DEBUG_ORTHO=1 / N2V2R_TRACE=1: where the
first Krylov block leaves orthonormality."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import scipy.sparse as sp  # noqa: E402
from conftest import load_fixture  # noqa: E402
from test_oracle_golden import lowrank_exact_layers  # noqa: E402

from node2vec2rank_amd import _lib  # noqa: E402

fx = load_fixture("lowrank_exact")
layers = [sp.csr_matrix(a) for a in lowrank_exact_layers(fx)]
e = _lib.Engine(0)
e.set_layers(layers)
st = e.uase(8, seed=42, max_restarts=int(sys.argv[1]) if len(sys.argv) > 1 else 3,
            solver_flags=int(sys.argv[2]) if len(sys.argv) > 2 else 0,
            raise_on_no_convergence=False)
print({k: st[k] for k in ("restarts", "block_applications", "converged", "max_residual")},
      e.singular_values()[:3])
