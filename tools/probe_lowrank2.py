"""Probe 2: the lowrank_exact CSR failure -- SpMM vs scipy on the fixture's layers (rows of 2000
entries, negative weights), and the fit under variants that separate the exact low rank from
the storage (dense rank-8 layers as CSR; the same layers with a small full-rank perturbation)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from conftest import load_fixture  # noqa: E402
from test_oracle_golden import lowrank_exact_layers  # noqa: E402

from node2vec2rank_amd import _lib  # noqa: E402

fx = load_fixture("lowrank_exact")
dense = lowrank_exact_layers(fx)
layers = [sp.csr_matrix(a) for a in dense]
eng = _lib.Engine(0)
eng.set_layers(layers)
X = np.random.default_rng(1).standard_normal((2000, 8)).astype(np.float32)
for k, A in enumerate(layers):
    for tr in (False, True):
        Y, _, _ = eng.bench_spmm(k, X, transpose=tr, reps=1)
        M = (A.T if tr else A).astype(np.float64)
        ref = M @ X.astype(np.float64)
        print(f"spmm layer {k} transpose {tr}: max abs err {np.abs(Y - ref).max():.3e}, "
              f"ref scale {np.abs(ref).max():.3e}", flush=True)


def fit(name, L, **kw):
    e = _lib.Engine(0)
    e.set_layers(L, **{k: v for k, v in kw.items() if k in ("symmetric", "storage")})
    st = e.uase(8, seed=42, raise_on_no_convergence=False,
                **{k: v for k, v in kw.items() if k in ("block", "solver_flags")})
    print(name, {k: st[k] for k in ("restarts", "block_applications", "converged",
                                    "max_residual")}, "sigma[0:3]", e.singular_values()[:3],
          flush=True)
    e.close()


print("ref sigma[0:3]", fx["sigma"][:3])
fit("csr default", layers)
fit("csr b16", layers, block=16)
fit("csr dense RR", layers, solver_flags=2)
fit("csr sym=no", layers, symmetric=0)
rng = np.random.default_rng(2)
pert = [sp.csr_matrix(a + 1e-3 * rng.standard_normal(a.shape).astype(np.float32)) for a in dense]
fit("csr rank-8 + 1e-3 noise", pert)
sparse = []
for a in dense:
    m = a.copy()
    m[rng.random(m.shape) < 0.9] = 0
    sparse.append(sp.csr_matrix(m))
fit("csr 10% of the entries (full rank)", sparse)
