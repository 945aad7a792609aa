"""SpMM b = 8 on graphs of the same size (N = 100k, ~2M entries) with different panel locality:
how much of the row kernel's time is the gather's cache behaviour.

    python tools/spmm_locality.py"""
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, ".")
from node2vec2rank_amd import _lib, synthetic  # noqa: E402


def sym_from(rows, cols, n):
    keep = rows != cols
    rows, cols = rows[keep], cols[keep]
    a = sp.csr_matrix((np.ones(2 * len(rows), np.float32),
                       (np.concatenate([rows, cols]), np.concatenate([cols, rows]))), shape=(n, n))
    a.sum_duplicates()
    a.data[:] = 1.0
    a.sort_indices()
    return a


n, deg = 100_000, 20
rng = np.random.default_rng(0)
m = n * deg // 2
graphs = {"er": synthetic.er_layer(n, deg, 1000)}
for w in (256, 4096, 32768):
    r = rng.integers(0, n, m)
    c = (r + rng.integers(1, w, m)) % n
    graphs[f"band{w}"] = sym_from(r, c, n)
for span in (10_000, 50_000):  # random columns drawn from a window of `span` rows only
    r = rng.integers(0, n, 2 * m)
    c = rng.integers(0, span, 2 * m)
    a = sp.csr_matrix((np.ones(2 * m, np.float32), (r, c)), shape=(n, n))
    a.sum_duplicates()
    a.data[:] = 1.0
    a.sort_indices()
    graphs[f"cols{span}"] = a  # directed (timed as A x only)
eng = _lib.Engine(0)
X = rng.standard_normal((n, 8)).astype(np.float32)
for name, A in graphs.items():
    eng.set_layers([A, A], symmetric=1)
    _, ms, by = eng.bench_spmm(0, X, reps=50, want_y=False)
    print(f"{name:10s} nnz {A.nnz:9d} avg_us {ms * 1e3:7.2f}  algo GB/s {by / ms / 1e6:7.1f}  "
          f"gathered GB/s {A.nnz * 32 / ms / 1e6:7.1f}", flush=True)
