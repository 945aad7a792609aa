"""CSR ingest on the GPU (n2v2r_set_layer_csr): range check, unweighted detection, the stable
radix transpose and the symmetry test, on the inputs a caller may hand over uncanonical
(unsorted rows, duplicate entries, empty rows, an empty layer).  A^T X through the stored
transpose is checked against scipy; a wrong symmetric verdict would fail it."""
import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu


def _shuffle_rows(A, rng):
    """Same matrix, each row's entries in a random order (scipy keeps them as given)."""
    A = sp.csr_matrix(A)
    ix = A.indices.copy()
    dv = A.data.copy()
    for r in range(A.shape[0]):
        p0, p1 = A.indptr[r], A.indptr[r + 1]
        perm = rng.permutation(p1 - p0) + p0
        ix[p0:p1] = A.indices[perm]
        dv[p0:p1] = A.data[perm]
    out = sp.csr_matrix((dv, ix, A.indptr.copy()), shape=A.shape)
    out.has_sorted_indices = False
    return out


def _check_products(engine, A, rng):
    n = A.shape[0]
    X = rng.standard_normal((n, 8)).astype(np.float32)
    for tr in (False, True):
        Y, _, _ = engine.bench_spmm(0, X, transpose=tr, reps=1)
        M = (A.T if tr else A).astype(np.float64)
        ref = M @ X.astype(np.float64)
        scale = np.abs(M) @ np.abs(X).astype(np.float64)
        assert np.all(np.abs(Y - ref) <= 1e-5 * scale + 1e-6), tr


@pytest.mark.parametrize("symmetric", [True, False])
@pytest.mark.parametrize("weighted", [True, False])
def test_unsorted_rows(engine, symmetric, weighted):
    rng = np.random.default_rng(3)
    n = 5000
    A = sp.random(n, n, density=12.0 / n, format="csr", dtype=np.float32, random_state=rng)
    A.data = (rng.integers(1, 4, A.nnz).astype(np.float32) if weighted
              else np.ones(A.nnz, np.float32))
    if symmetric:
        A = (A + A.T).tocsr()
        if not weighted:
            A.data[:] = 1.0
    U = _shuffle_rows(A, rng)
    engine.set_layers([U])
    _check_products(engine, A, rng)
    # the symmetry verdict: a symmetric layer keeps no transpose, a directed one does; both
    # give the same products, so compare the stored transpose with scipy explicitly
    engine.set_layers([U], symmetric=0)
    _check_products(engine, A, rng)


def test_duplicates_and_empty_rows(engine):
    rng = np.random.default_rng(8)
    n = 3001
    rows = rng.integers(0, n // 2, 20_000)          # the upper half of the rows stays empty
    cols = rng.integers(0, n, 20_000)
    vals = rng.standard_normal(20_000).astype(np.float32)
    # uncanonical CSR: 500 entries repeated as separate entries of their rows
    rows = np.concatenate([rows, rows[:500]])
    cols = np.concatenate([cols, cols[:500]])
    vals = np.concatenate([vals, vals[:500]])
    order = np.argsort(rows, kind="stable")
    indptr = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.int64)
    raw = sp.csr_matrix((vals[order], cols[order].astype(np.int32), indptr), shape=(n, n))
    engine.set_layers([raw])
    ref = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))  # scipy sums the duplicates
    _check_products(engine, ref, rng)


def test_empty_layer(engine):
    n = 1000
    E = sp.csr_matrix((n, n), dtype=np.float32)
    engine.set_layers([E, E])
    X = np.ones((n, 8), np.float32)
    for tr in (False, True):
        Y, _, _ = engine.bench_spmm(0, X, transpose=tr, reps=1)
        assert np.all(Y == 0)
    np.testing.assert_array_equal(engine.column_sums(1), np.zeros(n, np.float32))
