"""Dense layers (BASELINE cfg3 path): MFMA GEMM Gram application, dense ingest, UASE on dense
storage vs the CSR path and the reference's golden vectors, row-partitioned dense."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import FIXTURES, fixture_layers, load_fixture
from oracle import n2v2r_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("form", ["tn", "lds"])
@pytest.mark.parametrize("b", [8, 16, 32, 64])
@pytest.mark.parametrize("n", [1000, 1037, 2501])
def test_dense_gemm_matches_numpy(engine, n, b, form, monkeypatch):
    """Both dense GEMM kernels (b <= 32: the B-operand streaming dense_tn_kernel by default,
    N2V2R_DENSE_TN=0 the LDS-staged dense_gemm_kernel; b = 64 always the latter) against an
    fp64 product, for A and A^T of a directed layer."""
    monkeypatch.setenv("N2V2R_DENSE_TN", "1" if form == "tn" else "0")
    rng = np.random.default_rng(n + b)
    A = rng.standard_normal((n, n)).astype(np.float32)
    engine.set_layers([A, A.T.copy()], storage="dense", symmetric=-1)
    X = rng.standard_normal((n, b)).astype(np.float32)
    for k, M in enumerate([A, A.T]):
        for tr in (False, True):
            Y, ms, by = engine.bench_spmm(k, X, transpose=tr, reps=2)
            ref = (M.T if tr else M).astype(np.float64) @ X.astype(np.float64)
            scale = np.abs(M.T if tr else M).astype(np.float64) @ np.abs(X).astype(np.float64)
            assert np.all(np.abs(Y - ref) <= 2e-6 * scale + 1e-6), (k, tr)
            assert ms > 0 and by == pytest.approx(4.0 * n * n + 4.0 * 2 * n * b)


def test_dense_symmetry_detection(engine):
    rng = np.random.default_rng(5)
    S = rng.random((300, 300)).astype(np.float32)
    S = S + S.T
    engine.set_layers([S, S], storage="dense", symmetric=-1)
    X = rng.standard_normal((300, 8)).astype(np.float32)
    Y0, _, _ = engine.bench_spmm(0, X, transpose=False, reps=1)
    Y1, _, _ = engine.bench_spmm(0, X, transpose=True, reps=1)
    np.testing.assert_array_equal(Y0, Y1)  # symmetric: A^T is A itself


@pytest.mark.parametrize("name", [f for f in FIXTURES if f != "directed_weighted"] + ["directed_weighted"])
def test_uase_dense_storage_matches_reference(engine, name):
    """The reference's own fixtures fed as dense arrays: same bar as the CSR path."""
    fx = load_fixture(name)
    layers = [np.asarray(a.todense(), dtype=np.float32) for a in fixture_layers(fx)]
    d = int(fx["dims"].max())
    engine.set_layers(layers, storage="dense")
    engine.uase(d, seed=int(fx["seed"]))
    np.testing.assert_allclose(engine.singular_values(), fx["sigma"], rtol=2e-5)
    Ya, _, _ = orc.uase(fixture_layers(fx), d, seed=int(fx["seed"]) + 1)
    env = np.abs(orc.align_signs(Ya, fx["Y"]) - fx["Y"]).max() / np.abs(fx["Y"]).max()
    Y = orc.align_signs(engine.embedding().astype(np.float64), fx["Y"])
    err = np.abs(Y - fx["Y"]).max() / np.abs(fx["Y"]).max()
    assert err <= max(5e-4, 3 * env), (name, err, env)


def test_uase_dense_corr_residuals(engine):
    """cfg3-shaped (abs corrcoef, K=4) at N=3000, d=64: true Ritz residuals in fp64 and sigma
    vs the oracle's ARPACK."""
    from node2vec2rank_amd import synthetic
    layers = synthetic.corr_layers(3000, 4, samples=200, seed_base=0)
    d = 64
    engine.set_layers(layers)
    assert engine.storage == "dense"
    st = engine.uase(d, seed=42)
    assert st["converged"] == d or (st["stagnated"] == 1 and st["max_residual"] <= st["stag_cap"]), st
    s = engine.singular_values()
    X = engine.left_embedding().astype(np.float64) / np.sqrt(s)[None, :]
    A = np.hstack([a.astype(np.float64) for a in layers])
    R = A @ (A.T @ X) - X * (s ** 2)[None, :]
    res = np.linalg.norm(R, axis=0) / s[0] ** 2
    assert res.max() < 1e-5, res.max()
    _, s_ref, _ = orc.uase([sp.csr_matrix(a) for a in layers], d, seed=42)
    np.testing.assert_allclose(s, s_ref, rtol=1e-5)
    # ranking through the dense path
    ncmp, ncols = engine.rank("sequential", [16, 64], ["cosine", "euclidean"])
    assert (ncmp, ncols) == (3, 4)
    for c in range(ncmp):
        b = engine.borda(c)
        assert b.min() >= ncols and b.max() <= ncols * 3000
    cs = engine.column_sums(1)
    np.testing.assert_allclose(cs, layers[1].sum(axis=0), rtol=1e-5)


def test_dense_partitioned_matches_single(engine):
    from test_gpu_dist import _run_ranks
    from node2vec2rank_amd import synthetic
    layers = synthetic.corr_layers(1500, 3, samples=100, seed_base=7)
    d = 24

    def fn(eng, r):
        eng.set_layers(layers)
        eng.uase(d, seed=3)
        eng.rank("sequential", [d], ["cosine", "euclidean"])
        return dict(Y=eng.embedding(), s=eng.singular_values(), D=eng.distances(0))

    res = _run_ranks(2, fn)
    engine.set_layers(layers)
    engine.uase(d, seed=3)
    engine.rank("sequential", [d], ["cosine", "euclidean"])
    np.testing.assert_allclose(res[0]["s"], engine.singular_values(), rtol=1e-5)
    Y = np.concatenate([r["Y"] for r in res], axis=1).astype(np.float64)
    Y1 = engine.embedding().astype(np.float64)
    Y = orc.align_signs(Y, Y1)
    assert np.abs(Y - Y1).max() <= 1e-3 * np.abs(Y1).max()
    np.testing.assert_allclose(res[0]["D"], engine.distances(0), atol=1e-4)
