"""The solver's paired-panel mode (N2V2R_EIG_PANEL16; solver.cpp "pair", pair.hip): the basis in
8-wide blocks, every application of M = sum_k A_k A_k^T multiplying the last two as one N x 16
panel with the tiled SpMM at 64-B panel rows, the projected matrix (half-bandwidth 16) assembled
from the local passes' saved Gram rows and solved by the dense Rayleigh-Ritz.  Off by default
(measured slower at BASELINE cfg4 / cfg5: block width 16 needs 1.28x / 1.49x the vectors of
width 8, profiles/r06_pair_fits.jsonl); checked here for correctness (reference model.py:51-55
via svds semantics): host fp64 residuals, orthonormality, singular values against the 8-wide
fit, the reference's own bit-exact fixture end to end."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_fixture

pytestmark = pytest.mark.gpu


def test_pair_mode_er_residuals(monkeypatch):
    from node2vec2rank_amd import _lib, synthetic
    monkeypatch.setenv("N2V2R_SPMM_CB", "1")  # (the mode rides on the tiled SpMM)
    layers = synthetic.er_layers(100_000, 20, 2, seed_base=1000)
    d = 64
    eng = _lib.Engine(0)
    try:
        eng.set_layers(layers)
        st8 = eng.uase(d, seed=42, solver_flags=_lib.EIG_PANEL8)
        s8 = eng.singular_values()
        st = eng.uase(d, seed=42, solver_flags=_lib.EIG_PANEL16)
        s = eng.singular_values()
        U = eng.left_embedding() / np.sqrt(s)[None, :].astype(np.float32)
    finally:
        eng.close()
    print(f"pair mode: {st['block_applications']} blocks in {st['restarts']} cycles "
          f"(8-wide: {st8['block_applications']} in {st8['restarts']}), max residual "
          f"{st['max_residual']:.2e}")
    assert st8["panel"] == 8 and st["panel"] == 16
    assert st["converged"] == d, st
    np.testing.assert_allclose(s, s8, rtol=1e-5)
    cols = [0, 1, d // 2, d - 2, d - 1]
    X = U[:, cols].astype(np.float64)
    MX = np.zeros_like(X)
    for A in layers:
        A64 = A.astype(np.float64).tocsr()
        MX += A64 @ (A64.T @ X)
    th = s.astype(np.float64) ** 2
    res = np.linalg.norm(MX - X * th[cols][None, :], axis=0) / th[0]
    assert np.all(res <= 5e-6), res
    assert np.abs(U.T.astype(np.float64) @ U - np.eye(d)).max() <= 1e-5


def test_pair_mode_lowrank_exact_bit_exact(monkeypatch):
    """The reference's tie-free fixture through the drop-in API in paired mode: integer ranks
    bit-exact with the reference's (tests/test_gpu_exact.py's bar)."""
    from test_oracle_golden import lowrank_exact_layers

    from node2vec2rank_amd import _lib
    from node2vec2rank_amd.model import N2V2R
    monkeypatch.setenv("N2V2R_SPMM_CB", "1")
    fx = load_fixture("lowrank_exact")
    layers = [sp.csr_matrix(a) for a in lowrank_exact_layers(fx)]
    nodes = [str(x) for x in fx["nodes"]]
    cfg = dict(embed_dimensions=[int(x) for x in fx["dims"]],
               distance_metrics=[str(x) for x in fx["metrics"]], seed=int(fx["seed"]),
               comp_strategy="sequential", verbose=-1, save_dir=None)
    m = N2V2R(layers, nodes, cfg, eig_options={"solver_flags": _lib.EIG_PANEL16})
    ranks = m.fit_transform_rank()
    agg = m.aggregate_transform()
    assert m.eig_stats["panel"] == 16, m.eig_stats
    assert m.eig_stats["converged"] == 8, m.eig_stats
    derr = np.abs(ranks["1"].to_numpy() - fx["sequential/1/D"]).max(axis=0)
    assert np.all(derr < fx["min_gap"] / 2), derr
    assert np.array_equal(agg["1"]["borda_ranks"].to_numpy(), fx["sequential/1/borda"])


@pytest.mark.parametrize("name", ["er_cfg2", "er_cfg4g"])
def test_pair_mode_reference_fixtures(monkeypatch, name):
    """BASELINE cfg2 and the bench's cfg4 grid (d = 128, 10 columns) against the reference's own
    outputs in paired mode, at the bar the 8-wide fit meets (test_gpu_configs.py): sigma rtol
    2e-5, per-column distance error within max(1e-4, the reference's seed envelope), Kendall
    tau >= 0.998 and the identical top-100 set."""
    from scipy.stats import kendalltau

    from node2vec2rank_amd import _lib, synthetic
    from node2vec2rank_amd.model import N2V2R
    monkeypatch.setenv("N2V2R_SPMM_CB", "1")
    fx = load_fixture(name)
    n = int(fx["n"])
    layers = synthetic.er_layers(n, float(fx["avg_deg"]), int(fx["num_layers"]),
                                 seed_base=int(fx["seed_base"]))
    np.testing.assert_array_equal(synthetic.fingerprint(layers), fx["checksum"])
    cfg = dict(embed_dimensions=[int(x) for x in fx["dims"]],
               distance_metrics=[str(x) for x in fx["metrics"]], seed=int(fx["seed"]),
               comp_strategy="sequential", verbose=-1, save_dir=None)
    m = N2V2R(layers, list(range(n)), cfg, eig_options={"solver_flags": _lib.EIG_PANEL16})
    ranks = m.fit_transform_rank()
    agg = m.aggregate_transform()
    st = m.eig_stats
    d = max(int(x) for x in fx["dims"])
    assert st["panel"] == 16, st
    assert st["converged"] == d or (st["stagnated"] and st["max_residual"] <= st["stag_cap"]), st
    np.testing.assert_allclose(m._engine.singular_values(), fx["sigma"], rtol=2e-5)
    derr = np.abs(ranks["1"].to_numpy() - fx["sequential/1/D"]).max(axis=0)
    env = fx["env_distance_per_col"]
    b = agg["1"]["borda_ranks"].to_numpy()
    ref = fx["sequential/1/borda"]
    tau = kendalltau(b, ref).statistic
    top = len(set(np.argsort(-b, kind="stable")[:100]) & set(np.argsort(-ref, kind="stable")[:100]))
    print(f"{name} paired: {st['block_applications']} blocks, distance err {derr.max():.2e}, "
          f"tau {tau:.6f}, top-100 {top}")
    assert np.all(derr <= np.maximum(1e-4, env)), (derr, env)
    assert tau >= 0.998, tau
    assert top == 100, top
