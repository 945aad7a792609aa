"""SURVEY 8(c)(4), end to end: the drop-in API's integer ranks are BIT-EXACT with the reference's
on a tie-free fixture whose sorted distance columns have every adjacent gap >= 1e-4 (needs the
GPU).

tests/golden/lowrank_exact.npz was made by running the reference model.py itself
(make_golden.py lowrank_exact): a weighted directed two-layer network, N = 2000, rank 8, dims
{2, 4, 6, 8} x {cosine, euclidean} (8 columns), seed 42, sequential.  The layers go through
``N2V2R(...).fit_transform_rank()`` + ``aggregate_transform()`` as dense arrays (dense storage,
the MFMA path) and as scipy CSR (the CSR SpMM path, b = 8), and the Borda column must equal the
reference's ``borda_ranks`` element for element (reference model.py:98-201,
model_utils.py:22-36).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_fixture
from test_oracle_golden import lowrank_exact_layers

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("storage", ["dense", "csr"])
def test_lowrank_exact_borda_bit_exact(storage):
    from node2vec2rank_amd.model import N2V2R
    fx = load_fixture("lowrank_exact")
    layers = lowrank_exact_layers(fx)
    if storage == "csr":
        layers = [sp.csr_matrix(a) for a in layers]
    nodes = [str(x) for x in fx["nodes"]]
    dims = [int(x) for x in fx["dims"]]
    metrics = [str(x) for x in fx["metrics"]]
    cfg = dict(embed_dimensions=dims, distance_metrics=metrics, seed=int(fx["seed"]),
               comp_strategy="sequential", verbose=-1, save_dir=None)
    m = N2V2R(layers, nodes, cfg)
    ranks = m.fit_transform_rank()
    agg = m.aggregate_transform()
    st = m.eig_stats
    assert st["converged"] == 8, st
    np.testing.assert_allclose(m._engine.singular_values(), fx["sigma"], rtol=1e-5)
    assert list(ranks) == ["1"] and list(agg) == ["1"]
    assert list(ranks["1"].columns) == [str(c) for c in fx["sequential/1/cols"]]
    assert list(agg["1"].index) == nodes and list(ranks["1"].index) == nodes
    D = ranks["1"].to_numpy()
    Dref = fx["sequential/1/D"]
    derr = np.abs(D - Dref).max(axis=0)
    # every column's order is decided when each distance is within half the column's smallest
    # adjacent gap of the reference's (>= 1e-4 by the fixture's construction)
    half = fx["min_gap"] / 2
    for c in range(D.shape[1]):
        np.testing.assert_array_equal(np.argsort(-D[:, c], kind="stable"),
                                      np.argsort(-Dref[:, c], kind="stable"))
    b = agg["1"]["borda_ranks"].to_numpy()
    ref = fx["sequential/1/borda"]
    exact = bool(np.array_equal(b, ref))
    print(f"lowrank_exact [{storage}]: {st['restarts']} cycles, {st['block_applications']} "
          f"block applications, max residual {st['max_residual']:.2e}; distance error per "
          f"column {derr} (half the smallest gaps {half}); bit-exact {exact}")
    assert np.all(derr < half), (derr, half)
    assert b.dtype == np.int64
    assert exact
