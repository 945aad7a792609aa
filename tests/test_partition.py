"""Host side of the row partition (CPU): the counter-based ER generator's per-rank row blocks
are exactly the rows of the full layer, for even and ragged splits."""
import numpy as np
import pytest
import scipy.sparse as sp

from node2vec2rank_amd import synthetic


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_er_rows_union_is_the_layer(world):
    n = 3001
    full = synthetic.er_layer_rows(n, 8.0, 11)
    assert (full != full.T).nnz == 0
    assert full.diagonal().sum() == 0
    assert set(np.unique(full.data)) == {1.0}
    R = -(-n // world)
    parts = []
    for g in range(world):
        r0 = min(n, g * R)
        nl = max(0, min(n, r0 + R) - r0)
        blk = synthetic.er_layer_rows(n, 8.0, 11, r0, nl, chunk=1000)
        assert blk.shape == (nl, n)
        parts.append(blk)
    assert (sp.vstack(parts).tocsr() != full).nnz == 0


def test_er_rows_mean_degree():
    a = synthetic.er_layer_rows(20000, 12.0, 3)
    assert abs(a.nnz / 20000 - 12.0) < 0.1
