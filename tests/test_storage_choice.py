"""Storage choice of Engine.set_layers for dense arrays (_lib._denser_than_quarter): dense in
HBM when more than a quarter of the entries are non-zero.  CPU only (no engine call)."""
import numpy as np

from node2vec2rank_amd._lib import _denser_than_quarter


def test_far_from_threshold_decided_by_sample():
    rng = np.random.default_rng(0)
    dense = rng.random((4000, 4000)).astype(np.float32)
    assert _denser_than_quarter(dense)
    sparse = np.zeros((4000, 4000), np.float32)
    sparse[::9] = 1.0
    assert not _denser_than_quarter(sparse)


def test_near_threshold_is_exact():
    a = np.zeros((3000, 3000), np.float32)
    a[:, :750] = 1.0                      # exactly a quarter: not more than a quarter
    assert not _denser_than_quarter(a)
    a[5, 750] = 1.0                       # one entry over
    assert _denser_than_quarter(a)


def test_edge_shapes():
    assert not _denser_than_quarter(np.zeros((0, 0), np.float32))
    assert _denser_than_quarter(np.ones((7, 7), np.float32))
    assert not _denser_than_quarter(np.eye(50, dtype=np.float32))
