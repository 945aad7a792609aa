"""C-ABI library: loads, exports every symbol include/n2v2r.h declares, host-side pieces.
CPU only (no compute calls need a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "n2v2r.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(n2v2r_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from node2vec2rank_amd import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.EXPORTED) == syms
    assert lib.n2v2r_version().startswith(b"n2v2r-mi355x")


def test_library_is_gfx950_code_object():
    from node2vec2rank_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_fails_loudly():
    """Without a HIP device the engine must raise, never fall back to the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from node2vec2rank_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.Engine(0)


def test_null_handle_is_rejected():
    from node2vec2rank_amd import _lib
    lib = _lib.load()
    assert lib.n2v2r_uase(None, 8, None, None) == _lib.ERR_BAD_ARG
    assert lib.n2v2r_synchronize(None) == _lib.ERR_BAD_ARG


@pytest.mark.parametrize("c,p", [(3, 3), (40, 12), (200, 64)])
def test_host_rayleigh_ritz_eigensolver(c, p):
    """The host Rayleigh-Ritz solver (tridiagonalisation + QL + inverse iteration) vs LAPACK,
    including a cluster of near-equal eigenvalues."""
    from node2vec2rank_amd import _lib
    f = _lib.load().n2v2r_host_sym_eig_top
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, np.ctypeslib.ndpointer(np.float64), ctypes.c_int,
                  np.ctypeslib.ndpointer(np.float64), np.ctypeslib.ndpointer(np.float64)]
    rng = np.random.default_rng(c)
    Q, _ = np.linalg.qr(rng.standard_normal((c, c)))
    ev = np.sort(rng.standard_normal(c)) * 10
    k = min(4, c)
    ev[-k:] = ev[-1] + np.arange(k) * 1e-9
    a = (Q * ev) @ Q.T
    a = 0.5 * (a + a.T)
    A = a.copy()
    w = np.zeros(p)
    Z = np.zeros((c, p))
    assert f(c, A, p, w, Z) == 0
    wr = np.linalg.eigvalsh(a)[::-1][:p]
    np.testing.assert_allclose(w, wr, atol=1e-11)
    assert np.abs(a @ Z - Z * w).max() < 1e-10
    assert np.abs(Z.T @ Z - np.eye(p)).max() < 1e-10
