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


