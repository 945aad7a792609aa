"""C-ABI library: loads, exports every symbol include/*.h declares, host-side pieces.
CPU only (no compute calls need a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def _header_symbols():
    txt = "".join(open(os.path.join(REPO, "include", h)).read()
                  for h in ("n2v2r.h", "n2v2r_diag.h"))
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




def test_engine_pool_reuse_and_takeover(monkeypatch):
    """The per-device handle pool behind N2V2R (_lib.acquire_engine), with a stub handle whose
    constructor loads the library as Engine's does (the pool lock is re-entered): a handle whose
    owner is gone is reused, a new one is made while all are owned (up to POOL_MAX), and beyond
    that the least recently acquired one is taken over after its owner's _hand_over()."""
    import gc
    import threading
    from node2vec2rank_amd import _lib

    class Stub:
        def __init__(self, device):
            _lib.load()
            self.h = object()

    class Owner:
        handed = 0

        def _hand_over(self):
            Owner.handed += 1

    monkeypatch.setattr(_lib, "Engine", Stub)
    monkeypatch.setattr(_lib, "_pool", {})
    out = {}

    def work():
        owners = [Owner() for _ in range(_lib.POOL_MAX)]
        engs = [_lib.acquire_engine(7, o) for o in owners]
        out["distinct"] = len({id(e) for e in engs})
        extra = Owner()
        e5 = _lib.acquire_engine(7, extra)
        out["takeover"] = e5 is engs[0] and Owner.handed == 1
        out["owner"] = _lib.engine_owner(e5) is extra
        del owners[1]
        gc.collect()
        out["reuse"] = _lib.acquire_engine(7, Owner()) is engs[1]

    t = threading.Thread(target=work, daemon=True)
    t.start()
    t.join(30)
    assert not t.is_alive(), "acquire_engine deadlocked"
    assert out == dict(distinct=_lib.POOL_MAX, takeover=True, owner=True, reuse=True), out


def test_reference_descending_order_is_the_references():
    """The host half of the reference tie order (_lib.reference_descending_order, used only for
    the columns the GPU flags as tied) reproduces the reference's Borda on every fixture column
    set, ties included (model.py:173-174 + model_utils.py:22-34)."""
    import numpy as np
    from conftest import FIXTURES, load_fixture
    from node2vec2rank_amd import _lib
    for name in FIXTURES:
        fx = load_fixture(name)
        for strategy in [str(x) for x in fx["strategies"]]:
            for key in [str(k) for k in fx[f"{strategy}/keys"]]:
                D = fx[f"{strategy}/{key}/D"]
                n = D.shape[0]
                score = np.zeros(n, dtype=np.int64)
                for c in D.T:
                    pos = np.empty(n, dtype=np.int64)
                    pos[_lib.reference_descending_order(c)] = np.arange(n)
                    score += n - pos
                np.testing.assert_array_equal(score, fx[f"{strategy}/{key}/borda"])
