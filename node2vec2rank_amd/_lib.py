"""ctypes binding of libn2v2r_hip.so (the C-ABI in include/n2v2r.h).

There is no CPU fallback: if the library is missing, or no GPU is visible, every entry point
raises.  Status codes map onto the exception types the reference raises for the same
conditions (model_utils.py:64-65, model.py:182-183, model.py:199).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("N2V2R_LIB", os.path.join(_HERE, "lib", "libn2v2r_hip.so"))

OK = 0
ERR_BAD_ARG = 1
ERR_UNSUPPORTED_METRIC = 2
ERR_NO_CONVERGENCE = 3
ERR_HIP = 4
ERR_OUT_OF_MEMORY = 5
ERR_NOT_READY = 6
ERR_UNSUPPORTED_AGG = 7
ERR_INTERNAL = 8
ERR_RCCL = 9
AGG_BORDA, AGG_NONE = 0, -1
EIG_TIME_SPMM = 16
EIG_TEST_NO_STAGNATION = 64
EIG_TEST_FAIL_ALONE = 128
EIG_PANEL16 = 256
EIG_PANEL8 = 512

STRATEGY = {"sequential": 0, "one_vs_before": 1, "one_vs_rest": 2}
METRIC = {"cosine": 0, "euclidean": 1, "correlation": 2}
SYM_DETECT, SYM_NO, SYM_YES = -1, 0, 1

# every symbol include/n2v2r.h and include/n2v2r_diag.h declare (checked by tests/test_capi.py)
EXPORTED = [
    "n2v2r_create", "n2v2r_destroy", "n2v2r_last_error", "n2v2r_version",
    "n2v2r_set_num_layers", "n2v2r_set_layer_csr", "n2v2r_uase", "n2v2r_get_embedding",
    "n2v2r_get_left_embedding", "n2v2r_get_singular_values", "n2v2r_set_embedding",
    "n2v2r_rank", "n2v2r_get_distances", "n2v2r_get_borda", "n2v2r_rank_timing",
    "n2v2r_pairwise_distances", "n2v2r_borda_columns", "n2v2r_borda_columns_ex",
    "n2v2r_column_sums",
    "n2v2r_synchronize", "n2v2r_bench_spmm", "n2v2r_bench_spmm_tiled", "n2v2r_spmm_col_blocks",
    "n2v2r_comm_unique_id", "n2v2r_create_rccl", "n2v2r_simgroup_create",
    "n2v2r_simgroup_destroy", "n2v2r_create_sim", "n2v2r_dist_info", "n2v2r_set_layer_csr_rows",
    "n2v2r_rr_top", "n2v2r_rr_band_top", "n2v2r_set_layer_dense", "n2v2r_project",
    "n2v2r_create_multi", "n2v2r_multi_devices", "n2v2r_h2d_layer_bytes",
]
UNIQUE_ID_BYTES = 128


class ArpackNoConvergence(RuntimeError):
    """UASE eigensolver did not reach the residual tolerance (scipy raises
    ``ArpackNoConvergence`` in the reference's svds path)."""


class EigOpts(ctypes.Structure):
    _fields_ = [("block", ctypes.c_int), ("max_basis", ctypes.c_int), ("keep", ctypes.c_int),
                ("max_restarts", ctypes.c_int), ("tol", ctypes.c_double),
                ("seed", ctypes.c_uint64), ("solver_flags", ctypes.c_int)]


class EigStats(ctypes.Structure):
    _fields_ = [("restarts", ctypes.c_int), ("block_applications", ctypes.c_int),
                ("converged", ctypes.c_int), ("basis", ctypes.c_int),
                ("max_residual", ctypes.c_double), ("ms_total", ctypes.c_double),
                ("ms_spmm", ctypes.c_double), ("ms_ortho", ctypes.c_double),
                ("ms_rr_host", ctypes.c_double), ("spmm_launches", ctypes.c_int64),
                ("spmm_algo_bytes", ctypes.c_double), ("stagnated", ctypes.c_int),
                ("rr_fallbacks", ctypes.c_int), ("gpu_ms_spmm", ctypes.c_double * 2),
                ("spmm_timed_launches", ctypes.c_int64 * 2),
                ("spmm_stage_bytes", ctypes.c_double * 2), ("est_scale", ctypes.c_double),
                ("lean_checks", ctypes.c_int), ("pool_blocks", ctypes.c_int),
                ("spmm_form", ctypes.c_int), ("stag_cap", ctypes.c_double),
                ("y_captured", ctypes.c_int), ("tri_fallbacks", ctypes.c_int),
                ("panel", ctypes.c_int)]

    def as_dict(self):
        out = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            out[k] = list(v) if isinstance(v, ctypes.Array) else v
        return out


_lib = None
_lock = threading.RLock()  # re-entered: acquire_engine -> Engine() -> load()

_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64


def _p(dtype):
    return np.ctypeslib.ndpointer(dtype=dtype, flags="C_CONTIGUOUS")


def load(path: str | None = None):
    """Load (once) and return the ctypes library.  Raises if the .so is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"n2v2r HIP library not found at {p}; build it with "
                "`python -m node2vec2rank_amd.build` (there is no CPU fallback)")
        lib = ctypes.CDLL(p)
        # (registered after the library's own load-time registrations -- HIP's fat-binary
        # module constructor -- and after torch's, so it runs before their teardown)
        atexit.register(_teardown)
        sig = {
            "n2v2r_create": (_i, [_i, ctypes.POINTER(_vp)]),
            "n2v2r_destroy": (None, [_vp]),
            "n2v2r_last_error": (_i, [_vp, ctypes.c_char_p, ctypes.c_size_t]),
            "n2v2r_version": (ctypes.c_char_p, []),
            "n2v2r_set_num_layers": (_i, [_vp, _i, _i64]),
            "n2v2r_set_layer_csr": (_i, [_vp, _i, _i64, _i64, _p(np.int64), _p(np.int32),
                                         _p(np.float32), _i]),
            "n2v2r_uase": (_i, [_vp, _i, ctypes.POINTER(EigOpts), ctypes.POINTER(EigStats)]),
            "n2v2r_get_embedding": (_i, [_vp, _p(np.float32)]),
            "n2v2r_get_left_embedding": (_i, [_vp, _p(np.float32)]),
            "n2v2r_get_singular_values": (_i, [_vp, _p(np.float64)]),
            "n2v2r_set_embedding": (_i, [_vp, _i, _i64, _i, _p(np.float32)]),
            "n2v2r_rank": (_i, [_vp, _i, _p(np.int32), _i, _p(np.int32), _i, _i,
                                ctypes.POINTER(_i), ctypes.POINTER(_i)]),
            "n2v2r_get_distances": (_i, [_vp, _i, _p(np.float64)]),
            "n2v2r_get_borda": (_i, [_vp, _i, _p(np.int64)]),
            "n2v2r_rank_timing": (_i, [_vp, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double)]),
            "n2v2r_pairwise_distances": (_i, [_vp, _p(np.float64), _p(np.float64), _i64, _i, _i,
                                              _p(np.float64)]),
            "n2v2r_borda_columns": (_i, [_vp, _p(np.float64), _i64, _i, _p(np.int64)]),
            "n2v2r_borda_columns_ex": (_i, [_vp, _p(np.float64), _i64, _i, _vp, _i, _vp,
                                            _p(np.int64), _p(np.int32)]),
            "n2v2r_column_sums": (_i, [_vp, _i, _p(np.float32)]),
            "n2v2r_synchronize": (_i, [_vp]),
            "n2v2r_bench_spmm": (_i, [_vp, _i, _i, _i, _i, _p(np.float32), _vp,
                                      ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double)]),
            "n2v2r_bench_spmm_tiled": (_i, [_vp, _i, _i, _i, _i, _i, _p(np.float32), _vp,
                                            ctypes.POINTER(ctypes.c_double)]),
            "n2v2r_spmm_col_blocks": (_i, [_vp, _i]),
            "n2v2r_rr_top": (_i, [_vp, _i, _p(np.float64), _i, _p(np.float64), _p(np.float32)]),
            "n2v2r_rr_band_top": (_i, [_vp, _i, _i, _p(np.float64), ctypes.c_int64, _vp, _i,
                                       _p(np.float64), _p(np.float32)]),
            "n2v2r_set_layer_dense": (_i, [_vp, _i, _i64, _p(np.float32), _i]),
            "n2v2r_project": (_i, [_vp, _i64, _i64, _p(np.float64), _i, _p(np.float64)]),
            "n2v2r_comm_unique_id": (_i, [ctypes.c_char_p, ctypes.c_size_t]),
            "n2v2r_create_rccl": (_i, [_i, _i, _i, ctypes.c_char_p, ctypes.POINTER(_vp)]),
            "n2v2r_simgroup_create": (_i, [_i, ctypes.POINTER(_vp)]),
            "n2v2r_simgroup_destroy": (None, [_vp]),
            "n2v2r_create_sim": (_i, [_i, _vp, _i, ctypes.POINTER(_vp)]),
            "n2v2r_dist_info": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i),
                                     ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
            "n2v2r_set_layer_csr_rows": (_i, [_vp, _i, _i64, _i64, _i64, _i64, _p(np.int64),
                                              _p(np.int32), _p(np.float32)]),
            "n2v2r_create_multi": (_i, [_p(np.int32), _i, ctypes.POINTER(_vp)]),
            "n2v2r_multi_devices": (_i, [_vp, _vp, _i]),
            "n2v2r_h2d_layer_bytes": (_i, [_vp, _vp, _i]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
        return lib


def comm_unique_id() -> bytes:
    """RCCL unique id (rank 0 creates it and broadcasts the bytes over its control plane)."""
    lib = load()
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    st = lib.n2v2r_comm_unique_id(buf, UNIQUE_ID_BYTES)
    if st != OK:
        raise RuntimeError(f"n2v2r_comm_unique_id failed with status {st}")
    return buf.raw


class SimGroup:
    """W ranks as threads of one process on one GPU (the row-partitioned algorithm without W
    devices).  Create one, then one thread per rank builds ``Engine.sim(device, group, r)``."""

    def __init__(self, world: int):
        self.lib = load()
        g = _vp()
        st = self.lib.n2v2r_simgroup_create(int(world), ctypes.byref(g))
        if st != OK:
            raise RuntimeError(f"n2v2r_simgroup_create failed with status {st}")
        self.g = g
        self.world = int(world)

    def close(self):
        if getattr(self, "g", None):
            self.lib.n2v2r_simgroup_destroy(self.g)
            self.g = None


_live = weakref.WeakSet()  # every open Engine (closed by _teardown at interpreter exit)


def _teardown():
    """At interpreter exit, while the HIP runtime (and a profiler tool, under rocprofv3) is
    still up: destroy every open handle -- its device allocations, streams, events and RCCL
    communicators -- before the C exit handlers unregister the library's kernels and tear the
    runtime down, so no library object outlives the runtime.  N2V2R_EXIT_MAPS=path also writes
    /proc/self/maps there (to map the PCs of a crash trace printed later in exit to libraries)."""
    for eng in list(_live):
        try:
            eng.close()
        except Exception:
            pass
    path = os.environ.get("N2V2R_EXIT_MAPS")
    if path:
        try:
            with open("/proc/self/maps") as src, open(path, "w") as dst:
                dst.write(src.read())
        except OSError:
            pass


class Engine:
    """One GPU, one handle.  Thin, typed wrapper over the C-ABI.

    Distributed handles (``Engine.rccl`` / ``Engine.sim``) own rows [row0, row0 + n_local) of
    the node set: ``embedding()`` / ``left_embedding()`` return those rows; distances, Borda,
    singular values and column sums are global on every rank."""

    def __init__(self, device: int = 0, _handle=None):
        self.lib = load()
        if _handle is None:
            h = _vp()
            st = self.lib.n2v2r_create(int(device), ctypes.byref(h))
            if st != OK:
                raise RuntimeError(
                    f"n2v2r_create(device={device}) failed with status {st}: no usable HIP GPU "
                    "(the engine has no CPU fallback)")
        else:
            h = _handle
        self.h = h
        self.device = device
        _live.add(self)

    @classmethod
    def rccl(cls, device: int, rank: int, world: int, unique_id: bytes) -> "Engine":
        lib = load()
        h = _vp()
        st = lib.n2v2r_create_rccl(int(device), int(rank), int(world), bytes(unique_id),
                                   ctypes.byref(h))
        if st != OK:
            raise RuntimeError(f"n2v2r_create_rccl(rank={rank}, world={world}) failed: {st}")
        return cls(device, _handle=h)

    @classmethod
    def multi(cls, devices) -> "Engine":
        """One process, len(devices) GPUs (n2v2r_create_multi): the row-partitioned fit with one
        host thread per GPU inside the library, RCCL over distinct devices (a repeated device:
        the in-process thread group, W ranks sharing it).  Used exactly like a one-GPU engine;
        embeddings, distances and Borda come back global."""
        lib = load()
        devs = np.ascontiguousarray([int(d) for d in devices], dtype=np.int32)
        h = _vp()
        st = lib.n2v2r_create_multi(devs, int(devs.size), ctypes.byref(h))
        if st != OK:
            raise RuntimeError(f"n2v2r_create_multi(devices={devs.tolist()}) failed with status "
                               f"{st}" + (" (RCCL)" if st == ERR_RCCL else ""))
        eng = cls(int(devs[0]), _handle=h)
        eng.devices = tuple(int(d) for d in devs)
        return eng

    @classmethod
    def sim(cls, device: int, group: SimGroup, rank: int) -> "Engine":
        lib = load()
        h = _vp()
        st = lib.n2v2r_create_sim(int(device), group.g, int(rank), ctypes.byref(h))
        if st != OK:
            raise RuntimeError(f"n2v2r_create_sim(rank={rank}) failed with status {st}")
        return cls(device, _handle=h)

    def h2d_layer_bytes(self):
        """Layer bytes each rank of this handle copied host -> device (a list, one per rank)."""
        out = np.zeros(64, dtype=np.int64)
        w = self.lib.n2v2r_h2d_layer_bytes(self.h, out.ctypes.data_as(ctypes.c_void_p), 64)
        if w < 0:
            self._check(w, "h2d_layer_bytes")
        return [int(x) for x in out[:w]]

    def dist_info(self):
        """(rank, world, row0, n_local) of this handle's row block."""
        r, w, r0, nl = _i(), _i(), _i64(), _i64()
        self._check(self.lib.n2v2r_dist_info(self.h, ctypes.byref(r), ctypes.byref(w),
                                             ctypes.byref(r0), ctypes.byref(nl)), "dist_info")
        return r.value, w.value, r0.value, nl.value

    def close(self):
        if getattr(self, "h", None):
            self.lib.n2v2r_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- errors --------------------------------------------------------------------------
    def _err(self) -> str:
        buf = ctypes.create_string_buffer(1024)
        self.lib.n2v2r_last_error(self.h, buf, len(buf))
        return buf.value.decode(errors="replace")

    def _check(self, st: int, what: str):
        if st == OK:
            return
        msg = f"{what}: {self._err()}"
        if st == ERR_UNSUPPORTED_METRIC:
            raise NotImplementedError("Unsupported metric")
        if st == ERR_UNSUPPORTED_AGG:
            raise NotImplementedError("Aggregation method not found. Available methods: Borda")
        if st == ERR_NOT_READY:
            raise ValueError("No n2v2r embeddings found")
        if st == ERR_NO_CONVERGENCE:
            raise ArpackNoConvergence(msg)
        if st == ERR_OUT_OF_MEMORY:
            raise MemoryError(msg)
        if st == ERR_BAD_ARG:
            raise ValueError(msg)
        if st == ERR_RCCL:
            raise RuntimeError(f"RCCL failure: {msg}")
        raise RuntimeError(msg)

    # -- layers ----------------------------------------------------------------------------
    def set_layers(self, layers, symmetric=SYM_DETECT, storage="auto"):
        """layers: list of scipy.sparse matrices (any format) or dense arrays, N x N.

        storage: "csr", "dense" (fp32 N x N in HBM, MFMA GEMMs) or "auto" (dense when every
        layer is a dense array with more than 1/4 of its entries non-zero)."""
        import scipy.sparse as sp
        if storage == "auto":
            storage = "csr"
            if all(not sp.issparse(a) for a in layers):
                arrs = [np.asarray(a) for a in layers]
                if all(_denser_than_quarter(a) for a in arrs):
                    storage = "dense"
        if storage == "dense":
            arrs = [np.ascontiguousarray(np.asarray(a.todense() if sp.issparse(a) else a),
                                         dtype=np.float32) for a in layers]
            n = arrs[0].shape[0]
            for a in arrs:
                if a.shape != (n, n):
                    raise ValueError("all layers must be square and share the node set")
            self._check(self.lib.n2v2r_set_num_layers(self.h, len(arrs), n), "set_num_layers")
            for k, a in enumerate(arrs):
                self._check(self.lib.n2v2r_set_layer_dense(self.h, k, n, a, int(symmetric)),
                            f"layer {k}")
            self.n = n
            self.num_layers = len(arrs)
            self.storage = "dense"
            return
        mats = [sp.csr_matrix(a, dtype=np.float32) for a in layers]
        n = mats[0].shape[0]
        for m in mats:
            if m.shape != (n, n):
                raise ValueError("all layers must be square and share the node set")
        self._check(self.lib.n2v2r_set_num_layers(self.h, len(mats), n), "set_num_layers")
        for k, m in enumerate(mats):
            # no sum_duplicates / sort_indices here (an O(nnz) host pass each): the engine
            # checks row order on the GPU and compares unsorted layers through (A^T)^T, and a
            # duplicate entry adds into every product exactly as its summed value would
            indptr = np.ascontiguousarray(m.indptr, dtype=np.int64)
            indices = np.ascontiguousarray(m.indices, dtype=np.int32)
            data = np.ascontiguousarray(m.data, dtype=np.float32)
            self._check(self.lib.n2v2r_set_layer_csr(self.h, k, n, int(m.nnz), indptr, indices,
                                                     data, int(symmetric)), f"layer {k}")
        self.n = n
        self.num_layers = len(mats)
        self.storage = "csr"

    def set_layer_rows(self, n: int, num_layers: int, local_layers):
        """Distributed ingest of symmetric layers from this rank's own rows only:
        ``local_layers[k]`` is the (n_local x n) CSR block of rows [row0, row0 + n_local)."""
        import scipy.sparse as sp
        self._check(self.lib.n2v2r_set_num_layers(self.h, int(num_layers), int(n)),
                    "set_num_layers")
        _, _, row0, nl = self.dist_info()
        for k, blk in enumerate(local_layers):
            m = sp.csr_matrix(blk, dtype=np.float32)
            m.sum_duplicates()
            m.sort_indices()
            if m.shape != (nl, n):
                raise ValueError(f"layer {k}: local block must be {nl} x {n}, got {m.shape}")
            self._check(self.lib.n2v2r_set_layer_csr_rows(
                self.h, k, int(n), int(row0), int(nl), int(m.nnz),
                np.ascontiguousarray(m.indptr, dtype=np.int64),
                np.ascontiguousarray(m.indices, dtype=np.int32),
                np.ascontiguousarray(m.data, dtype=np.float32)), f"layer {k} rows")
        self.n = int(n)
        self.num_layers = int(num_layers)

    # -- UASE ------------------------------------------------------------------------------
    def uase(self, d: int, block=0, max_basis=0, keep=0, max_restarts=0, tol=0.0, seed=0,
             solver_flags=0, raise_on_no_convergence=True):
        o = EigOpts(int(block), int(max_basis), int(keep), int(max_restarts), float(tol),
                    int(seed) & 0xFFFFFFFFFFFFFFFF, int(solver_flags))
        s = EigStats()
        st = self.lib.n2v2r_uase(self.h, int(d), ctypes.byref(o), ctypes.byref(s))
        if st == ERR_NO_CONVERGENCE and not raise_on_no_convergence:
            pass
        else:
            self._check(st, "uase")
        self.d = int(d)
        return s.as_dict()

    def _n_local(self):
        return self.dist_info()[3]

    def embedding(self):
        Y = np.empty((self.num_layers, self._n_local(), self.d), dtype=np.float32)
        self._check(self.lib.n2v2r_get_embedding(self.h, Y), "get_embedding")
        return Y

    def left_embedding(self):
        X = np.empty((self._n_local(), self.d), dtype=np.float32)
        self._check(self.lib.n2v2r_get_left_embedding(self.h, X), "get_left_embedding")
        return X

    def singular_values(self):
        s = np.empty(self.d, dtype=np.float64)
        self._check(self.lib.n2v2r_get_singular_values(self.h, s), "get_singular_values")
        return s

    def set_embedding(self, Y):
        Y = np.ascontiguousarray(Y, dtype=np.float32)
        K, n, d = Y.shape
        self._check(self.lib.n2v2r_set_embedding(self.h, K, n, d, Y), "set_embedding")
        self.num_layers, self.n, self.d = K, n, d

    # -- rank --------------------------------------------------------------------------------
    def rank(self, strategy: str, dims, metrics, method: int = AGG_BORDA):
        """Distances for every (comparison, dim, metric) column on the GPU; their Borda aggregate
        too unless ``method=AGG_NONE``."""
        if strategy not in STRATEGY:
            raise ValueError(f"unknown comp_strategy {strategy!r}")
        mids = []
        for m in metrics:
            if m not in METRIC:
                raise NotImplementedError("Unsupported metric")
            mids.append(METRIC[m])
        dims_a = np.ascontiguousarray(dims, dtype=np.int32)
        met_a = np.ascontiguousarray(mids, dtype=np.int32)
        ncmp = ctypes.c_int()
        ncol = ctypes.c_int()
        self._check(self.lib.n2v2r_rank(self.h, STRATEGY[strategy], dims_a, len(dims_a), met_a,
                                        len(met_a), int(method), ctypes.byref(ncmp),
                                        ctypes.byref(ncol)), "rank")
        self.ncmp, self.ncols = ncmp.value, ncol.value
        return self.ncmp, self.ncols

    def distances(self, comparison: int):
        D = np.empty((self.ncols, self.n), dtype=np.float64)
        self._check(self.lib.n2v2r_get_distances(self.h, int(comparison), D), "get_distances")
        return D.T  # N x C view (column-major on device)

    def borda(self, comparison: int):
        b = np.empty(self.n, dtype=np.int64)
        self._check(self.lib.n2v2r_get_borda(self.h, int(comparison), b), "get_borda")
        return b

    def rank_timing(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        self.lib.n2v2r_rank_timing(self.h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    # -- seams ------------------------------------------------------------------------------
    def pairwise_distances(self, m1, m2, metric: str):
        if metric not in METRIC:
            raise NotImplementedError("Unsupported metric")
        a = np.ascontiguousarray(m1, dtype=np.float64)
        b = np.ascontiguousarray(m2, dtype=np.float64)
        if a.ndim == 1:
            a = a[:, None]
            b = b[:, None]
        n, dim = a.shape
        out = np.empty(n, dtype=np.float64)
        self._check(self.lib.n2v2r_pairwise_distances(self.h, a, b, n, dim, METRIC[metric], out),
                    "pairwise_distances")
        return out

    def borda_columns(self, D, tie_order: str = "stable", return_tied: bool = False):
        """D: N x C float64 (one ranking column per column) -> int64 Borda in row order.

        tie_order "stable": every column sorted on the GPU, equal values by ascending row.
        "reference": columns holding exact ties (flagged by the GPU) are ordered as the
        reference orders them, pandas ``Series.sort_values(ascending=False)`` (numpy quicksort,
        ``model.py:173-174``), whose order of equal values is implementation-defined, and their
        positions go into the same GPU Borda; tie-free columns (every ER graph of BASELINE) are
        never touched on the host.  return_tied: also return the per-column tie flags."""
        if tie_order not in ("stable", "reference"):
            raise ValueError(f"unknown tie_order {tie_order!r}")
        Dc = np.ascontiguousarray(np.asarray(D, dtype=np.float64).T)
        c, n = Dc.shape
        out = np.empty(n, dtype=np.int64)
        tied = np.zeros(c, dtype=np.int32)
        self._check(self.lib.n2v2r_borda_columns_ex(self.h, Dc, n, c, None, 0, None, out, tied),
                    "borda_columns")
        cols = np.flatnonzero(tied)
        if tie_order == "reference" and cols.size:
            orders = np.empty((cols.size, n), dtype=np.int32)
            for g, j in enumerate(cols):
                orders[g] = reference_descending_order(Dc[j])
            gc = np.ascontiguousarray(cols, dtype=np.int32)
            self._check(self.lib.n2v2r_borda_columns_ex(
                self.h, Dc, n, c, gc.ctypes.data_as(_vp), int(cols.size),
                orders.ctypes.data_as(_vp), out, tied), "borda_columns")
        return (out, tied.astype(bool)) if return_tied else out

    def column_sums(self, k: int):
        out = np.empty(self.n, dtype=np.float32)
        self._check(self.lib.n2v2r_column_sums(self.h, int(k), out), "column_sums")
        return out

    def bench_spmm(self, k: int, X, transpose: bool = False, reps: int = 20, want_y=True):
        """Time the SpMM kernel alone (HIP events on the engine stream)."""
        X = np.ascontiguousarray(X, dtype=np.float32)
        n, b = X.shape
        Y = np.empty((self._n_local(), b), dtype=np.float32) if want_y else None
        ms, by = ctypes.c_double(), ctypes.c_double()
        yp = Y.ctypes.data_as(ctypes.c_void_p) if want_y else None
        self._check(self.lib.n2v2r_bench_spmm(self.h, int(k), int(bool(transpose)), int(b),
                                              int(reps), X, yp, ctypes.byref(ms),
                                              ctypes.byref(by)), "bench_spmm")
        return Y, ms.value, by.value

    def bench_spmm_tiled(self, k: int, X, transpose: bool = False, nb: int = 0, reps: int = 20,
                         want_y=True):
        """Time the flat-window tiled SpMM (panel width 8) of layer k alone."""
        X = np.ascontiguousarray(X, dtype=np.float32)
        n, b = X.shape
        Y = np.empty((self._n_local(), b), dtype=np.float32) if want_y else None
        ms = ctypes.c_double()
        yp = Y.ctypes.data_as(ctypes.c_void_p) if want_y else None
        self._check(self.lib.n2v2r_bench_spmm_tiled(self.h, int(k), int(bool(transpose)), int(b),
                                                    int(nb), int(reps), X, yp, ctypes.byref(ms)),
                    "bench_spmm_tiled")
        return Y, ms.value

    def spmm_col_blocks(self, b: int = 8) -> bool:
        """True when the SpMM at panel width b runs the XCD-local column-block form."""
        r = self.lib.n2v2r_spmm_col_blocks(self.h, int(b))
        if r < 0 or r > 1:
            self._check(r, "spmm_col_blocks")
        return r == 1

    def project(self, W, on: str = "columns"):
        """W^T W (on="columns") or W W^T (on="rows") of a dense m x n matrix, fp64 on the GPU
        (the reference's float64 ``np.matmul``, ``preprocessing_utils.py:22-24``)."""
        W = np.ascontiguousarray(np.asarray(W), dtype=np.float64)
        m, n = W.shape
        oc = on.casefold() == "columns"
        if not oc and on.casefold() != "rows":
            raise ValueError("Unknown projection type, options are columns or rows")
        k = n if oc else m
        out = np.empty((k, k), dtype=np.float64)
        self._check(self.lib.n2v2r_project(self.h, m, n, W, int(oc), out), "project")
        return out

    def rr_top(self, H, p: int):
        """Rayleigh-Ritz stage alone: top-p eigenpairs of symmetric H (GPU tridiagonalisation,
        bisection + inverse iteration, back-transform).  Returns (w, S)."""
        H = np.ascontiguousarray(H, dtype=np.float64)
        c = H.shape[0]
        w = np.empty(p, dtype=np.float64)
        S = np.empty((c, p), dtype=np.float32)
        self._check(self.lib.n2v2r_rr_top(self.h, c, H, int(p), w, S), "rr_top")
        return w, S

    def rr_band_top(self, hband, c: int, kp: int, theta_prev, p: int):
        """Banded Rayleigh-Ritz stage alone (see n2v2r_rr_band_top).  Returns (w, S)."""
        hband = np.ascontiguousarray(hband, dtype=np.float64).ravel()
        tp = None
        if kp > 0:
            tp = np.ascontiguousarray(theta_prev, dtype=np.float64)
        w = np.empty(p, dtype=np.float64)
        S = np.empty((c, p), dtype=np.float32)
        self._check(self.lib.n2v2r_rr_band_top(
            self.h, int(c), int(kp), hband, int(hband.size),
            None if tp is None else tp.ctypes.data_as(ctypes.c_void_p), int(p), w, S),
            "rr_band_top")
        return w, S

    def synchronize(self):
        self._check(self.lib.n2v2r_synchronize(self.h), "synchronize")


def reference_descending_order(col) -> np.ndarray:
    """Row indices of one ranking column best first, exactly as the reference sorts it:
    ``pd.Series(col, index=node_names).sort_values(ascending=False)`` (``model.py:173-174``),
    i.e. pandas ``nargsort``: reverse, ``argsort(kind='quicksort')``, reverse, NaNs last in row
    order.  The order of equal values is whatever this host's numpy quicksort gives, as in the
    reference; only columns the GPU flags as tied come here."""
    import pandas as pd
    return pd.Series(np.asarray(col, dtype=np.float64)).sort_values(
        ascending=False).index.to_numpy(dtype=np.int64)


_default = {}


def new_engine(device) -> Engine:
    """An engine on one device (int) or on several (a tuple of devices: Engine.multi)."""
    if isinstance(device, tuple):
        return Engine.multi(device)
    return Engine(device)


def default_engine(device: int = 0) -> Engine:
    """Process-wide engine per device (the handle is not thread-safe)."""
    e = _default.get(device)
    if e is None or e.h is None:
        e = Engine(device)
        _default[device] = e
    return e


def _denser_than_quarter(a) -> bool:
    """More than a quarter of the entries non-zero (the storage choice of ``set_layers``; dense
    and CSR storage give the same products).  A strided sample of ~2M entries decides when its
    density is clearly on one side of 1/4 (a dense co-expression layer: one pass over 1/200 of
    it instead of a quarter of it, 0.12 s per 20k x 20k layer); otherwise the exact count, in row
    blocks that stop as soon as the answer is known."""
    if a.size == 0:
        return False
    a2 = a.reshape(a.shape[0], -1) if a.ndim > 1 else a.reshape(1, -1)
    rows, cols = a2.shape
    stride = max(1, rows // max(1, (1 << 21) // max(1, cols)))
    if stride > 1:
        sample = a2[::stride]
        p = np.count_nonzero(sample) / sample.size
        if p > 0.3:
            return True
        if p < 0.2:
            return False
    need = a.size // 4
    step = max(1, (1 << 24) // max(1, cols))
    nz = 0
    for r in range(0, rows, step):
        nz += int(np.count_nonzero(a2[r:r + step]))
        if nz > need:
            return True
        if nz + (rows - r - step) * cols <= need:
            return False
    return nz > need


# Handles per device for the drop-in N2V2R models: a handle whose owner model is gone (or has
# none) is reused with its device allocations; a new one is made while every handle is owned,
# up to POOL_MAX, beyond which the least recently acquired handle is taken over (its owner's
# ``_hand_over()`` first copies what it still needs to the host).
POOL_MAX = 4
_pool = {}
_pool_tick = [0]


def engine_owner(eng: Engine):
    ref = getattr(eng, "_owner", None)
    return ref() if ref is not None else None


def acquire_engine(device: int, owner) -> Engine:
    import weakref
    with _lock:
        handles = _pool.setdefault(device, [])
        handles[:] = [e for e in handles if e.h is not None]
        free = [e for e in handles if engine_owner(e) is None]
        if free:
            eng = free[0]
        elif len(handles) < POOL_MAX:
            eng = new_engine(device)
            handles.append(eng)
        else:
            eng = min(handles, key=lambda e: getattr(e, "_tick", 0))
            prev = engine_owner(eng)
            if prev is not None and hasattr(prev, "_hand_over"):
                prev._hand_over()
        _pool_tick[0] += 1
        eng._tick = _pool_tick[0]
        eng._owner = weakref.ref(owner)
        return eng
