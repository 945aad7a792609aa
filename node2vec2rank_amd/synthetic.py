"""Synthetic multilayer graphs for tests and the bench (host-side numpy, not on the hot path).

Layer recipe follows SURVEY.md 8(d): symmetric Erdos-Renyi, no self loops, binary weights
1.0f, one ``numpy.random.default_rng(seed_base + k)`` stream per layer, so layers are
independent and distances have no exact ties.  Edges are drawn as ``N*avg_deg/2`` random
(i, j) pairs; duplicates and self loops are dropped, so the realised mean degree is a hair
under ``avg_deg``.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def er_layer(n: int, avg_deg: float, seed: int, dtype=np.float32) -> sp.csr_matrix:
    rng = np.random.default_rng(seed)
    m = int(round(n * avg_deg / 2.0))
    i = rng.integers(0, n, size=m, dtype=np.int64)
    j = rng.integers(0, n, size=m, dtype=np.int64)
    keep = i != j
    i, j = i[keep], j[keep]
    lo = np.minimum(i, j)
    hi = np.maximum(i, j)
    key = np.unique(lo * n + hi)
    lo = key // n
    hi = key % n
    rows = np.concatenate([lo, hi])
    cols = np.concatenate([hi, lo])
    data = np.ones(rows.shape[0], dtype=dtype)
    a = sp.csr_matrix((data, (rows, cols)), shape=(n, n))
    a.sum_duplicates()
    a.sort_indices()
    return a


def er_layers(n: int, avg_deg: float, num_layers: int = 2, seed_base: int = 1000):
    return [er_layer(n, avg_deg, seed_base + k) for k in range(num_layers)]


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def er_layer_rows(n: int, avg_deg: float, seed: int, row0: int = 0, n_rows: int | None = None,
                  chunk: int = 1 << 23, dtype=np.float32) -> sp.csr_matrix:
    """Rows [row0, row0 + n_rows) of a symmetric ER layer whose edges are counter-based:
    edge e (0 <= e < N avg_deg / 2) joins splitmix64 draws i(e), j(e).  Every rank of a
    row-partitioned run builds only its own rows (scanning the edge counter in chunks, memory
    O(local nnz)), and the union over ranks is exactly ``er_layer_rows(n, avg_deg, seed)``.
    Self loops dropped, duplicate pairs merged, weights 1.0 (same recipe as ``er_layer``, a
    different random stream)."""
    if n_rows is None:
        n_rows = n - row0
    row1 = row0 + n_rows
    m = int(round(n * avg_deg / 2.0))
    s = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    nn = np.uint64(n)
    keys = []
    with np.errstate(over="ignore"):
        for e0 in range(0, m, chunk):
            e = np.arange(e0, min(m, e0 + chunk), dtype=np.uint64)
            h1 = _splitmix64(s ^ (e * np.uint64(0x2545F4914F6CDD1D)))
            h2 = _splitmix64(h1)
            i = ((h1 >> np.uint64(32)) * nn) >> np.uint64(32)
            j = ((h2 >> np.uint64(32)) * nn) >> np.uint64(32)
            i = i.astype(np.int64)
            j = j.astype(np.int64)
            ok = i != j
            i, j = i[ok], j[ok]
            a = (i >= row0) & (i < row1)
            b = (j >= row0) & (j < row1)
            keys.append((i[a] - row0) * n + j[a])
            keys.append((j[b] - row0) * n + i[b])
    key = np.unique(np.concatenate(keys)) if keys else np.zeros(0, np.int64)
    rows = key // n
    cols = (key % n).astype(np.int32)
    indptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=n_rows), out=indptr[1:])
    return sp.csr_matrix((np.ones(key.shape[0], dtype=dtype), cols, indptr),
                         shape=(n_rows, n))


def fingerprint(layers) -> np.ndarray:
    """Cheap fingerprint of regenerated layers (nnz, sum of column indices, a row-pointer hash
    per layer): fixtures that store a generator instead of the CSR check it."""
    out = []
    for a in layers:
        a = sp.csr_matrix(a)
        out.append([int(a.nnz), int(a.indices.astype(np.int64).sum()),
                    int((a.indptr.astype(np.int64) * 7919 % 1000003).sum())])
    return np.asarray(out, dtype=np.int64)


def er_layer_p(n: int, p: float, seed: int) -> sp.csr_matrix:
    """ER with edge probability p (BASELINE cfg1: N=1000, p=0.01)."""
    return er_layer(n, p * (n - 1), seed)


def sbm_layers(n: int, num_layers: int, k_comm: int = 5, p_in: float = 0.2,
               p_out: float = 0.02, rewire_frac: float = 0.15, seed: int = 0):
    """Planted-partition layers whose first community's links are rewired layer by layer
    (a small stand-in for the reference's demo graphs, data/networks/demo)."""
    rng = np.random.default_rng(seed)
    comm = rng.integers(0, k_comm, size=n)
    layers = []
    for k in range(num_layers):
        p = np.where(comm[:, None] == comm[None, :], p_in, p_out)
        if k > 0:
            changed = comm == 0
            shuffle = rng.permutation(k_comm)
            ck = np.where(changed, shuffle[comm], comm)
            flip = changed & (rng.random(n) < max(rewire_frac * k, 1.0))
            ck = np.where(flip, ck, comm)
            p = np.where(ck[:, None] == ck[None, :], p_in, p_out)
        u = rng.random((n, n)) < p
        u = np.triu(u, 1)
        a = (u | u.T).astype(np.float32)
        layers.append(sp.csr_matrix(a))
    return layers, comm


def lowrank_layers(us: np.ndarray, right: list) -> list:
    """Dense float32 layers ``A_k = us @ right[k].T`` of a rank-r two-layer network given its
    factors (``tests/golden/make_golden.py lowrank_exact``: ``us`` = left singular vectors x
    singular values, ``right[k]`` = layer k's rows of the right singular vectors).  The product
    is summed term by term in float64 with elementwise numpy operations (no BLAS, no fused
    multiply-add), so the float32 result is the same bytes on every host; the fixture stores
    their SHA-256."""
    out = []
    for v in right:
        acc = np.zeros((us.shape[0], v.shape[0]), dtype=np.float64)
        for j in range(us.shape[1]):
            acc = acc + np.multiply.outer(us[:, j], v[:, j])
        out.append(np.ascontiguousarray(acc.astype(np.float32)))
    return out


def corr_layer(n: int, samples: int = 200, seed: int = 0) -> np.ndarray:
    """Dense co-expression layer (BASELINE cfg3): |corrcoef| of an n x samples
    Gaussian matrix drawn from ``default_rng(seed)``, fp32, symmetric, unit diagonal."""
    g = np.random.default_rng(seed).standard_normal((n, samples))
    g -= g.mean(axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    c = g @ g.T
    np.abs(c, out=c)
    out = c.astype(np.float32)
    del c
    # exact symmetry (the GEMM is symmetric up to rounding) and unit diagonal, as corrcoef
    out = np.triu(out) + np.triu(out, 1).T
    np.fill_diagonal(out, 1.0)
    return np.ascontiguousarray(out)


def corr_layers(n: int, num_layers: int = 4, samples: int = 200, seed_base: int = 0):
    return [corr_layer(n, samples, seed_base + k) for k in range(num_layers)]
