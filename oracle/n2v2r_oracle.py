"""CPU restatement of the node2vec2rank fit-and-rank path -- TEST INFRASTRUCTURE ONLY.

This module is the parity *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product package
(``node2vec2rank_amd``) never imports it and has no CPU fallback.

Parity pin: every function here is checked against golden vectors produced by running the
reference itself (``/root/reference/node2vec2rank/model.py`` unchanged, with a restated
``spectral_embedding.UASE``) in the survey container -- see ``tests/golden/make_golden.py``
and ``tests/test_oracle_golden.py``.  The UASE arithmetic lives in the un-vendored, unpinned
third-party package ``spectral_embedding`` (git+https://github.com/iggallagher/Spectral-Embedding,
``environment.yaml:19``), which delegates to ``scipy.sparse.linalg.svds`` (reference pins scipy
1.10.1, ``environment.yaml:10``; 1.15.3 here).  Its restatement below is pinned only through
its observable consequences: the demo notebook's recall 0.68 / DeDi 0.0
(``notebooks/node2vec2rank_demo.ipynb:176-177``) and the (K, N, d) indexing contract at
``node2vec2rank/model.py:75-84``.

Two flavours are provided:
  * ``faithful`` -- the reference's own algorithm: ARPACK ``svds`` with the start vector drawn
    from ``RandomState(seed)`` exactly as ``N2V2R.__init__`` seeds the global RNG
    (``model.py:36-38``), per-row scipy distances (``model_utils.py:55-63``) and the
    quicksort-ordered Borda (``model.py:171-175`` + ``model_utils.py:22-34``).  Bit-exact with
    the reference on this container.
  * ``fast`` -- vectorised distances and an O(N log N) Borda; tie order = stable sort
    (descending value, ascending node index, NaN last), which is the order the HIP path
    implements.  On tie-free inputs both flavours agree exactly.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.spatial.distance
from scipy.sparse.linalg import svds

STRATEGIES = ("sequential", "one_vs_before", "one_vs_rest")
METRICS = ("cosine", "euclidean", "correlation")


# --------------------------------------------------------------------------------------
# A3/A4: UASE = truncated SVD of the unfolded matrix [A_1 | ... | A_K]
# --------------------------------------------------------------------------------------
def uase(layers, d: int, seed=None):
    """Restates ``se.UASE(list_of_csc, d)`` as called at ``model.py:53-55``.

    ``A = hstack(A_k)`` (N x K*N); ``svds(A, d)`` (ARPACK on the Gram operator ``A A^T``
    because N < K*N, start vector ``standard_normal(N)`` from the seeded global RandomState,
    scipy ``_svds.py:507-508``); singular values reordered descending; right embedding
    ``V diag(sqrt(s))`` split into K row blocks -> (K, N, d) float64.
    Returns ``(Y, s_desc, X_left)``.
    """
    mats = [sp.csc_matrix(g) for g in layers]  # model.py:53
    K = len(mats)
    n = mats[0].shape[0]
    A = sp.hstack(mats)
    rs = np.random.RandomState(seed) if seed else np.random.mtrand._rand
    u, s, vT = svds(A, d, random_state=rs)
    o = np.argsort(s[::-1])  # upstream idiom: ascending svds output -> descending order
    S = np.sqrt(s[o])
    x_left = u[:, o] @ np.diag(S)
    y_right = vT.T[:, o] @ np.diag(S)
    Y = np.zeros((K, n, d))
    for k in range(K):
        Y[k] = y_right[k * n:(k + 1) * n]
    return Y, s[o], x_left


# --------------------------------------------------------------------------------------
# A5: comparison keys and the (embed_one, embed_two) pairs per strategy
# --------------------------------------------------------------------------------------
def comparisons(num_graphs: int, strategy: str):
    """Keys and layer index i of each comparison (``model.py:59-66``)."""
    if strategy not in STRATEGIES:
        raise ValueError(f"unknown comp_strategy {strategy!r}")
    out = []
    for i in range(num_graphs):
        if i == 0 and strategy != "one_vs_rest":
            continue
        key = str(i) if strategy != "one_vs_rest" else str(i + 1)
        out.append((key, i))
    return out


def embed_pair(Y, i: int, dim: int, strategy: str):
    """(embed_one, embed_two) for comparison layer i at prefix dim (``model.py:74-84``)."""
    if strategy == "sequential":
        return Y[i - 1, :, :dim], Y[i, :, :dim]
    if strategy == "one_vs_before":
        return np.mean(Y[:i, :, :dim], axis=0), Y[i, :, :dim]
    if strategy == "one_vs_rest":
        return np.mean(Y[np.arange(Y.shape[0]) != i, :, :dim], axis=0), Y[i, :, :dim]
    raise ValueError(strategy)


def column_names(dims, metrics):
    """Column order of a comparison's DataFrame: dims outer, metrics inner, cosine skipped at
    dim == 1 (``model.py:73,87-90``)."""
    cols = []
    for dim in dims:
        for m in metrics:
            if m == "cosine" and dim == 1:
                continue
            cols.append((dim, m, f"dim-{dim}_distance-{m}"))
    return cols


# --------------------------------------------------------------------------------------
# A6: per-node distances
# --------------------------------------------------------------------------------------
def distances_faithful(m1, m2, metric: str):
    """Per-row scipy calls exactly as ``model_utils.py:55-63``."""
    if metric == "cosine":
        f = scipy.spatial.distance.cosine
    elif metric == "euclidean":
        f = scipy.spatial.distance.euclidean
    elif metric == "correlation":
        f = scipy.spatial.distance.correlation
    else:
        raise NotImplementedError("Unsupported metric")
    with np.errstate(all="ignore"):
        return np.array([f(a, b) for a, b in zip(m1, m2)], dtype=np.float64)


def distances_fast(m1, m2, metric: str):
    """Vectorised fp64 restatement of scipy's formulas
    (``scipy/spatial/distance.py``: ``correlation(centered=False)`` for cosine,
    ``1 - uv/sqrt(uu*vv)`` clipped to [0, 2]; euclidean ``sqrt((u-v).(u-v))``)."""
    m1 = np.asarray(m1, dtype=np.float64)
    m2 = np.asarray(m2, dtype=np.float64)
    with np.errstate(all="ignore"):
        if metric == "euclidean":
            diff = m1 - m2
            return np.sqrt(np.einsum("ij,ij->i", diff, diff))
        if metric == "cosine":
            a, b = m1, m2
        elif metric == "correlation":
            a = m1 - m1.mean(axis=1, keepdims=True)
            b = m2 - m2.mean(axis=1, keepdims=True)
        else:
            raise NotImplementedError("Unsupported metric")
        uv = np.einsum("ij,ij->i", a, b)
        uu = np.einsum("ij,ij->i", a, a)
        vv = np.einsum("ij,ij->i", b, b)
        return np.clip(1.0 - uv / np.sqrt(uu * vv), 0.0, 2.0)


def rank_distances(Y, dims, metrics, strategy: str, faithful: bool = False):
    """``N2V2R.__rank`` (``model.py:57-96``): dict key -> (column names, N x C float64)."""
    fn = distances_faithful if faithful else distances_fast
    out = {}
    cols = column_names(dims, metrics)
    for key, i in comparisons(Y.shape[0], strategy):
        D = np.empty((Y.shape[1], len(cols)), dtype=np.float64)
        for c, (dim, m, _) in enumerate(cols):
            e1, e2 = embed_pair(Y, i, dim, strategy)
            D[:, c] = fn(e1, e2, m)
        out[key] = ([name for _, _, name in cols], D)
    return out


# --------------------------------------------------------------------------------------
# A8/A9: Borda aggregation
# --------------------------------------------------------------------------------------
def _descending_order_pandas(col, kind: str):
    """``Series.sort_values(ascending=False)`` = pandas ``nargsort``: reverse, argsort
    (``kind``), reverse; NaNs appended last in index order
    (``pandas/core/sorting.py:437-441``; called from ``model.py:173-174``)."""
    col = np.asarray(col, dtype=np.float64)
    idx = np.arange(col.shape[0])
    mask = np.isnan(col)
    good_idx = idx[~mask]
    good = col[~mask]
    order = good_idx[::-1][good[::-1].argsort(kind=kind)][::-1]
    return np.concatenate([order, idx[mask]])


def borda(D, faithful: bool = False):
    """int64 Borda scores in node order: ``score[n] = sum_c (N - pos_c(n))``
    (``model_utils.py:22-34``, reordered to node order at ``model.py:185``).

    ``faithful``: numpy quicksort exactly as the reference (tie order implementation-defined).
    otherwise: stable sort (descending value, ascending node index on ties, NaN last)."""
    D = np.asarray(D, dtype=np.float64)
    n, c = D.shape
    score = np.zeros(n, dtype=np.int64)
    for j in range(c):
        order = _descending_order_pandas(D[:, j], "quicksort" if faithful else "stable")
        pos = np.empty(n, dtype=np.int64)
        pos[order] = np.arange(n)
        score += n - pos
    return score


def borda_reference_loop(D):
    """The literal O(C N^2) loop of ``model_utils.py:22-25`` (small N only; baseline timing)."""
    D = np.asarray(D, dtype=np.float64)
    n, c = D.shape
    rankings = [list(_descending_order_pandas(D[:, j], "quicksort")) for j in range(c)]
    index = rankings[0]
    res = np.asarray([[n - r.index(node) for node in index] for r in rankings])
    tot = res.sum(axis=0)
    out = np.empty(n, dtype=np.int64)
    out[np.asarray(index)] = tot
    return out


def _get_ranking(ranking, index):
    """``model_utils.py:22-25``: N - position of every node of ``index`` in ``ranking``."""
    n = len(index)
    return [n - ranking.index(node) for node in index]


def borda_reference_parallel(D, n_jobs=-2):
    """``borda_aggregate_parallel`` (``model_utils.py:28-36``) as the reference runs it: the
    per-column rankings as Python lists of node ids (``model.py:171-175``), the O(N^2)
    ``list.index`` scoring fanned out over a joblib process pool, int64 sums; returned in node
    order (``model.py:185``).  Baseline timing only (small N)."""
    from joblib import Parallel, delayed
    D = np.asarray(D, dtype=np.float64)
    n, c = D.shape
    rankings = [list(_descending_order_pandas(D[:, j], "quicksort")) for j in range(c)]
    index = rankings[0]
    res = np.asarray(Parallel(n_jobs=n_jobs)(delayed(_get_ranking)(r, index) for r in rankings))
    out = np.empty(n, dtype=np.int64)
    out[np.asarray(index)] = res.sum(axis=0)
    return out


# --------------------------------------------------------------------------------------
# Whole path + DeDi (model.py:282-311)
# --------------------------------------------------------------------------------------
def fit_rank_borda(layers, dims, metrics, strategy="sequential", seed=42, faithful=True):
    Y, s, _ = uase(layers, max(dims), seed=seed)
    ranks = rank_distances(Y, dims, metrics, strategy, faithful=faithful)
    agg = {k: borda(D, faithful=faithful) for k, (_, D) in ranks.items()}
    return Y, s, ranks, agg


def degree_difference(layers):
    """``degree_difference_ranking`` (``model.py:282-311``): float32 column sums of layer i-1
    minus layer i -> (DeDi, absDeDi) per key."""
    out = {}
    for i in range(1, len(layers)):
        a = np.asarray(sp.csr_matrix(layers[i - 1]).sum(axis=0), dtype=np.float32).ravel()
        b = np.asarray(sp.csr_matrix(layers[i]).sum(axis=0), dtype=np.float32).ravel()
        dedi = a - b
        out[str(i)] = (dedi, np.abs(dedi))
    return out


def signed_transform_single(ranks, prior):
    """``signed_transform_single`` (``model_utils.py:7-19``), literally: for every node of
    ``ranks`` (a Series) that the prior's index holds, the rank if the prior's value is > 0,
    else its negation; returns a Series in ``ranks``' order.  Small inputs only (a Python loop
    with ``prior.loc`` per node, as the reference)."""
    import pandas as pd
    names, vals = [], []
    for index, rank in ranks.items():
        if index in prior.index:
            names.append(index)
            vals.append(rank if prior.loc[index] > 0 else -rank)
    return pd.Series(vals, index=names)


# --------------------------------------------------------------------------------------
# Helpers for parity checks
# --------------------------------------------------------------------------------------
def align_signs(Y_test, Y_ref):
    """Flip each embedding column of ``Y_test`` (K, N, d) to best match ``Y_ref``; the SVD's
    per-column sign is arbitrary and cancels in every distance."""
    Y_test = np.array(Y_test, dtype=np.float64, copy=True)
    for j in range(Y_ref.shape[2]):
        if np.sum(Y_test[:, :, j] * Y_ref[:, :, j]) < 0:
            Y_test[:, :, j] *= -1
    return Y_test


def kendall_tau(a, b):
    from scipy.stats import kendalltau
    return kendalltau(a, b).statistic
