"""GPU forms of the reference's numeric seams (``node2vec2rank/model_utils.py``).

``compute_pairwise_distances`` (model_utils.py:39-67) and ``borda_aggregate_parallel``
(model_utils.py:28-36) keep their signatures and return types; the arithmetic runs in
libn2v2r_hip.so.  ``signed_transform_single`` (model_utils.py:7-19) is host bookkeeping.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from . import _lib


def compute_pairwise_distances(mat1, mat2, distance='cosine'):
    """Per-row distance between two (n_nodes, d) embedding matrices -> list of floats."""
    if distance not in ("cosine", "euclidean", "correlation"):
        raise NotImplementedError("Unsupported metric")
    return list(_lib.default_engine().pairwise_distances(mat1, mat2, distance))


def borda_aggregate_parallel(rankings: list):
    """Borda over label rankings (each a list of node labels, best first) ->
    ``DataFrame(index=rankings[0], columns=['borda_ranks'])``, int64."""
    index = pd.Index(rankings[0])
    n = len(index)
    # a ranking's order is encoded as the value -position, so the GPU's descending sort
    # reproduces it exactly (no ties: positions are distinct)
    D = np.empty((n, len(rankings)), dtype=np.float64)
    for c, r in enumerate(rankings):
        pos = np.empty(n, dtype=np.float64)
        loc = index.get_indexer(pd.Index(r))
        if (loc < 0).any() or len(r) != n:
            raise ValueError("every ranking must be a permutation of the same node labels")
        pos[loc] = np.arange(n, dtype=np.float64)
        D[:, c] = -pos
    scores = _lib.default_engine().borda_columns(D)
    return pd.DataFrame(scores, index=index, columns=['borda_ranks'])


def signed_transform_single(ranks: pd.Series, prior_signed_ranks: pd.Series):
    """``model_utils.py:7-19``: the nodes of ``ranks`` that the prior's index holds, in ``ranks``'
    order, each rank kept where the prior's value is > 0 and negated otherwise (a NaN prior
    fails ``> 0``: negated).  Negation, not a multiplication by -1, as the reference (``-rank``,
    ``model_utils.py:17``): the two differ on a NaN rank's sign bit."""
    keep = ranks.index.isin(prior_signed_ranks.index)
    sub = ranks[keep]
    if len(sub) == 0:
        return pd.Series([], index=[])  # the reference's pd.Series([], index=[])
    pos = prior_signed_ranks.reindex(sub.index).to_numpy() > 0
    vals = sub.to_numpy()
    return pd.Series(np.where(pos, vals, -vals), index=sub.index)
