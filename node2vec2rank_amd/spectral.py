"""GPU ``UASE`` with the call contract of ``spectral_embedding.UASE`` as the reference uses it
(``node2vec2rank/model.py:53-55``, indexing contract ``model.py:75-84``)."""
from __future__ import annotations

import numpy as np

from . import _lib


def UASE(As, d, seed=None, device=0, **eig_options):
    """Unfolded adjacency spectral embedding of layers ``As`` (K square N x N matrices).

    Returns ``(XA, YA)``: left embedding ``U diag(sqrt(sigma))`` (N x d) and the right
    embedding ``V diag(sqrt(sigma))`` split per layer, shape (K, N, d), columns in descending
    singular-value order.
    """
    eng = _lib.default_engine(device)
    eng.set_layers(list(As))
    if seed is None:
        seed = int(np.random.randint(1, 2**31 - 1))
    eng.uase(int(d), seed=seed, **eig_options)
    return eng.left_embedding().astype(np.float64), eng.embedding().astype(np.float64)
