"""The output frames' node index (model._label_index) equals pandas' own ``pd.Index(nodes)``
-- values, dtype and inferred type -- for every label kind the reference accepts (CPU)."""
import numpy as np
import pandas as pd
import pytest

from node2vec2rank_amd.model import _label_index


@pytest.mark.parametrize("nodes", [
    [f"gene{i}" for i in range(20_000)],                  # the fast path
    [f"gene{i}" for i in range(20_000)] + [None],         # a missing label: pandas' path
    [f"gene{i}" for i in range(20_000)] + [7],            # mixed
    [f"gene{i}" for i in range(20_000)] + [np.nan],
    [f"gene{i}" for i in range(20_000)] + [("a", 1)],    # a tuple after strings
    [f"gene{i}" for i in range(20_000)] + [b"raw"],
    [f"gene{i}" for i in range(20_000)] + [pd.Timestamp("2020-01-01")],
    [f"2020-01-{1 + i % 28:02d}" for i in range(20_000)],  # date-like strings stay strings
    [f"{i}" for i in range(20_000)],                      # digit strings stay strings
    list(range(20_000)),                                  # integer labels
    [float(i) for i in range(20_000)],
    [("a", i) for i in range(5000)],                      # tuples: a MultiIndex
    ["x", "y", "z"],                                      # short lists
])
def test_label_index_matches_pandas(nodes):
    a, b = _label_index(nodes), pd.Index(nodes)
    assert type(a) is type(b)
    assert a.dtype == b.dtype and a.inferred_type == b.inferred_type
    assert a.equals(b)
    assert list(a[:5]) == list(b[:5])
