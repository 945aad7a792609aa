"""CSR ingest: the reference ``DataLoader`` (``node2vec2rank/dataloader.py:14-109``) without
its dense N x N path, so cfg4/cfg5-sized graphs can be fed from files.

Same config keys and the same sequence of operations as the reference:

* per file (``dataloader.py:85-105``): weighted edge list (``is_edge_list``; networkx
  ``read_weighted_edgelist(nodetype=str)`` semantics: undirected, a repeated pair keeps its
  LAST weight, self loops kept once, node order = order of first appearance) or an adjacency
  table (CSV with a header row and an index column, or HDF5); optional transpose;
* ``match_networks`` (``preprocessing_utils.py:291-306``): rows and columns restricted to the
  labels common to every layer;
* ``network_transform`` (``preprocessing_utils.py:116-141``) per layer: absolute ->
  threshold (entries < threshold -> 0) -> bipartite projection of non-square layers (GPU,
  ``Engine.project``) -> drop entries below the ``100 - top_percent_keep`` percentile of the
  non-zeros -> binarize -> float32.

Layers come out as scipy CSR float32 (``get_graphs()``) over the common nodes
(``get_nodes()``), ready for ``node2vec2rank_amd.model.N2V2R``.

Deliberate difference: the reference orders the common nodes by ``list(set(...))``, i.e. by
Python string hashing (it changes with PYTHONHASHSEED, ``preprocessing_utils.py:300-301``).
Here the order is deterministic: the first layer's order, restricted to the common labels.
Every downstream result is permutation-equivariant, so outputs agree label by label.
"""
from __future__ import annotations

import os
import time

import numpy as np
import pandas as pd
import scipy.sparse as sp


class Layer:
    """A loaded layer: CSR values over (row labels x column labels)."""

    def __init__(self, mat: sp.csr_matrix, rows, cols):
        self.mat = sp.csr_matrix(mat)
        self.rows = np.asarray(rows, dtype=object)
        self.cols = np.asarray(cols, dtype=object)

    @property
    def shape(self):
        return self.mat.shape

    def T(self):
        return Layer(self.mat.T.tocsr(), self.cols, self.rows)


def read_weighted_edgelist(path: str, separator: str = " ") -> Layer:
    """networkx ``read_weighted_edgelist(delimiter=separator, nodetype=str)`` +
    ``to_numpy_array`` as a sparse symmetric matrix (``dataloader.py:96-100``)."""
    sep = separator if separator not in (None, " ") else r"\s+"
    df = pd.read_csv(path, sep=sep, header=None, names=["u", "v", "w"], dtype={"u": str, "v": str},
                     engine="c" if sep != r"\s+" else "python", comment="#")
    u = df["u"].to_numpy(dtype=object)
    v = df["v"].to_numpy(dtype=object)
    w = df["w"].to_numpy(dtype=np.float64)
    # node order: first appearance, u before v on each line (networkx add_edge order)
    inter = np.empty(2 * len(u), dtype=object)
    inter[0::2] = u
    inter[1::2] = v
    codes, labels = pd.factorize(inter, sort=False)
    iu, iv = codes[0::2].astype(np.int64), codes[1::2].astype(np.int64)
    n = len(labels)
    # an undirected pair keeps the last weight written (add_edge overwrites)
    lo, hi = np.minimum(iu, iv), np.maximum(iu, iv)
    key = lo * n + hi
    last = pd.Series(np.arange(len(key))).groupby(key).last().to_numpy()
    lo, hi, w = lo[last], hi[last], w[last]
    off = lo != hi
    rows = np.concatenate([lo, hi[off]])
    cols = np.concatenate([hi, lo[off]])
    vals = np.concatenate([w, w[off]])
    mat = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    mat.sum_duplicates()
    return Layer(mat, labels, labels)


def read_adjacency(path: str, separator: str = ",") -> Layer:
    """``pd.read_csv(index_col=0, header=0, sep=separator)`` or ``pd.read_hdf`` of an adjacency
    table (``dataloader.py:86-94``)."""
    if path.split(".")[-1] == "h5":
        df = pd.read_hdf(path)
    else:
        df = pd.read_csv(path, index_col=0, header=0, sep=separator)
    vals = np.asarray(df.values, dtype=np.float64)
    return Layer(sp.csr_matrix(vals), df.index.to_numpy(), df.columns.to_numpy())


def match_layers(layers: list[Layer]) -> list[Layer]:
    """``match_networks`` (``preprocessing_utils.py:291-306``) with a deterministic order."""
    common_r = set(layers[0].rows)
    common_c = set(layers[0].cols)
    for L in layers[1:]:
        common_r &= set(L.rows)
        common_c &= set(L.cols)
    rows = [x for x in layers[0].rows if x in common_r]
    cols = [x for x in layers[0].cols if x in common_c]
    out = []
    for L in layers:
        ri = pd.Index(L.rows).get_indexer(rows)
        ci = pd.Index(L.cols).get_indexer(cols)
        out.append(Layer(L.mat[ri][:, ci], rows, cols))
    return out


def _percentile_cut(values: np.ndarray, q: float) -> float:
    return float(np.percentile(values, q))


def transform(layer: Layer, threshold=None, top_percent_keep=100, binarize=False,
              absolute=False, project_unipartite_on="columns", engine=None) -> Layer:
    """``network_transform`` (``preprocessing_utils.py:116-141``) on a sparse layer."""
    m = layer.mat.astype(np.float64).tocsr(copy=True)
    rows, cols = layer.rows, layer.cols
    if absolute:
        m.data = np.abs(m.data)
    if threshold is not None:
        m.data[m.data < threshold] = 0.0
        m.eliminate_zeros()
    r, c = m.shape
    if r != c:
        if project_unipartite_on is None:
            raise ValueError("Impossible transformation")
        if engine is None:
            from node2vec2rank_amd import _lib
            engine = _lib.default_engine()
        on = project_unipartite_on.casefold()
        m = sp.csr_matrix(engine.project(m.toarray(), on))
        rows = cols = (cols if on == "columns" else rows)
    m.eliminate_zeros()
    if m.nnz == 0:
        # the reference takes np.percentile of an empty array here and raises IndexError
        raise IndexError("network_transform: layer has no non-zero entries")
    cut = _percentile_cut(m.data, 100 - top_percent_keep)
    m.data[m.data < cut] = 0.0
    m.eliminate_zeros()
    if binarize:
        m.data[:] = 1.0
    return Layer(m.astype(np.float32), rows, cols)


class DataLoader:
    """``DataLoader(config)`` (``dataloader.py:14-109``) producing CSR layers."""

    def __init__(self, config: dict, engine=None):
        self.config = config
        self.graphs = []
        self.interest_nodes = []
        self._engine = engine
        self._load()

    def get_graphs(self):
        return self.graphs

    def get_nodes(self):
        return self.interest_nodes

    def _load_one(self, filename: str, index: int) -> Layer:
        path = os.path.join(self.config["data_dir"], filename)
        sep = self.config.get("separator", ",")
        if self.config.get("is_edge_list"):
            L = read_weighted_edgelist(path, sep)
        else:
            L = read_adjacency(path, sep)
        if self.config.get("transpose"):
            L = L.T()
        print(f"\tThere are {L.shape[0]} row nodes and {L.shape[1]} column nodes in graph "
              f"{index + 1}")
        return L

    def _load(self):
        tic = time.time()
        print("Loading graphs in memory ...")
        layers = [self._load_one(f, i) for i, f in enumerate(self.config["graph_filenames"])]
        layers = match_layers(layers)
        rows, cols = layers[0].rows, layers[0].cols
        proj = self.config.get("project_unipartite_on")
        if len(rows) != len(cols):
            if proj is not None and proj.casefold() == "rows":
                self.interest_nodes = rows
                print("\tGraphs are non-square and will be projected on row nodes")
            elif proj is not None and proj.casefold() == "columns":
                self.interest_nodes = cols
                print("\tGraphs are non-square and will be projected on column nodes")
            else:
                raise ValueError("Impossible transformation")
        else:
            self.interest_nodes = cols
        print(f"\tThere are {len(self.interest_nodes)} common nodes and resulting networks will "
              f"have size {len(self.interest_nodes)} by {len(self.interest_nodes)}")
        # passed through unchanged, as dataloader.py:74 does (a fractional percentage moves the cut)
        top = self.config.get("top_percent_keep", 100)
        out = [transform(L, threshold=self.config.get("threshold"), top_percent_keep=top,
                         binarize=bool(self.config.get("binarize")),
                         absolute=bool(self.config.get("absolute")),
                         project_unipartite_on=proj, engine=self._engine) for L in layers]
        self.graphs = [L.mat for L in out]
        self.rows = np.asarray(out[0].rows, dtype=object)  # labels of the layers' rows
        self.cols = np.asarray(out[0].cols, dtype=object)  # and columns (the same nodes)
        self.interest_nodes = self.cols
        print(f"Finished loading in {round(time.time() - tic, 2)} seconds \n")
