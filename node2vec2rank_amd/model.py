"""Drop-in ``N2V2R`` for the fit-and-rank path, backed by the MI355X engine.

Mirrors ``node2vec2rank/model.py:17-311`` of the reference: same constructor, config keys,
return types, column names, dict keys, index order, printed stage lines, output files and
exceptions.  The arithmetic runs in libn2v2r_hip.so (HIP on gfx950); nothing here computes
embeddings, distances or Borda scores on the host.

Differences a user can observe (documented in DESIGN.md):
  * embeddings come from a block Krylov-Schur solver instead of ARPACK, so they match the
    reference within the tolerance stated in tests (per-column signs are arbitrary there too);
  * Borda ties (exactly equal distances): ``aggregate_transform`` orders a column that holds
    exact ties as the reference does (pandas ``sort_values`` = numpy quicksort, model.py:173-174,
    an implementation-defined order of equal values); the GPU flags such columns and sums their
    positions.  ``tie_order="stable"`` (constructor) keeps the GPU's stable order instead:
    equal values by ascending node index.  Tie-free columns are sorted on the GPU either way.
"""
from __future__ import annotations

import json
import os
import random
import time
import weakref
from datetime import datetime

import numpy as np
import pandas as pd
import scipy.sparse as sp

from . import _lib


def _as_layer(g):
    """Layers as the engine takes them: scipy sparse stays sparse (CSR), dense arrays and
    DataFrames stay dense (the engine stores them dense in HBM when they are more than 1/4
    non-zero, CSR otherwise)."""
    if isinstance(g, pd.DataFrame):
        g = g.values
    if sp.issparse(g):
        return sp.csr_matrix(g, dtype=np.float32)
    return np.ascontiguousarray(np.asarray(g, dtype=np.float32))


def _label_index(nodes):
    """``pd.Index(nodes)``, the index of every output frame.  For a list whose first label is a
    ``str`` (gene names: the common case) pandas' inference can only give an object-dtype Index
    (all strings, or strings mixed with anything else), so the object array is filled by
    ``np.fromiter`` and wrapped as is: the identical Index about 6x faster than pandas' own list
    conversion (1M labels: 25 vs 157 ms here; the type scan of round 4 cost 14 ms more).
    Anything else -- numbers, tuples, pandas' future string inference -- goes through
    ``pd.Index`` itself, whose dtype inference it then keeps."""
    if (isinstance(nodes, list) and len(nodes) > 4096 and isinstance(nodes[0], str)
            and not pd.get_option("future.infer_string")):
        return pd.Index(np.fromiter(nodes, dtype=object, count=len(nodes)), dtype=object)
    return pd.Index(nodes)


class N2V2R:
    """``N2V2R(graphs, nodes, config)`` (reference ``model.py:18``)."""

    def __init__(self, graphs: list, nodes: list, config: dict, device: int = 0,
                 eig_options: dict | None = None, tie_order: str = "reference",
                 n_gpus: int | None = None, devices: list | None = None):
        self.config = config
        self.node_names = nodes
        self.graphs = graphs
        self.num_graphs = len(graphs)
        self.embed_dimensions = self.config['embed_dimensions']
        self.max_embed_dim = max(self.embed_dimensions)
        self.distance_metrics = self.config['distance_metrics']
        self.save_dir = None
        self.comp_strategy = self.config['comp_strategy']

        self._node_embeddings = None
        self.pairwise_ranks = None
        self.pairwise_signed_ranks = None
        self.pairwise_aggregate_ranks = None
        self.pairwise_signed_aggregate_ranks = None
        self.prior_singed_ranks = None
        self.eig_stats = None
        self.stage_seconds = {}

        # model.py:36-38: a falsy seed means "unseeded"
        self._seed = None
        if self.config["seed"]:
            random.seed(self.config["seed"])
            np.random.seed(self.config["seed"])
            self._seed = int(self.config["seed"])

        now = datetime.now().strftime(r"%m_%d_%Y_%H_%M_%S")
        if self.config.get("save_dir"):
            self.save_dir = os.path.join(self.config["save_dir"], now)
            print(self.save_dir)
            os.makedirs(self.save_dir)
            with open(os.path.join(self.save_dir, "config.json"), 'w', encoding="utf-8") as f:
                json.dump(self.config, f)

        # one engine per device, shared by every model of the process (its allocations and
        # solver workspace are reused across fits); the model that last loaded its layers owns it.
        # n_gpus / devices: one engine over several GPUs (the layers row-partitioned over them,
        # one host thread per GPU inside the library, RCCL between them); the frames are the same
        if devices is None and n_gpus is not None and int(n_gpus) > 1:
            devices = list(range(int(n_gpus)))
        # (an explicit `devices` list is a multi-GPU engine even with one entry: [0] is a one-rank
        # RCCL communicator, every collective of the partitioned path through RCCL)
        self._device = tuple(int(d) for d in devices) if devices else device
        if tie_order not in ("reference", "stable"):
            raise ValueError(f"unknown tie_order {tie_order!r}")
        self.tie_order = tie_order
        self._eig_options = dict(eig_options or {})
        self._layers_loaded = False
        self._keys = None
        self._cols = None

    # ------------------------------------------------------------------------------------
    def _write_frames(self, frames, suffix):
        """``{key}{suffix}.tsv`` per frame, tab-separated with the node-label index, as the
        reference writes them (model.py:142-145, 193-196, 269-278, 306-309)."""
        for key, frame in frames.items():
            frame.to_csv(os.path.join(self.save_dir, str(key) + suffix + ".tsv"), sep='\t',
                         index=True)

    def _node_index(self):
        """``pd.Index`` of the node labels, built once per label list (building it from a
        Python list is the slowest host step of a 1M-node call; every output frame shares it)."""
        if getattr(self, "_index_src", None) is not self.node_names:
            self._index = _label_index(self.node_names)
            self._index_src = self.node_names
        return self._index

    @property
    def _engine(self):
        """This model's engine handle, from the device's pool (``_lib.acquire_engine``): a handle
        no live model owns is reused with its allocations and solver workspace; when every
        handle is owned, the least recently used one is taken over and its previous owner first
        copies to the host what it still needs from HBM (its embedding)."""
        eng = getattr(self, "_eng", None)
        if eng is not None and eng.h is not None and _lib.engine_owner(eng) is self:
            return eng
        self._eng = _lib.acquire_engine(self._device, self)
        self._layers_loaded = False
        return self._eng

    def _hand_over(self):
        """Called by the pool before another model takes this model's handle."""
        if self.eig_stats is not None and self._node_embeddings is None:
            self._node_embeddings = self._eng.embedding().astype(np.float64)
        self._layers_loaded = False
        self._eng = None

    def _load_layers(self):
        eng = self._engine
        if not self._layers_loaded:
            eng.set_layers([_as_layer(g) for g in self.graphs])
            self._layers_loaded = True
        return eng

    def __fit(self):
        """UASE on the GPU (replaces ``se.UASE``, model.py:51-55)."""
        t0 = time.time()
        eng = self._load_layers()
        self.stage_seconds["load"] = time.time() - t0
        seed = self._seed if self._seed is not None else int(np.random.randint(1, 2**31 - 1))
        opts = dict(seed=seed)
        opts.update(self._eig_options)
        self._node_embeddings = None
        self.eig_stats = None
        self.eig_stats = eng.uase(self.max_embed_dim, **opts)

    def __rank(self):
        """Distances for every comparison on the GPU (model.py:57-96).  The Borda aggregate is
        computed by ``aggregate_transform`` from the frames as they are then, as the
        reference does (model.py:167-180)."""
        eng = self._engine
        ncmp, ncols = eng.rank(self.comp_strategy, self.embed_dimensions,
                               self.distance_metrics, method=_lib.AGG_NONE)
        if self.comp_strategy != 'one_vs_rest':
            keys = [str(i) for i in range(1, self.num_graphs)]
        else:
            keys = [str(i + 1) for i in range(self.num_graphs)]
        cols = []
        for dim in self.embed_dimensions:
            for m in self.distance_metrics:
                if m == 'cosine' and dim == 1:
                    continue
                cols.append(f"dim-{dim}_distance-{m}")
        assert len(keys) == ncmp and len(cols) == ncols
        self._keys, self._cols = keys, cols
        out = {}
        for c, key in enumerate(keys):
            D = eng.distances(c)
            out[key] = pd.DataFrame(D, index=self._node_index(), columns=cols)
        return out

    def fit_transform_rank(self):
        """Computes the differential ranks of nodes for a given sequence of graphs
        (reference ``model.py:98-147``).  Returns ``dict[str, DataFrame(N x C)]``."""
        if self.config["verbose"] >= 0:
            print(f"\nRunning n2v2r with dimensions {self.embed_dimensions} and distance "
                  f"metrics {self.distance_metrics} ...")
        tic = time.time()
        tic_uase = time.time()
        self.__fit()
        toc_uase = time.time()
        if self.config["verbose"] == 1:
            print(f"\tMulti-layer embedding in {round(toc_uase - tic_uase, 2)} seconds")
        self.pairwise_ranks = self.__rank()  # (the embedding is fetched lazily from HBM)
        num_rankings = sum(len(df.columns) for df in self.pairwise_ranks.values())
        toc = time.time()
        self.stage_seconds.update(uase=toc_uase - tic_uase, rank=toc - toc_uase)
        if self.config["verbose"] >= 0:
            print(f"n2v2r computed {num_rankings} rankings for {len(self.pairwise_ranks)} "
                  f"comparison(s) in {round(toc - tic, 2)} seconds")
        if self.save_dir:
            self._write_frames(self.pairwise_ranks, "")
        return self.pairwise_ranks

    @property
    def node_embeddings(self):
        """(K, N, d_max) float64 embeddings, as ``node_embeddings`` in the reference
        (fetched from HBM on first access after ``fit_transform_rank``)."""
        if self._node_embeddings is None and self.eig_stats is not None:
            self._node_embeddings = self._engine.embedding().astype(np.float64)
        return self._node_embeddings

    @node_embeddings.setter
    def node_embeddings(self, value):
        self._node_embeddings = value

    def aggregate_transform(self, method='Borda'):
        """Borda aggregation (reference ``model.py:149-201``) of every column of the current
        ``pairwise_ranks`` frames, on the GPU (radix sort per column, int64 sums).  As in the
        reference each column is read against ``node_names`` (``pd.Series(col,
        index=node_names)``, model.py:173): rows missing from a frame rank last (NaN).
        Returns ``dict[str, DataFrame['borda_ranks']]``."""
        if self.pairwise_ranks:
            start = time.time()
            if self.config["verbose"] >= 0:
                print("\nRank aggregation with Borda ...")
            if method.casefold() != 'borda':
                raise NotImplementedError('Aggregation method not found. Available methods: Borda')
            eng = self._engine
            idx = self._node_index()
            out = {}
            for key, df in self.pairwise_ranks.items():
                if df.index is not idx and not df.index.equals(idx):
                    df = df.reindex(idx)
                b = eng.borda_columns(df.to_numpy(dtype=np.float64), tie_order=self.tie_order)
                out[key] = pd.DataFrame(b, index=idx, columns=['borda_ranks'])
            self.pairwise_aggregate_ranks = out
            if self.config["verbose"] == 1:
                print(f"\tFinished aggregation in {round(time.time() - start, 2)} seconds")
            if self.save_dir:
                self._write_frames(self.pairwise_aggregate_ranks, "_agg")
        else:
            raise ValueError("No n2v2r embeddings found")
        return self.pairwise_aggregate_ranks

    def degree_difference_ranking(self):
        """DeDi (reference ``model.py:282-311``): float32 column sums on the GPU."""
        eng = self._load_layers()
        sums = [eng.column_sums(k) for k in range(self.num_graphs)]
        out = {}
        for i in range(1, self.num_graphs):
            dedi = sums[i - 1] - sums[i]
            ranking = pd.DataFrame({"DeDi": dedi, "absDeDi": np.abs(dedi)})
            ranking.index = self.node_names
            out[str(i)] = ranking
        self.prior_singed_ranks = [v.iloc[:, 0] for v in out.values()]
        if self.save_dir:
            self._write_frames(out, "_degDif")
        return out

    def signed_ranks_transform(self, prior_signed_ranks=None):
        """Sign each ranking by a prior (reference ``model.py:203-280`` +
        ``model_utils.py:7-19``): rank kept where prior > 0, negated otherwise, restricted to
        nodes present in the prior."""
        if prior_signed_ranks is None:
            if self.prior_singed_ranks:
                prior_signed_ranks = self.prior_singed_ranks
            else:
                raise ValueError("Prior signed ranks needed, run degree_difference_ranking "
                                 "beforehand or provide them in arguments.")
        if not self.pairwise_ranks:
            raise ValueError("No n2v2r embeddings found")
        print("\nSigned ranks transformation ...")
        start = time.time()
        signed, signed_agg = {}, {}
        for index, key in enumerate(self.pairwise_ranks):
            prior = prior_signed_ranks[index]
            df = self.pairwise_ranks[key]
            keep = df.index.isin(prior.index)
            sub = df.loc[keep]
            pos = prior.reindex(sub.index).to_numpy() > 0  # NaN prior: negated, as `> 0` fails
            vals = sub.to_numpy()
            # negation (not a multiplication by -1, which keeps a NaN's sign bit)
            signed[key] = pd.DataFrame(np.where(pos[:, None], vals, -vals), index=sub.index,
                                       columns=df.columns)
            if self.pairwise_aggregate_ranks:
                agg = self.pairwise_aggregate_ranks[key].iloc[:, 0]
                agg = agg.loc[agg.index.isin(prior.index)]
                pos = prior.reindex(agg.index).to_numpy() > 0
                a = agg.to_numpy()
                signed_agg[key] = pd.DataFrame(np.where(pos, a, -a), index=agg.index,
                                               columns=["signed_agg_ranks"])
        self.pairwise_signed_ranks = signed
        if self.pairwise_aggregate_ranks:
            self.pairwise_signed_aggregate_ranks = signed_agg
        if self.config["verbose"] == 1:
            print(f"\tFinished signed transformation in {round(time.time() - start, 2)} seconds")
        if self.save_dir:
            self._write_frames(self.pairwise_signed_ranks, "_signed")
            if self.pairwise_aggregate_ranks:
                self._write_frames(self.pairwise_signed_aggregate_ranks, "_agg_signed")
        return self.pairwise_signed_ranks
