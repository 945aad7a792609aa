"""The drop-in API's output files on the GPU path against the files the reference wrote
(tests/golden/writer_er_cfg1/, see test_writer.py for the CPU half)."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN
from oracle import n2v2r_oracle as orc

pytestmark = pytest.mark.gpu

WDIR = os.path.join(GOLDEN, "writer_er_cfg1")


def _read(path):
    return pd.read_csv(path, sep="\t", index_col=0, float_precision="round_trip")


def _bytes(path):
    with open(path, "rb") as f:
        return f.read()


def _layers():
    from node2vec2rank_amd import synthetic
    return [synthetic.er_layer_p(1000, 0.01, 1000 + k) for k in range(2)]


def test_output_files_end_to_end(tmp_path, monkeypatch):
    """fit_transform_rank -> aggregate_transform -> degree_difference_ranking ->
    signed_ranks_transform with save_dir set: config.json and {key}_degDif.tsv byte-identical
    (DeDi is exact), the distance files with the reference's header, index and layout and
    values within the UASE tolerance, the sign pattern of the signed files identical."""
    from node2vec2rank_amd.model import N2V2R
    cfg = json.loads(_bytes(os.path.join(WDIR, "config.json")))
    monkeypatch.chdir(tmp_path)
    layers = _layers()
    nodes = [f"g{i}" for i in range(1000)]
    m = N2V2R(graphs=layers, nodes=nodes, config=cfg)
    m.fit_transform_rank()
    m.aggregate_transform()
    m.degree_difference_ranking()
    m.signed_ranks_transform()
    (run,) = os.listdir(tmp_path / "out")
    run = tmp_path / "out" / run
    assert sorted(os.listdir(run)) == sorted(os.listdir(WDIR))
    for f in ("config.json", "1_degDif.tsv"):
        assert _bytes(run / f) == _bytes(os.path.join(WDIR, f)), f
    # the reference's own seed-to-seed envelope of these distances (ARPACK start vector)
    Ya, _, _ = orc.uase(layers, max(cfg["embed_dimensions"]), seed=cfg["seed"])
    Yb, _, _ = orc.uase(layers, max(cfg["embed_dimensions"]), seed=cfg["seed"] + 1)
    Da = orc.rank_distances(Ya, cfg["embed_dimensions"], cfg["distance_metrics"], "sequential")
    Db = orc.rank_distances(orc.align_signs(Yb, Ya), cfg["embed_dimensions"],
                            cfg["distance_metrics"], "sequential")
    env = np.nanmax(np.abs(Da["1"][1] - Db["1"][1]))
    for f in ("1.tsv", "1_signed.tsv"):
        ours, ref = _read(run / f), _read(os.path.join(WDIR, f))
        with open(run / f) as a, open(os.path.join(WDIR, f)) as b:
            assert a.readline() == b.readline()  # header line
        assert list(ours.index) == list(ref.index)
        np.testing.assert_array_equal(np.isnan(ours.to_numpy()), np.isnan(ref.to_numpy()))
        err = np.nanmax(np.abs(ours.to_numpy() - ref.to_numpy()))
        assert err <= max(1e-4, 20 * env), (f, err, env)
    s_ours = np.signbit(_read(run / "1_agg_signed.tsv").to_numpy())
    s_ref = np.signbit(_read(os.path.join(WDIR, "1_agg_signed.tsv")).to_numpy())
    np.testing.assert_array_equal(s_ours, s_ref)


def test_agg_tsv_byte_identical_from_reference_frames(tmp_path, monkeypatch):
    """aggregate_transform recomputes Borda on the GPU from the current frames (as the
    reference does, model.py:167-185): given the reference's distance frame it writes the
    reference's {key}_agg.tsv byte for byte (these columns are tie-free)."""
    from node2vec2rank_amd.model import N2V2R
    cfg = json.loads(_bytes(os.path.join(WDIR, "config.json")))
    monkeypatch.chdir(tmp_path)
    nodes = [f"g{i}" for i in range(1000)]
    m = N2V2R(graphs=_layers(), nodes=nodes, config=cfg)
    ref = _read(os.path.join(WDIR, "1.tsv"))
    D = ref.to_numpy()
    assert all(len(np.unique(c[~np.isnan(c)])) == (~np.isnan(c)).sum() for c in D.T)
    m.pairwise_ranks = {"1": ref}
    agg = m.aggregate_transform()
    (run,) = os.listdir(tmp_path / "out")
    assert _bytes(tmp_path / "out" / run / "1_agg.tsv") == _bytes(os.path.join(WDIR, "1_agg.tsv"))
    np.testing.assert_array_equal(agg["1"]["borda_ranks"].to_numpy(),
                                  orc.borda_reference_loop(D))


def test_aggregate_follows_edited_frames():
    """Like the reference, Borda is taken from the frames as they are when
    aggregate_transform runs: a dropped column, reordered rows and rows removed from a frame
    (read against node_names: missing nodes rank last) all change the result the same way
    the reference's restatement does."""
    from node2vec2rank_amd.model import N2V2R
    layers = _layers()
    nodes = [f"g{i}" for i in range(1000)]
    cfg = dict(embed_dimensions=[2, 8], distance_metrics=["cosine", "euclidean"], seed=42,
               comp_strategy="sequential", verbose=-1, save_dir=None)
    m = N2V2R(graphs=layers, nodes=nodes, config=cfg)
    ranks = m.fit_transform_rank()
    full = m.aggregate_transform()["1"]["borda_ranks"].to_numpy()
    np.testing.assert_array_equal(full, orc.borda(ranks["1"].to_numpy()))
    edited = ranks["1"].drop(columns=["dim-2_distance-cosine"]).iloc[::-1].iloc[:900]
    m.pairwise_ranks = {"1": edited}
    got = m.aggregate_transform()["1"]
    assert list(got.index) == nodes
    D = edited.reindex(nodes).to_numpy()
    np.testing.assert_array_equal(got["borda_ranks"].to_numpy(), orc.borda(D))
