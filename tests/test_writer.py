"""Output files and the signed-ranks transform against the reference's own files (CPU).

tests/golden/writer_er_cfg1/ holds what the reference's N2V2R wrote for the er_cfg1 graphs with
``save_dir="out"`` (tests/golden/make_golden.py ``writer``): config.json (model.py:40-48),
1.tsv (:142-145), 1_agg.tsv (:193-196), 1_degDif.tsv (:306-309), 1_signed.tsv and
1_agg_signed.tsv (:269-278).  Here the reference's own frames are fed to the drop-in N2V2R
(no GPU needed: its engine is created on first use) and every file it writes must be
byte-identical; test_gpu_writer.py runs the whole path on the GPU."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN
from oracle import n2v2r_oracle as orc

WDIR = os.path.join(GOLDEN, "writer_er_cfg1")


def _read(name, **kw):
    return pd.read_csv(os.path.join(WDIR, name), sep="\t", index_col=0,
                       float_precision="round_trip", **kw)


def _bytes(path):
    with open(path, "rb") as f:
        return f.read()


def _model(tmp_path, monkeypatch):
    from node2vec2rank_amd.model import N2V2R
    cfg = json.loads(_bytes(os.path.join(WDIR, "config.json")))
    monkeypatch.chdir(tmp_path)
    nodes = [f"g{i}" for i in range(1000)]
    m = N2V2R(graphs=[None, None], nodes=nodes, config=cfg)
    (run,) = os.listdir(tmp_path / "out")
    return m, tmp_path / "out" / run, nodes


def test_config_json_byte_identical(tmp_path, monkeypatch):
    _, run, _ = _model(tmp_path, monkeypatch)
    assert _bytes(run / "config.json") == _bytes(os.path.join(WDIR, "config.json"))


def test_rank_and_agg_tsv_byte_identical(tmp_path, monkeypatch):
    """The writer of fit_transform_rank / aggregate_transform, given the reference's frames."""
    m, run, _ = _model(tmp_path, monkeypatch)
    m._write_frames({"1": _read("1.tsv")}, "")
    m._write_frames({"1": _read("1_agg.tsv")}, "_agg")
    assert _bytes(run / "1.tsv") == _bytes(os.path.join(WDIR, "1.tsv"))
    assert _bytes(run / "1_agg.tsv") == _bytes(os.path.join(WDIR, "1_agg.tsv"))


def test_signed_ranks_byte_identical(tmp_path, monkeypatch):
    """signed_ranks_transform (model.py:203-280, model_utils.py:7-19) on the reference's
    distance and Borda frames with its own DeDi prior: both output files byte-identical."""
    m, run, _ = _model(tmp_path, monkeypatch)
    m.pairwise_ranks = {"1": _read("1.tsv")}
    m.pairwise_aggregate_ranks = {"1": _read("1_agg.tsv")}
    prior = [_read("1_degDif.tsv").iloc[:, 0]]
    out = m.signed_ranks_transform(prior)
    assert list(out) == ["1"]
    assert _bytes(run / "1_signed.tsv") == _bytes(os.path.join(WDIR, "1_signed.tsv"))
    assert _bytes(run / "1_agg_signed.tsv") == _bytes(os.path.join(WDIR, "1_agg_signed.tsv"))
    # the transform itself vs the literal restatement, column by column
    for col in m.pairwise_ranks["1"].columns:
        ref = orc.signed_transform_single(m.pairwise_ranks["1"][col], prior[0])
        got = out["1"][col]
        assert list(got.index) == list(ref.index)
        np.testing.assert_array_equal(got.to_numpy(), ref.to_numpy())
    assert m.pairwise_signed_aggregate_ranks["1"]["signed_agg_ranks"].dtype == np.int64


def test_signed_ranks_partial_prior_and_zero_signs(tmp_path, monkeypatch):
    """A prior that covers only some nodes (others dropped), holds zeros and negatives (rank
    negated, -0.0 kept), in a different order than the frame, and NaN distances."""
    m, _, nodes = _model(tmp_path, monkeypatch)
    rng = np.random.default_rng(4)
    D = pd.DataFrame(rng.random((1000, 3)), index=nodes, columns=["a", "b", "c"])
    D.iloc[::50, 1] = np.nan
    D.iloc[::70, 2] = 0.0
    B = pd.DataFrame(rng.integers(3, 3000, 1000), index=nodes, columns=["borda_ranks"])
    pick = rng.permutation(1000)[:700]
    prior = pd.Series(rng.integers(-2, 3, 700).astype(np.float32), index=[nodes[i] for i in pick])
    m.pairwise_ranks = {"1": D}
    m.pairwise_aggregate_ranks = {"1": B}
    out = m.signed_ranks_transform([prior])["1"]
    for col in D.columns:
        ref = orc.signed_transform_single(D[col], prior)
        assert list(out[col].index) == list(ref.index)
        np.testing.assert_array_equal(out[col].to_numpy(), ref.to_numpy())
        np.testing.assert_array_equal(np.signbit(out[col].to_numpy()), np.signbit(ref.to_numpy()))
    ref = orc.signed_transform_single(B.iloc[:, 0], prior)
    got = m.pairwise_signed_aggregate_ranks["1"]["signed_agg_ranks"]
    assert list(got.index) == list(ref.index)
    np.testing.assert_array_equal(got.to_numpy(), ref.to_numpy())


def test_signed_ranks_needs_prior(tmp_path, monkeypatch):
    m, _, _ = _model(tmp_path, monkeypatch)
    with pytest.raises(ValueError):
        m.signed_ranks_transform()


def test_signed_transform_single_seam():
    """node2vec2rank_amd.model_utils.signed_transform_single (the seam of model_utils.py:7-19)
    vs the literal restatement: order, kept nodes, values and the sign bit of NaN / 0 ranks."""
    from node2vec2rank_amd import model_utils as mu
    rng = np.random.default_rng(8)
    names = [f"g{i}" for i in range(500)]
    vals = rng.standard_normal(500)
    vals[::40] = np.nan
    vals[::55] = 0.0
    ranks = pd.Series(vals, index=names)
    pick = rng.permutation(500)[:320]
    prior = pd.Series(rng.integers(-2, 3, 320).astype(np.float32), index=[names[i] for i in pick])
    prior.iloc[::17] = np.nan
    for r in (ranks, pd.Series(rng.integers(1, 900, 500), index=names)):
        got = mu.signed_transform_single(r, prior)
        ref = orc.signed_transform_single(r, prior)
        assert list(got.index) == list(ref.index)
        np.testing.assert_array_equal(got.to_numpy(), ref.to_numpy())
        np.testing.assert_array_equal(np.signbit(got.to_numpy()), np.signbit(ref.to_numpy()))
        assert got.dtype == ref.dtype
    empty = mu.signed_transform_single(ranks, pd.Series([1.0], index=["absent"]))
    assert len(empty) == 0
