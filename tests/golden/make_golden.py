"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE itself.

Run in the survey container only (needs /root/reference; never runs on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONHASHSEED=0 python tests/golden/make_golden.py

The reference's ``node2vec2rank/model.py`` is imported unchanged.  Its UASE dependency
(``spectral_embedding``, un-vendored and unavailable offline, ``environment.yaml:19``) is
provided as an in-memory module restating ``UASE`` per SURVEY.md Appendix A
(hstack -> ``svds`` -> descending reorder -> sqrt scaling -> split into (K, N, d)).
``DataLoader`` is bypassed (its ``match_networks`` set-intersection makes node order depend on
PYTHONHASHSEED, ``preprocessing_utils.py:300-304``): graphs go to ``N2V2R`` directly, in file
order, after the reference's own ``network_transform`` with the demo config's defaults.

Each fixture holds the inputs (CSR per layer) and the reference's outputs: embeddings Y
(K, N, d_max), singular values, per comparison key the N x C float64 distance matrix with its
column names and the int64 Borda scores, and the DeDi ranking.  The script also checks that
``oracle/n2v2r_oracle.py`` (faithful mode) reproduces every output bit-exactly before writing.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import pandas as pd
import scipy.sparse as sp
from scipy.sparse.linalg import svds

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


def _uase_shim(As, d, **_kw):
    A = sp.hstack(As)
    u, s, vT = svds(A, d)
    o = np.argsort(s[::-1])
    S = np.sqrt(s[o])
    XA = u[:, o] @ np.diag(S)
    XB = vT.T[:, o] @ np.diag(S)
    K = len(As)
    n = As[0].shape[0]
    YA = np.zeros((K, n, d))
    for t in range(K):
        YA[t] = XB[n * t:n * (t + 1)]
    return XA, YA


def _import_reference():
    mod = types.ModuleType("spectral_embedding")
    mod.UASE = _uase_shim
    sys.modules["spectral_embedding"] = mod
    sys.path.insert(0, REF)
    from node2vec2rank.model import N2V2R  # noqa: E402
    from node2vec2rank.preprocessing_utils import network_transform  # noqa: E402
    return N2V2R, network_transform


def _run_reference(N2V2R, graphs, nodes, dims, metrics, strategy, seed):
    config = dict(embed_dimensions=list(dims), distance_metrics=list(metrics), seed=seed,
                  comp_strategy=strategy, verbose=-1, save_dir=None)
    model = N2V2R(graphs=graphs, nodes=nodes, config=config)
    ranks = model.fit_transform_rank()
    agg = model.aggregate_transform()
    dedi = model.degree_difference_ranking() if strategy == "sequential" else {}
    return model, ranks, agg, dedi


def _pack_case(name, layers, nodes, dims, metrics, strategies, seed, N2V2R):
    from oracle import n2v2r_oracle as orc
    out = {}
    for li, a in enumerate(layers):
        a = sp.csr_matrix(a, dtype=np.float32)
        a.sort_indices()
        out[f"layer{li}_indptr"] = a.indptr.astype(np.int64)
        out[f"layer{li}_indices"] = a.indices.astype(np.int32)
        out[f"layer{li}_data"] = a.data.astype(np.float32)
    out["num_layers"] = np.int64(len(layers))
    out["n"] = np.int64(layers[0].shape[0])
    out["nodes"] = np.asarray([str(x) for x in nodes])
    out["dims"] = np.asarray(dims, dtype=np.int64)
    out["metrics"] = np.asarray(metrics)
    out["strategies"] = np.asarray(strategies)
    out["seed"] = np.int64(seed)
    dense = [np.asarray(sp.csr_matrix(a).todense(), dtype=np.float32) for a in layers]
    for strategy in strategies:
        model, ranks, agg, dedi = _run_reference(N2V2R, dense, list(nodes), dims, metrics,
                                                 strategy, seed)
        if "Y" not in out:
            out["Y"] = np.asarray(model.node_embeddings, dtype=np.float64)
        # oracle (faithful) must match bit-exactly
        Yo, so, _ = orc.uase([sp.csc_matrix(g) for g in dense], max(dims), seed=seed)
        assert np.array_equal(Yo, out["Y"]), f"{name}: oracle UASE differs from reference"
        out["sigma"] = so
        od = orc.rank_distances(Yo, dims, metrics, strategy, faithful=True)
        for key, df in ranks.items():
            cols = list(df.columns)
            D = df.to_numpy(dtype=np.float64)
            ocols, oD = od[key]
            assert cols == ocols, (cols, ocols)
            assert np.array_equal(np.isnan(D), np.isnan(oD))
            assert np.array_equal(np.nan_to_num(D, nan=-1), np.nan_to_num(oD, nan=-1)), name
            b = agg[key]["borda_ranks"].to_numpy(dtype=np.int64)
            ob = orc.borda(D, faithful=True)
            assert np.array_equal(b, ob), f"{name}/{strategy}/{key}: oracle Borda differs"
            out[f"{strategy}/{key}/D"] = D
            out[f"{strategy}/{key}/cols"] = np.asarray(cols)
            out[f"{strategy}/{key}/borda"] = b
            out[f"{strategy}/{key}/borda_stable"] = orc.borda(D, faithful=False)
        out[f"{strategy}/keys"] = np.asarray(list(ranks.keys()))
        for key, df in dedi.items():
            out[f"dedi/{key}"] = df["DeDi"].to_numpy(dtype=np.float32)
            od_ = orc.degree_difference(dense)[key][0]
            assert np.array_equal(od_, out[f"dedi/{key}"])
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KB)")


def make_cfg2(N2V2R):
    """BASELINE cfg2 at its own size (2-layer ER N=100k, avg-deg 20, d=64, cosine + euclidean,
    sequential; the bench's rank-0 graph, synthetic.er_layers(..., seed_base=1000)).  Sparse
    layers go to the reference N2V2R directly (``csc_matrix(sparse)`` at model.py:53).  Y and
    the layers are not stored (100 MB / 16 MB): the test regenerates the layers and checks the
    fingerprint."""
    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    n, deg, seed = 100_000, 20.0, 42
    layers = synthetic.er_layers(n, deg, 2, seed_base=1000)
    nodes = list(range(n))
    config = dict(embed_dimensions=[64], distance_metrics=["cosine", "euclidean"], seed=seed,
                  comp_strategy="sequential", verbose=1, save_dir=None)
    model = N2V2R(graphs=[sp.csr_matrix(a) for a in layers], nodes=nodes, config=config)
    ranks = model.fit_transform_rank()
    agg = model.aggregate_transform()
    D = ranks["1"].to_numpy(dtype=np.float64)
    b = agg["1"]["borda_ranks"].to_numpy(dtype=np.int64)
    Yo, so, _ = orc.uase([sp.csc_matrix(g) for g in layers], 64, seed=seed)
    assert np.array_equal(Yo, np.asarray(model.node_embeddings)), "cfg2: oracle UASE differs"
    oD = orc.rank_distances(Yo, [64], ["cosine", "euclidean"], "sequential", faithful=True)["1"][1]
    assert np.array_equal(oD, D)
    assert np.array_equal(orc.borda(D, faithful=True), b), "cfg2: oracle Borda differs"
    out = {"n": np.int64(n), "avg_deg": np.float64(deg), "seed_base": np.int64(1000),
           "num_layers": np.int64(2), "checksum": synthetic.fingerprint(layers),
           "dims": np.asarray([64], dtype=np.int64),
           "metrics": np.asarray(["cosine", "euclidean"]),
           "strategies": np.asarray(["sequential"]), "seed": np.int64(seed), "sigma": so,
           "sequential/keys": np.asarray(["1"]), "sequential/1/D": D,
           "sequential/1/cols": np.asarray(list(ranks["1"].columns)),
           "sequential/1/borda": b, "sequential/1/borda_stable": orc.borda(D, faithful=False)}
    path = os.path.join(HERE, "er_cfg2.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KB)")


def make_cfg2_env(_N2V2R=None):
    """The reference's own seed-to-seed envelope at cfg2, added to er_cfg2.npz: the oracle
    (bit-exact with the reference's model.py on this graph, checked by make_cfg2) re-run from
    the ARPACK start vectors of seeds 43 and 44 against the reference's seed-42 outputs: the
    largest distance difference and the lowest Kendall tau / top-100 overlap of the Borda
    ranks."""
    from scipy.stats import kendalltau

    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    path = os.path.join(HERE, "er_cfg2.npz")
    z = np.load(path, allow_pickle=False)
    out = {k: z[k] for k in z.files}
    layers = synthetic.er_layers(int(out["n"]), float(out["avg_deg"]), 2,
                                 seed_base=int(out["seed_base"]))
    Dr, br = out["sequential/1/D"], out["sequential/1/borda"]
    top = lambda b: set(np.argsort(-b, kind="stable")[:100].tolist())  # noqa: E731
    derr, taus, tops = [], [], []
    for seed in (43, 44):
        Y, _, _ = orc.uase(layers, 64, seed=seed)
        D = orc.rank_distances(Y, [64], ["cosine", "euclidean"], "sequential",
                               faithful=True)["1"][1]
        b = orc.borda(D, faithful=True)
        derr.append(np.abs(D - Dr).max(axis=0))
        taus.append(kendalltau(b, br).statistic)
        tops.append(len(top(b) & top(br)))
        print(f"seed {seed}: distance diff {derr[-1]}, tau {taus[-1]:.6f}, top-100 {tops[-1]}")
    out["env_distance_per_col"] = np.max(np.asarray(derr), axis=0)
    out["env_tau"] = np.float64(min(taus))
    out["env_top100"] = np.int64(min(tops))
    np.savez_compressed(path, **out)
    print(f"wrote {path}")


def make_cfg4g(N2V2R):
    """The bench's own grid (BASELINE cfg4: d in {8,16,32,64,128} x {cosine, euclidean}, 10
    columns, sequential, seed 42) on a cfg4-family graph the reference can finish: 2-layer ER
    N = 100k, avg-deg 50 (synthetic.er_layers(..., seed_base=1000), the generator bench.py
    uses).  The reference model.py runs unchanged; the oracle must reproduce it bit-exactly.
    Stored: sigma (128), the N x 10 distance table with its column names, the reference's
    Borda (numpy quicksort ties) and the stable-order Borda.  Y and the layers are not stored
    (the test regenerates the layers and checks the fingerprint)."""
    import time

    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    n, deg, seed = 100_000, 50.0, 42
    dims, metrics = [8, 16, 32, 64, 128], ["cosine", "euclidean"]
    layers = synthetic.er_layers(n, deg, 2, seed_base=1000)
    config = dict(embed_dimensions=dims, distance_metrics=metrics, seed=seed,
                  comp_strategy="sequential", verbose=1, save_dir=None)
    t0 = time.time()
    model = N2V2R(graphs=[sp.csr_matrix(a) for a in layers], nodes=list(range(n)), config=config)
    ranks = model.fit_transform_rank()
    agg = model.aggregate_transform()
    print(f"reference fit + rank + Borda: {time.time() - t0:.1f} s")
    D = ranks["1"].to_numpy(dtype=np.float64)
    b = agg["1"]["borda_ranks"].to_numpy(dtype=np.int64)
    Yo, so, _ = orc.uase([sp.csc_matrix(g) for g in layers], 128, seed=seed)
    assert np.array_equal(Yo, np.asarray(model.node_embeddings)), "cfg4g: oracle UASE differs"
    oD = orc.rank_distances(Yo, dims, metrics, "sequential", faithful=True)["1"][1]
    assert np.array_equal(oD, D)
    assert np.array_equal(orc.borda(D, faithful=True), b), "cfg4g: oracle Borda differs"
    out = {"n": np.int64(n), "avg_deg": np.float64(deg), "seed_base": np.int64(1000),
           "num_layers": np.int64(2), "checksum": synthetic.fingerprint(layers),
           "dims": np.asarray(dims, dtype=np.int64), "metrics": np.asarray(metrics),
           "strategies": np.asarray(["sequential"]), "seed": np.int64(seed), "sigma": so,
           "sequential/keys": np.asarray(["1"]), "sequential/1/D": D,
           "sequential/1/cols": np.asarray(list(ranks["1"].columns)),
           "sequential/1/borda": b, "sequential/1/borda_stable": orc.borda(D, faithful=False)}
    path = os.path.join(HERE, "er_cfg4g.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KB)")


def make_cfg4g_env(_N2V2R=None):
    """The reference's seed-to-seed envelope on the er_cfg4g graph (as make_cfg2_env): the
    oracle, bit-exact with the reference there, re-run from the ARPACK start vectors of seeds 43
    and 44.  No sign alignment anywhere (cosine / euclidean are sign-invariant)."""
    _envelope("er_cfg4g.npz", (43, 44))


def _envelope(fname, seeds):
    from scipy.stats import kendalltau

    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    path = os.path.join(HERE, fname)
    z = np.load(path, allow_pickle=False)
    out = {k: z[k] for k in z.files}
    layers = synthetic.er_layers(int(out["n"]), float(out["avg_deg"]), int(out["num_layers"]),
                                 seed_base=int(out["seed_base"]))
    dims = [int(x) for x in out["dims"]]
    metrics = [str(x) for x in out["metrics"]]
    Dr, br = out["sequential/1/D"], out["sequential/1/borda"]
    top = lambda b: set(np.argsort(-b, kind="stable")[:100].tolist())  # noqa: E731
    derr, taus, tops = [], [], []
    for seed in seeds:
        Y, _, _ = orc.uase(layers, max(dims), seed=seed)
        D = orc.rank_distances(Y, dims, metrics, "sequential", faithful=True)["1"][1]
        b = orc.borda(D, faithful=True)
        derr.append(np.abs(D - Dr).max(axis=0))
        taus.append(kendalltau(b, br).statistic)
        tops.append(len(top(b) & top(br)))
        print(f"seed {seed}: distance diff {derr[-1]}, tau {taus[-1]:.6f}, top-100 {tops[-1]}")
    out["env_distance_per_col"] = np.max(np.asarray(derr), axis=0)
    out["env_tau"] = np.float64(min(taus))
    out["env_top100"] = np.int64(min(tops))
    np.savez_compressed(path, **out)
    print(f"wrote {path}")


def _rotation_design(n, rho, lam, th, ms, seed=0, iters=12):
    """Latent rows of a two-layer network whose UASE distances are known in closed form.

    Node i carries B complex coordinates z_ib = rho_b exp(1j phi_ib) (the 2-D blocks of an
    embedding of width 2B); in layer 2 block b is rotated by lam_b theta_i.  For every prefix of
    whole blocks, cosine = 1 - sum rho_b^2 cos(lam_b theta_i) / sum rho_b^2 and euclidean^2 =
    sum 4 rho_b^2 sin^2(lam_b theta_i / 2): strictly increasing in theta_i on [0, pi] when
    0 <= lam_b <= 1, so equally spaced theta gives every distance column a designed minimum gap.
    The phases phi are solved (Gauss-Newton from phi_ib = m_b 2 pi i / n) so that the stacked
    rows Z = [Y1; Y2] have Z^T Z block diagonal: the SVD of Z then only rotates inside each 2-D
    block, which leaves every whole-block prefix distance unchanged.  Returns Y1, Y2, theta."""
    rng = np.random.default_rng(seed)
    nb = len(rho)
    rho = np.asarray(rho, dtype=np.float64)
    lam = np.asarray(lam, dtype=np.float64)
    i = np.arange(n)
    alpha = 2 * np.pi * i / n
    theta = th[0] + (th[1] - th[0]) * (i + 0.5) / n
    ph = np.stack([m * alpha + rng.uniform(0, 2 * np.pi) for m in ms])
    rot = np.exp(1j * lam[:, None] * theta[None, :])
    pairs = [(b, c) for b in range(nb) for c in range(b + 1, nb)]

    def resid_jac(ph):
        z = rho[:, None] * np.exp(1j * ph)
        r, jac = [], []
        for b, c in pairs:
            # off-block Gram entries over both layers: sum z_b conj(z_c) (1 + rot_b conj(rot_c))
            # and sum z_b z_c (1 + rot_b rot_c), as complex numbers
            t1 = z[b] * np.conj(z[c]) * (1 + rot[b] * np.conj(rot[c]))
            t2 = z[b] * z[c] * (1 + rot[b] * rot[c])
            r += [t1.sum(), t2.sum()]
            j1 = np.zeros((nb, n), complex)
            j1[b], j1[c] = 1j * t1, -1j * t1
            j2 = np.zeros((nb, n), complex)
            j2[b], j2[c] = 1j * t2, 1j * t2
            jac += [j1.ravel(), j2.ravel()]
        r, jac = np.asarray(r), np.asarray(jac)
        return np.concatenate([r.real, r.imag]), np.vstack([jac.real, jac.imag])

    for _ in range(iters):
        r, jac = resid_jac(ph)
        if np.abs(r).max() < 1e-13 * n:
            break
        ph = ph + np.linalg.lstsq(jac, -r, rcond=None)[0].reshape(nb, n)
    z = rho[:, None] * np.exp(1j * ph)
    w = z * rot
    rows = lambda c: np.stack([c.real, c.imag], axis=2).transpose(1, 0, 2).reshape(n, 2 * nb)  # noqa: E731
    return rows(z), rows(w), theta


def make_lowrank_exact(N2V2R):
    """SURVEY 8(c)(4)'s end-to-end clause: integer ranks bit-exact on a tie-free fixture whose
    sorted distance columns have every adjacent gap >= 1e-4.

    Why not a sampled SBM: the distances of a random graph are random, so with N values in a
    range L about N^2 g / L adjacent gaps fall below g (birthday bound) -- 300 seeds of a
    4-community, 120-node SBM gave a best smallest gap of 5e-6, and N = 1-2k is hopeless.  The
    fixture is therefore a weighted directed two-layer network (dense float32, both signs, as a
    co-expression network) of rank 8 built from a prescribed SVD: right singular vectors from
    _rotation_design (every node rotates, by its own angle, in layer 2: no unchanged nodes),
    singular values 1086 .. 268 (four 2-D blocks, ratio >= 1.5 between blocks), random
    orthonormal left vectors, nodes relabelled by a random permutation.  The reference model.py
    runs on it unchanged; the script asserts the oracle reproduces it bit-exactly and that every
    sorted column of the REFERENCE's distance table has adjacent gaps >= 1e-4.  Stored: the
    factors (the test regenerates the float32 layers with synthetic.lowrank_layers and checks
    their SHA-256), the reference's sigma, Y, distance table, column names and Borda."""
    import hashlib

    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    n, d, seed = 2000, 8, 42
    dims, metrics = [2, 4, 6, 8], ["cosine", "euclidean"]
    y1, y2, theta = _rotation_design(n, (1.0, 0.8, 0.64, 0.512), (1.0, 0.5, 0.25, 0.0),
                                     (0.4, 2.7), (1, 3, 7, 12))
    zst = np.vstack([y1, y2])
    p, s, _ = np.linalg.svd(zst, full_matrices=False)
    u, _ = np.linalg.qr(np.random.default_rng(7).standard_normal((n, d)))
    perm = np.random.default_rng(3).permutation(n)
    us = (u * (s ** 2)[None, :])[perm]
    right = [p[:n][perm], p[n:][perm]]
    layers = synthetic.lowrank_layers(us, right)
    nodes = [f"v{int(x):04d}" for x in np.random.default_rng(5).permutation(n)]
    model, ranks, agg, _ = _run_reference(N2V2R, layers, nodes, dims, metrics, "sequential", seed)
    Y = np.asarray(model.node_embeddings, dtype=np.float64)
    Yo, so, _ = orc.uase([sp.csc_matrix(g) for g in layers], d, seed=seed)
    assert np.array_equal(Yo, Y), "lowrank_exact: oracle UASE differs from reference"
    D = ranks["1"].to_numpy(dtype=np.float64)
    cols = list(ranks["1"].columns)
    oc, oD = orc.rank_distances(Yo, dims, metrics, "sequential", faithful=True)["1"]
    assert cols == oc and np.array_equal(oD, D)
    b = agg["1"]["borda_ranks"].to_numpy(dtype=np.int64)
    assert np.array_equal(orc.borda(D, faithful=True), b)
    gaps = np.array([np.diff(np.sort(D[:, c])).min() for c in range(D.shape[1])])
    print("lowrank_exact: smallest adjacent gap per column", gaps)
    assert gaps.min() >= 1e-4, gaps
    # the design's closed form holds (monotone in the rotation angle theta[perm])
    o = np.argsort(theta[perm])
    assert np.all(np.diff(D[o], axis=0) > 0)
    assert np.array_equal(orc.borda(D, faithful=False), b)  # tie-free: any correct sort agrees
    out = {"n": np.int64(n), "num_layers": np.int64(2), "us": us, "right0": right[0],
           "right1": right[1],
           "sha256": np.asarray([hashlib.sha256(a.tobytes()).hexdigest() for a in layers]),
           "nodes": np.asarray(nodes), "dims": np.asarray(dims, dtype=np.int64),
           "metrics": np.asarray(metrics), "strategies": np.asarray(["sequential"]),
           "seed": np.int64(seed), "sigma": so, "Y": Y, "min_gap": gaps,
           "sequential/keys": np.asarray(["1"]), "sequential/1/D": D,
           "sequential/1/cols": np.asarray(cols), "sequential/1/borda": b}
    path = os.path.join(HERE, "lowrank_exact.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KB)")


def make_writer(N2V2R):
    """The reference's output files (model.py:40-48 config.json, :142-145 {key}.tsv,
    :193-196 {key}_agg.tsv, :306-309 {key}_degDif.tsv, :269-278 {key}_signed.tsv and
    {key}_agg_signed.tsv) for the er_cfg1 graphs, written with save_dir="out" from inside a
    scratch directory (so config.json holds the relative path) and the timestamp directory
    renamed away.  Copied byte for byte into tests/golden/writer_er_cfg1/."""
    import glob
    import shutil
    import tempfile
    from node2vec2rank_amd import synthetic
    layers = [synthetic.er_layer_p(1000, 0.01, 1000 + k) for k in range(2)]
    dense = [np.asarray(a.todense(), dtype=np.float32) for a in layers]
    nodes = [f"g{i}" for i in range(1000)]
    dst = os.path.join(HERE, "writer_er_cfg1")
    os.makedirs(dst, exist_ok=True)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            config = dict(embed_dimensions=[2, 8], distance_metrics=["cosine", "euclidean"],
                          seed=42, comp_strategy="sequential", verbose=-1, save_dir="out")
            model = N2V2R(graphs=dense, nodes=nodes, config=config)
            model.fit_transform_rank()
            model.aggregate_transform()
            model.degree_difference_ranking()
            model.signed_ranks_transform()
            (run,) = glob.glob(os.path.join(tmp, "out", "*"))
            for f in sorted(os.listdir(run)):
                shutil.copyfile(os.path.join(run, f), os.path.join(dst, f))
                print(f"wrote {os.path.join(dst, f)}")
        finally:
            os.chdir(cwd)


def main():
    N2V2R, network_transform = _import_reference()
    from node2vec2rank_amd import synthetic
    only = sys.argv[1:]
    if only:
        for name in only:
            {"er_cfg2": make_cfg2, "er_cfg2_env": make_cfg2_env,
             "er_cfg4g": make_cfg4g, "er_cfg4g_env": make_cfg4g_env,
             "lowrank_exact": make_lowrank_exact, "writer": make_writer}[name](N2V2R)
        return

    # 1. the reference's demo graphs (data/networks/demo, configs/config_demo_adj.json)
    demo_dir = os.path.join(REF, "data", "networks", "demo")
    g = [pd.read_csv(os.path.join(demo_dir, f), index_col=0, header=0, sep=",")
         for f in ("adj_matrix_1.csv", "adj_matrix_2.csv")]
    nodes = list(g[0].columns)
    g = [network_transform(x, threshold=None, top_percent_keep=100, binarize=False,
                           absolute=False, project_unipartite_on=None) for x in g]
    comm = pd.read_csv(os.path.join(demo_dir, "comm_asiggnments.csv"), index_col=0, header=0)
    _pack_case("demo", [sp.csr_matrix(x) for x in g], nodes, list(range(4, 25, 2)),
               ["euclidean", "cosine"], ["sequential"], 42, N2V2R)
    np.save(os.path.join(HERE, "demo_communities.npy"), comm["0"].to_numpy(dtype=np.int64))

    # 2. BASELINE cfg1: 2-layer ER N=1000, p=0.01, d=8
    layers = [synthetic.er_layer_p(1000, 0.01, 1000 + k) for k in range(2)]
    _pack_case("er_cfg1", layers, list(range(1000)), [8], ["cosine", "euclidean"],
               ["sequential"], 42, N2V2R)

    # 3. K=4, all three strategies, dim 1 (cosine skipped) and correlation
    layers, _ = synthetic.sbm_layers(400, 4, seed=3)
    _pack_case("k4_strategies", layers, list(range(400)), [1, 2, 4, 6],
               ["cosine", "euclidean", "correlation"],
               ["sequential", "one_vs_before", "one_vs_rest"], 7, N2V2R)

    # 4. ties (planted unchanged nodes) + NaN cosine (a node isolated in layer 2)
    rng = np.random.default_rng(11)
    a1 = synthetic.er_layer(300, 12, 21).toarray()
    a2 = synthetic.er_layer(300, 12, 22).toarray()
    same = rng.choice(300, size=20, replace=False)
    a2[same, :] = a1[same, :]
    a2[:, same] = a1[:, same]
    a2[5, :] = 0
    a2[:, 5] = 0
    _pack_case("ties_nan", [sp.csr_matrix(a1), sp.csr_matrix(a2)], list(range(300)),
               [2, 4, 8], ["cosine", "euclidean"], ["sequential"], 42, N2V2R)

    # 5. directed, weighted layers (exercises A_k^T and non-binary values)
    rng = np.random.default_rng(5)
    lay = []
    for k in range(3):
        m = (rng.random((250, 250)) < 0.05).astype(np.float32)
        np.fill_diagonal(m, 0)
        m *= rng.random((250, 250)).astype(np.float32) + 0.5
        lay.append(sp.csr_matrix(m))
    _pack_case("directed_weighted", lay, list(range(250)), [3, 5, 10],
               ["cosine", "euclidean"], ["sequential", "one_vs_rest"], 123, N2V2R)


if __name__ == "__main__":
    main()
