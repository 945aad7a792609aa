"""End-to-end rank agreement with the reference fixtures (GPU): Kendall tau and top-100 sets.

    python tools/parity_probe.py [fixture ...]  > gpurun_out/parity.json

For every fixture / strategy / comparison key: Kendall tau of the engine's Borda against the
reference's (its stable-order restatement on the reference distances, and the reference's own
quicksort Borda), the top-100 (or top-N/10) set overlap, and the reference's own envelope
(ARPACK start vector seed vs seed + 1).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from scipy.stats import kendalltau

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import FIXTURES, fixture_layers, load_fixture  # noqa: E402
from oracle import n2v2r_oracle as orc  # noqa: E402


def top_set(b, k):
    return set(np.argsort(-b, kind="stable")[:k].tolist())


def main():
    from node2vec2rank_amd.model import N2V2R
    names = sys.argv[1:] or FIXTURES + ["er_cfg2"]
    out = []
    for name in names:
        try:
            fx = load_fixture(name)
        except FileNotFoundError:
            continue
        if "layer0_indptr" in fx:
            layers = fixture_layers(fx)
        else:  # generator fixture (er_cfg2)
            from node2vec2rank_amd import synthetic
            layers = synthetic.er_layers(int(fx["n"]), float(fx["avg_deg"]),
                                         int(fx["num_layers"]), seed_base=int(fx["seed_base"]))
            fx["nodes"] = np.arange(int(fx["n"]))
        nodes = [str(x) for x in fx["nodes"]]
        dims = [int(x) for x in fx["dims"]]
        metrics = [str(x) for x in fx["metrics"]]
        d = max(dims)
        Yb = None
        if len(nodes) <= 20000:
            Yb, _, _ = orc.uase(layers, d, seed=int(fx["seed"]) + 1)
            Yb = orc.align_signs(Yb, fx["Y"]) if "Y" in fx else Yb
        for strategy in [str(x) for x in fx["strategies"]]:
            cfg = dict(embed_dimensions=dims, distance_metrics=metrics, seed=int(fx["seed"]),
                       comp_strategy=strategy, verbose=-1, save_dir=None)
            m = N2V2R(layers, nodes, cfg)
            m.fit_transform_rank()
            agg = m.aggregate_transform()
            for key in [str(k) for k in fx[f"{strategy}/keys"]]:
                b = agg[key]["borda_ranks"].to_numpy()
                Dref = fx[f"{strategy}/{key}/D"]
                ref_stable = orc.borda(Dref)
                ref_fast = fx[f"{strategy}/{key}/borda"]
                k = min(100, len(nodes) // 10)
                rec = dict(fixture=name, strategy=strategy, key=key, n=len(nodes),
                           tau_stable=float(kendalltau(b, ref_stable).statistic),
                           tau_reference=float(kendalltau(b, ref_fast).statistic),
                           top_k=k, top_overlap=len(top_set(b, k) & top_set(ref_fast, k)),
                           exact=bool(np.array_equal(b, ref_fast)),
                           d_err=float(np.nanmax(np.abs(m.pairwise_ranks[key].to_numpy() - Dref))))
                if Yb is not None:
                    Db = orc.rank_distances(Yb, dims, metrics, strategy, faithful=True)[key][1]
                    bb = orc.borda(Db)
                    rec["tau_env"] = float(kendalltau(bb, ref_stable).statistic)
                    rec["top_overlap_env"] = len(top_set(bb, k) & top_set(ref_fast, k))
                print(json.dumps(rec), flush=True)
                out.append(rec)


if __name__ == "__main__":
    main()
