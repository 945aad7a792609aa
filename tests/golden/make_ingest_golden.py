"""Golden outputs of the reference's DataLoader for the ingest tests (tests/test_ingest.py).

Run in the survey container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ingest_golden.py [case ...]

Imports the reference's ``node2vec2rank/dataloader.py`` unchanged and loads the files in
``tests/golden/ingest_inputs/`` (the reference's own ``input/`` fixtures, copied as data, plus
small bipartite / duplicate-edge files written for this test) under a set of configs.  For
each case the npz holds the dense float32 layers, the node labels, and the row / column label
order of the layers (recorded by wrapping ``match_networks``; the reference orders labels by
hashing, ``preprocessing_utils.py:300-301``, and for a table whose index parses as integers
while its header stays text the two orders differ), so the tests compare label by label.
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
INPUTS = os.path.join(HERE, "ingest_inputs")
REF = "/root/reference"

BASE = {"data_dir": INPUTS, "transpose": False, "project_unipartite_on": None, "threshold": None,
        "top_percent_keep": 100, "binarize": False, "absolute": False}

CASES = {
    "named_edges": dict(graph_filenames=["test1_named.edgelist", "test2_named.edgelist"],
                        separator=" ", is_edge_list=True),
    "numeric_edges": dict(graph_filenames=["test1.edgelist", "test2.edgelist"], separator=" ",
                          is_edge_list=True),
    "dup_edges": dict(graph_filenames=["dups.edgelist", "dups2.edgelist"], separator=" ",
                      is_edge_list=True),
    "adj_csv": dict(graph_filenames=["test1.csv", "test2.csv"], separator=",",
                    is_edge_list=False),
    "sbm_txt": dict(graph_filenames=["sbm1.txt", "sbm2.txt"], separator=",", is_edge_list=False),
    "named_edges_top50_bin": dict(graph_filenames=["test1_named.edgelist",
                                                   "test2_named.edgelist"],
                                  separator=" ", is_edge_list=True, top_percent_keep=50,
                                  binarize=True),
    "named_edges_thresh": dict(graph_filenames=["test1_named.edgelist", "test2_named.edgelist"],
                               separator=" ", is_edge_list=True, threshold=3.0),
    # fractional percentages go to np.percentile unchanged (dataloader.py:74)
    # (37.5 and 62.5 keep more edges of dups.edgelist than 37 and 62 would)
    "dup_edges_top37p5": dict(graph_filenames=["dups.edgelist", "dups2.edgelist"], separator=" ",
                              is_edge_list=True, top_percent_keep=37.5),
    "dup_edges_top62p5_bin": dict(graph_filenames=["dups.edgelist", "dups2.edgelist"],
                                  separator=" ", is_edge_list=True, top_percent_keep=62.5,
                                  binarize=True),
    "bip_columns_abs_top30": dict(graph_filenames=["bip1.csv", "bip2.csv"], separator=",",
                                  is_edge_list=False, absolute=True, top_percent_keep=30,
                                  project_unipartite_on="columns"),
    "bip_rows_thresh": dict(graph_filenames=["bip1.csv", "bip2.csv"], separator=",",
                            is_edge_list=False, threshold=0.1,
                            project_unipartite_on="rows"),
    "bip_transpose_rows": dict(graph_filenames=["bip1.csv", "bip2.csv"], separator=",",
                               is_edge_list=False, transpose=True, absolute=True,
                               project_unipartite_on="rows"),
}


def main():
    sys.path.insert(0, REF)
    import node2vec2rank.dataloader as dlmod  # noqa: E402
    from node2vec2rank.dataloader import DataLoader  # noqa: E402
    seen = {}
    original = dlmod.match_networks

    def recording_match(graphs):  # observe (not alter) the reference's row/column label order
        out = original(graphs)
        seen["rows"] = [str(x) for x in out[0].index]
        seen["cols"] = [str(x) for x in out[0].columns]
        return out

    dlmod.match_networks = recording_match
    only = set(sys.argv[1:])  # optional case names: regenerate just those
    for name, case in CASES.items():
        if only and name not in only:
            continue
        cfg = dict(BASE, **case)
        cfg_out = {k: v for k, v in cfg.items() if k != "data_dir"}
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                dl = DataLoader(cfg)
        except Exception as e:  # the reference's own failure mode is part of the contract
            np.savez_compressed(os.path.join(HERE, f"ingest_{name}.npz"),
                                error=np.asarray(type(e).__name__),
                                config=np.asarray(json.dumps(cfg_out)))
            print(name, "raises", type(e).__name__)
            continue
        graphs = np.stack([np.asarray(g, dtype=np.float32) for g in dl.get_graphs()])
        nodes = np.asarray([str(x) for x in dl.get_nodes()])
        proj = cfg.get("project_unipartite_on")
        rows = seen["cols"] if proj == "columns" else seen["rows"]
        cols = seen["rows"] if proj == "rows" else seen["cols"]
        np.savez_compressed(os.path.join(HERE, f"ingest_{name}.npz"), graphs=graphs,
                            nodes=nodes, rows=np.asarray(rows), cols=np.asarray(cols),
                            config=np.asarray(json.dumps(cfg_out)))
        print(name, graphs.shape)


if __name__ == "__main__":
    main()
