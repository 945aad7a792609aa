"""Probe: the solver's paired-panel mode (two b = 8 blocks per SpMM application as one N x 16
panel) against the 8-wide fit on the same ER graph: block applications, cycles, fit time, SpMM
time, residuals, singular values of the two fits, and host fp64 residuals of a few pair-mode
vectors.  One JSON line per fit.
Usage: python tools/probe_pair.py N DEG D [reps] [modes, e.g. 8,16]"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1])
deg = float(sys.argv[2])
d = int(sys.argv[3])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
modes = [int(m) for m in (sys.argv[5] if len(sys.argv) > 5 else "8,16").split(",")]
t = time.time()
layers = (synthetic.er_layers(n, deg, 2, seed_base=1000) if n <= 2_000_000 else
          [synthetic.er_layer_rows(n, deg, 1000 + k) for k in range(2)])
print(json.dumps({"graph_s": round(time.time() - t, 1), "nnz": int(sum(a.nnz for a in layers))}),
      flush=True)
eng = _lib.Engine(0)
eng.set_layers(layers)
ref = {}
for mode in modes:
    flags = _lib.EIG_TIME_SPMM | (_lib.EIG_PANEL16 if mode == 16 else _lib.EIG_PANEL8)
    for r in range(reps):
        t = time.time()
        st = eng.uase(d, seed=42, solver_flags=flags, raise_on_no_convergence=False)
        wall = time.time() - t
        s = eng.singular_values()
        out = {"mode": mode, "rep": r, "panel": st["panel"], "wall_ms": round(wall * 1e3, 1),
               "apps": st["block_applications"], "cycles": st["restarts"],
               "basis": st["basis"], "converged": st["converged"],
               "max_res": st["max_residual"], "stagnated": st["stagnated"],
               "spmm_ms": [round(x, 1) for x in st["gpu_ms_spmm"]],
               "spmm_launches": st["spmm_timed_launches"],
               "lean_checks": st["lean_checks"], "est_scale": round(st["est_scale"], 3),
               "tri_fallbacks": st["tri_fallbacks"]}
        if r == reps - 1:
            ref[mode] = s
            if mode != modes[0]:
                out["sigma_rel_vs_first"] = float(np.max(np.abs(s - ref[modes[0]]) / ref[modes[0]]))
            if n <= 2_000_000:
                U = eng.left_embedding() / np.sqrt(s)[None, :].astype(np.float32)
                cols = sorted({0, d // 2, d - 1})
                X = U[:, cols].astype(np.float64)
                MX = np.zeros_like(X)
                for A in layers:
                    A64 = A.astype(np.float64).tocsr()
                    MX += A64 @ (A64.T @ X)
                th = s.astype(np.float64) ** 2
                R = MX - X * th[cols][None, :]
                out["host_res"] = [float(v) for v in np.linalg.norm(R, axis=0) / th[0]]
                out["orth"] = float(np.abs(U.T.astype(np.float64) @ U - np.eye(d)).max())
        print(json.dumps(out), flush=True)
eng.close()
