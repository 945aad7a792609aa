"""Selective reorthogonalisation probe on the bench workload (cfg2 by default): for each
N2V2R_REORTH_TOL value, one warm fit's wall time, block applications, true max residual,
orthonormality of U and the singular values against the always-reorthogonalising fit.

    python tools/reorth_probe.py [config] tol1 tol2 ...      (tol 0 = every full pass runs)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1][0].isdigit() else "cfg2"
tols = [a for a in sys.argv[1:] if a[0].isdigit()] or ["0", "1e-6", "1e-5", "1e-4"]
cfg = bench.CONFIGS[cfg_name]
eng = _lib.Engine(0)
eng.set_layers(synthetic.er_layers(cfg["n"], cfg["avg_deg"], 2, seed_base=1000))
d = cfg["d"]
flags = int(os.environ.get("PROBE_FLAGS", "0"))
base = None
for t in tols:
    os.environ["N2V2R_REORTH_TOL"] = t
    try:
        eng.uase(d, seed=42, solver_flags=flags)  # warm
    except _lib.ArpackNoConvergence as e:
        print(f"tol {t:>6s}: {e}", flush=True)
        continue
    eng.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        st = eng.uase(d, seed=42, solver_flags=flags)
    eng.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    s = eng.singular_values().astype(np.float64)
    U = eng.left_embedding().astype(np.float64) / np.sqrt(s)[None, :]
    orth = np.abs(U.T @ U - np.eye(d)).max()
    if base is None:
        base = s
    print(f"tol {t:>6s}: {ms:7.2f} ms/fit  apps {st['block_applications']:4d}  max_res "
          f"{st['max_residual']:.2e}  conv {st['converged']}/{d}  |U^T U - I| {orth:.1e}  "
          f"max|ds|/s {np.abs(s - base).max() / s[0]:.1e}", flush=True)
