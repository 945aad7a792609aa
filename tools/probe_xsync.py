"""A/B of the tiled SpMM's XCD phase alignment (N2V2R_SPMM_XSYNC = lag in phases; unset: off)
at cfg4: device time per stage launch (HIP events inside the fit) and fit wall time, the forms
alternated over several fits on one box.  Run with N2V2R_LIB pointing at the probe build."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
deg = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
forms = sys.argv[3].split(",") if len(sys.argv) > 3 else ["off", "0", "1", "2"]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
layers = synthetic.er_layers(n, deg, 2, seed_base=1000)
eng = _lib.Engine(0)
eng.set_layers(layers)
eng.uase(128, seed=42)  # warm-up (column blocks, workspace)
for r in range(reps):
    for f in forms:
        if f == "off":
            os.environ.pop("N2V2R_SPMM_XSYNC", None)
        else:
            os.environ["N2V2R_SPMM_XSYNC"] = f
        t0 = time.perf_counter()
        st = eng.uase(128, seed=42, solver_flags=_lib.EIG_TIME_SPMM)
        eng.synchronize()
        t = time.perf_counter() - t0
        ms = st["gpu_ms_spmm"]
        cnt = st["spmm_timed_launches"]
        print(json.dumps({"form": f, "rep": r, "fit_ms": round(t * 1e3, 1),
                          "stage_ms": [round(ms[j] / max(1, cnt[j]), 4) for j in range(2)],
                          "apps": st["block_applications"], "res": st["max_residual"]}),
              flush=True)
