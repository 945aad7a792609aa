"""A/B probe: BASELINE cfg3 fits (dense |corr| layers, N = 20k, K = 4, d = 256) with the dense
SpMM's stored-matrix stream loaded plainly or non-temporally (N2V2R_DENSE_NT, read per launch),
alternating on one box: fit wall time, applications, residual."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
layers = synthetic.corr_layers(20_000, 4)
eng = _lib.Engine(0)
eng.set_layers(layers, storage="dense", symmetric=1)
eng.uase(256, seed=42)  # warm-up
for r in range(reps):
    for form in ("0", "1"):
        os.environ["N2V2R_DENSE_NT"] = form
        t = time.perf_counter()
        st = eng.uase(256, seed=42)
        eng.synchronize()
        print(json.dumps({"nt": form, "rep": r, "fit_ms": round((time.perf_counter() - t) * 1e3, 1),
                          "apps": st["block_applications"], "res": st["max_residual"]}),
              flush=True)
eng.close()
