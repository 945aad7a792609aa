"""A/B probe of a solver switch read per fit: cfg4-shaped fits (2-layer ER, N and degree from
argv, d = 128) alternating the values of one environment variable on one engine.
Usage: python tools/probe_env_ab.py N DEG VAR v1,v2,... [reps]   ("-" = unset)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n, deg, var = int(sys.argv[1]), float(sys.argv[2]), sys.argv[3]
vals = sys.argv[4].split(",")
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 2
d = int(os.environ.get("PROBE_D", "128"))
layers = (synthetic.er_layers(n, deg, 2, seed_base=1000) if n <= 2_000_000 else
          [synthetic.er_layer_rows(n, deg, 1000 + k) for k in range(2)])
eng = _lib.Engine(0)
eng.set_layers(layers)
eng.uase(d, seed=42)  # warm-up (workspace, column blocks)
for r in range(reps):
    for v in vals:
        if v == "-":
            os.environ.pop(var, None)
        else:
            os.environ[var] = v
        t = time.perf_counter()
        st = eng.uase(d, seed=42, raise_on_no_convergence=False)
        eng.synchronize()
        print(json.dumps({var: v, "rep": r, "fit_ms": round((time.perf_counter() - t) * 1e3, 1),
                          "apps": st["block_applications"], "restarts": st["restarts"],
                          "converged": st["converged"], "res": st["max_residual"],
                          "stagnated": st["stagnated"]}), flush=True)
eng.close()
