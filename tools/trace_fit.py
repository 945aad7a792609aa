"""One UASE fit of a synthetic ER graph with the solver's per-cycle trace (N2V2R_TRACE=1 on
stderr) and the stats dict: convergence debugging on the GPU.

    N2V2R_TRACE=1 python tools/trace_fit.py N AVG_DEG D [seed_base=1000] [seed=42]
"""
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n, deg, d = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
sb = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
seed = int(sys.argv[5]) if len(sys.argv) > 5 else 42
layers = synthetic.er_layers(n, deg, 2, seed_base=sb)
eng = _lib.Engine(0)
eng.set_layers(layers)
t0 = time.time()
st = eng.uase(d, seed=seed, raise_on_no_convergence=False)
st["wall_s"] = round(time.time() - t0, 3)
print(json.dumps(st), flush=True)
