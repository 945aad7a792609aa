"""Convergence vs (keep, max_basis) on an ER graph: python tools/sweep_big.py N deg d '[[keep,c],...]' [max_restarts] [seed_base]"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from node2vec2rank_amd import _lib, synthetic
n, deg, d = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
cases = json.loads(sys.argv[4])
mr = int(sys.argv[5]) if len(sys.argv) > 5 else 60
sb = int(sys.argv[6]) if len(sys.argv) > 6 else 2000
eng = _lib.Engine(0)
layers = [synthetic.er_layer_rows(n, deg, sb + k) for k in range(2)]
eng.set_layers(layers, symmetric=1)
del layers
for keep, c in cases:
    t = time.time()
    st = eng.uase(d, seed=42, keep=keep, max_basis=c, max_restarts=mr, raise_on_no_convergence=False)
    print(json.dumps({"n": n, "deg": deg, "d": d, "seed_base": sb, "keep": keep, "c": c, "s": round(time.time() - t, 2), **{k: st[k] for k in ("restarts", "block_applications", "converged", "max_residual", "stagnated")}}), flush=True)
