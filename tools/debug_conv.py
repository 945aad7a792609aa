"""Convergence probe: UASE stats on ER graphs (no raise) for the current build."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from node2vec2rank_amd import _lib, synthetic
eng = _lib.Engine(0)
cases = [(2000, 20, 8), (5000, 20, 8), (20000, 20, 8), (20000, 20, 32), (20000, 5, 32),
         (100000, 20, 64), (50000, 20, 32)]
for n, deg, d in cases:
    layers = synthetic.er_layers(n, deg, 2)
    eng.set_layers(layers)
    for blk in (8, 16):
        for keep, mb in ((0, 0), (d + 24 if d > 8 else 0, 0)):
            st = eng.uase(d, seed=42, block=blk, keep=keep, max_basis=mb, max_restarts=200,
                          raise_on_no_convergence=False)
            print(n, deg, d, blk, keep, json.dumps({k: st[k] for k in ("restarts", "block_applications", "converged", "max_residual", "stagnated", "basis")}), flush=True)
