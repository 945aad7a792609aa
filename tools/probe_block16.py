"""Probe: vector applications of the block Krylov-Schur fit at panel width 8 vs 16 (cfg4 shape:
2-layer ER N = 1M, degree 50, d = 128), over a few kept / basis sizes.  The b = 16 fits run the
generic (row-kernel, dense Rayleigh-Ritz) path: their times are not the question, their
application counts are."""
import json
import os
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
deg = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
d = int(sys.argv[3]) if len(sys.argv) > 3 else 128
combos = [(8, 0, 0), (16, 0, 0), (16, 0, 640), (16, 0, 768), (16, 192, 640), (16, 224, 768)]
if len(sys.argv) > 4:  # "b:keep:basis,..."
    combos = [tuple(int(v) for v in c.split(":")) for c in sys.argv[4].split(",")]
seed_base = int(os.environ.get("PROBE_SEED", "2000"))
layers = (synthetic.er_layers(n, deg, 2, seed_base=seed_base) if n <= 2_000_000 else
          [synthetic.er_layer_rows(n, deg, seed_base + k) for k in range(2)])
eng = _lib.Engine(0)
eng.set_layers(layers)
for b, keep, basis in combos:
    t = time.perf_counter()
    st = eng.uase(d, block=b, keep=keep, max_basis=basis, seed=42, raise_on_no_convergence=False)
    eng.synchronize()
    print(json.dumps({"b": b, "keep": keep, "basis": basis, "apps": st["block_applications"],
                      "vectors": st["block_applications"] * b, "restarts": st["restarts"],
                      "converged": st["converged"], "res": st["max_residual"],
                      "c": st["basis"], "s": round(time.perf_counter() - t, 2)}), flush=True)
eng.close()
