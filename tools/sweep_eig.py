"""GPU sweep of eigensolver parameters on a synthetic ER workload (design tool)."""
import json
import sys
import time

sys.path.insert(0, ".")
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 64
deg = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
configs = json.loads(sys.argv[4]) if len(sys.argv) > 4 else [
    [32, 288, 96], [16, 288, 96], [16, 256, 80], [8, 256, 80], [8, 192, 80], [16, 192, 80],
    [32, 384, 96], [16, 384, 96], [8, 320, 80], [64, 384, 128]]
eng = _lib.Engine(0)
eng.set_layers(synthetic.er_layers(n, deg, 2))
for cfgv in configs:
    b, mc, keep = cfgv[:3]
    fl = cfgv[3] if len(cfgv) > 3 else 0
    try:
        eng.uase(d, seed=42, block=b, max_basis=mc, keep=keep, solver_flags=fl)  # warm
        t = time.perf_counter()
        st = eng.uase(d, seed=42, block=b, max_basis=mc, keep=keep, solver_flags=fl)
        dt = time.perf_counter() - t
        print(json.dumps(dict(b=b, c=mc, keep=keep, flags=fl, ms=round(dt * 1e3, 1),
                              cycles=st["restarts"], blockapps=st["block_applications"],
                              vecapps=st["block_applications"] * b,
                              rr_ms=round(st["ms_rr_host"], 1), res=st["max_residual"])),
              flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps(dict(b=b, c=mc, keep=keep, error=str(e))), flush=True)
