"""Repeat UASE at block 8/16/64 on the test fixtures in one process and report any run whose
residual check fails (hunting an intermittent non-convergence at block 16)."""
import sys
import time

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

from conftest import fixture_layers, load_fixture  # noqa: E402
from node2vec2rank_amd import _lib  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
eng = _lib.Engine(0)
bad = 0
t0 = time.time()
for rep in range(reps):
    for name in ["er_cfg1", "directed_weighted", "demo"]:
        fx = load_fixture(name)
        layers = fixture_layers(fx)
        d = int(fx["dims"].max())
        for block in [8, 16, 64]:
            eng.set_layers(layers)
            try:
                eng.uase(d, seed=int(fx["seed"]), block=block)
                s = eng.singular_values()
                ok = np.all(np.isfinite(s)) and np.allclose(s, fx["sigma"], rtol=2e-5)
            except Exception as e:  # noqa: BLE001
                ok = False
                print(f"rep {rep} {name} b={block}: {e}", flush=True)
            if not ok:
                bad += 1
                print(f"rep {rep} {name} b={block}: FAIL", flush=True)
print(f"reps={reps} failures={bad} {time.time() - t0:.1f}s", flush=True)
