"""Banded Rayleigh-Ritz microbenchmark: rr_band_top on a cfg2-shaped projected matrix
(c = 384, kp = 80, p = 88) REPS times; run under rocprofv3 --kernel-trace for per-kernel times."""
import sys
import time

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

from node2vec2rank_amd import _lib  # noqa: E402
from tests.test_gpu_parity import _band_problem  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 384
kp = int(sys.argv[2]) if len(sys.argv) > 2 else 80
p = int(sys.argv[3]) if len(sys.argv) > 3 else 88
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
eng = _lib.Engine(0)
H, hband, theta = _band_problem(c, kp, seed=7)
w, S = eng.rr_band_top(hband, c, kp, theta, p)
ref = np.sort(np.linalg.eigvalsh(H))[::-1][:p]
err = np.abs(w - ref).max() / np.abs(ref).max()
t0 = time.perf_counter()
for _ in range(reps):
    eng.rr_band_top(hband, c, kp, theta, p)
eng.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / reps
print(f"c={c} kp={kp} p={p} ms_per_call={ms:.3f} max_rel_eig_err={err:.2e}")
