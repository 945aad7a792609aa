"""Rayleigh-Ritz stage alone (rr_band_top, Sturm or reducing form via N2V2R_RR) on a synthetic
arrow + band matrix of the Krylov-Schur shape; run under rocprofv3 --kernel-trace --stats for
per-kernel times.

    python tools/rr_probe.py [c] [kp] [reps]"""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from node2vec2rank_amd import _lib  # noqa: E402
from test_gpu_parity import _band_problem  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 384
kp = int(sys.argv[2]) if len(sys.argv) > 2 else 80
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
eng = _lib.Engine(0)
H, hband, theta = _band_problem(c, kp, seed=c + kp, decoupled=kp // 2)
if kp:  # kept Ritz values slightly below the new eigenvalues, as in a converging cycle
    w_all = np.sort(np.linalg.eigvalsh(H))[::-1]
    theta = w_all[:kp] - 1e-9 * np.abs(w_all[:kp])
p = kp if kp else 80
for _ in range(reps):
    w, S = eng.rr_band_top(hband, c, kp, theta, p)
ref = np.sort(np.linalg.eigvalsh(H))[::-1][:p]
print(f"c {c} kp {kp} p {p}: max |w - eig| / |eig|_max = {np.abs(w - ref).max() / np.abs(ref).max():.2e}")
