"""Diagnose a Rayleigh-Ritz stage failure: run rr_band_top on the test's structured matrix and
compare the eigenvalues / vectors with numpy even when the residual check fails."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from node2vec2rank_amd import _lib  # noqa: E402
from test_gpu_parity import _band_problem  # noqa: E402

c, kp, p = (int(x) for x in sys.argv[1:4])
eng = _lib.Engine(0)
H, hband, theta = _band_problem(c, kp, seed=c + kp)
w = np.zeros(p)
S = np.zeros((c, p), np.float32)
th = np.zeros(max(c, 1)) if theta is None else np.ascontiguousarray(theta, dtype=np.float64)
st = eng.lib.n2v2r_rr_band_top(eng.h, c, kp, np.ascontiguousarray(hband), hband.size,
                               th.ctypes.data, p, w, S)
ref = np.sort(np.linalg.eigvalsh(H))[::-1][:p]
print("status", st, eng._err() if st else "")
err = np.abs(w - ref)
print("max eig err / scale", err.max() / np.abs(ref).max(), "at", int(err.argmax()))
bad = np.where(err > 1e-9 * np.abs(ref).max())[0]
print("bad eigen indices", bad[:20], "count", len(bad))
for j in bad[:5]:
    print(j, w[j], ref[j], ref[max(j-1,0)], ref[min(j+1,p-1)])
S = S.astype(np.float64)
R = np.linalg.norm(H @ S - S * w, axis=0)
print("worst residual cols", np.argsort(R)[::-1][:5], np.sort(R)[::-1][:5])
