import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from node2vec2rank_amd import _lib
eng = _lib.Engine(0)
for c in [64, 100, 128, 192, 255, 256, 257, 300, 384, 448, 500, 511, 512, 513, 600, 640, 641, 700, 760, 767, 768]:
    rng = np.random.default_rng(c)
    A = rng.standard_normal((c, c)); H = A + A.T
    p = 20
    errs = []
    for rep in range(3):
        w, S = eng.rr_top(H, p)
        ref = np.sort(np.linalg.eigvalsh(H))[::-1][:p]
        errs.append(np.abs(w - ref).max() / ref[0])
    print(c, " ".join(f"{e:.2e}" for e in errs), flush=True)
