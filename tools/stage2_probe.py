"""Time the b = 8 second SpMM stage W = sum_k A_k Z_k three ways (summed output; one output per
layer; one output per layer with the layers split over the XCDs) on ER layers.

    python tools/stage2_probe.py [n] [deg]"""
import sys

sys.path.insert(0, ".")
from node2vec2rank_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
deg = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
eng = _lib.Engine(0)
eng.set_layers(synthetic.er_layers(n, deg, 2))
for rep in range(2):
    t = [eng.probe_spmm_stage2(m, reps=100) * 1e3 for m in (0, 1, 2, 3, 4)]
    print(f"n {n} deg {deg}: stage 2 summed {t[0]:.2f} us  per-layer {t[1]:.2f} us  "
          f"xcd-split {t[2]:.2f} us | shared panel (stage 1): per-layer {t[3]:.2f} us  "
          f"xcd-split {t[4]:.2f} us", flush=True)
