"""Timing experiment: cfg2 fits with a fixed cycle count (7), to compare kernel times with and
without N2V2R_EXPERIMENT_W2 under rocprofv3 (results of the W2 run are invalid)."""
import sys
sys.path.insert(0, ".")
from node2vec2rank_amd import _lib, synthetic  # noqa: E402
eng = _lib.Engine(0)
eng.set_layers(synthetic.er_layers(100_000, 20.0, 2, seed_base=1000))
for _ in range(3):
    st = eng.uase(64, seed=42, max_restarts=7, raise_on_no_convergence=False)
print(st["block_applications"], st["restarts"])
