"""Uninitialised-read guard (needs an MI355X): one child process with every new allocation and,
at every fit, the eigensolver's scratch filled with NaN bytes (N2V2R_POISON=1) and every solver
stage checked for non-finite output (N2V2R_DEBUG_FINITE=1).  A kernel that reads something it
did not write during the fit turns the fit non-finite and the check names the stage.  The
switches are read once per process, hence the child."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, "tests")
from conftest import fixture_layers, load_fixture
from node2vec2rank_amd import _lib, synthetic
eng = _lib.Engine(0)
for name in ["er_cfg1", "directed_weighted", "demo"]:
    fx = load_fixture(name)
    layers = fixture_layers(fx)
    d = int(fx["dims"].max())
    for block in [8, 16, 64]:
        eng.set_layers(layers)
        eng.uase(d, seed=int(fx["seed"]), block=block)
        s = eng.singular_values()
        assert np.allclose(s, fx["sigma"], rtol=2e-5), (name, block, s, fx["sigma"])
        ncmp, ncols = eng.rank("sequential", [2, d], ["cosine", "euclidean"])
        assert np.isfinite(eng.distances(0)).all()
# a second, larger graph in the same process: the workspace now holds another fit's state
layers = synthetic.er_layers(20_000, 20, 2)
eng.set_layers(layers)
st = eng.uase(32, seed=42)
assert st["converged"] == 32, st
print("POISON_OK")
"""


def test_fits_with_poisoned_scratch():
    env = dict(os.environ, N2V2R_POISON="1", N2V2R_DEBUG_FINITE="1")
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "POISON_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
