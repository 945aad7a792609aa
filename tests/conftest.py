import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")
FIXTURES = ["demo", "er_cfg1", "k4_strategies", "ties_nan", "directed_weighted"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def load_fixture(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def fixture_layers(fx):
    import scipy.sparse as sp
    n = int(fx["n"])
    out = []
    for k in range(int(fx["num_layers"])):
        out.append(sp.csr_matrix((fx[f"layer{k}_data"], fx[f"layer{k}_indices"],
                                  fx[f"layer{k}_indptr"]), shape=(n, n)))
    return out


@pytest.fixture(scope="session")
def engine():
    from node2vec2rank_amd import _lib
    return _lib.Engine(0)
