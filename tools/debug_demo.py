import sys, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from conftest import load_fixture, fixture_layers
from oracle import n2v2r_oracle as orc
from node2vec2rank_amd import _lib
for name in ['demo', 'er_cfg1']:
    fx = load_fixture(name); layers = fixture_layers(fx); d = int(fx['dims'].max())
    e = _lib.Engine(0); e.set_layers(layers)
    for ov in (-1, 0, 2):
        for tol in (1e-6, 1e-7):
            try:
                st = e.uase(d, seed=42, overlap=ov, tol=tol)
            except Exception as ex:
                print(name, ov, tol, 'ERR', ex); continue
            s = e.singular_values()
            print(name, ov, tol, 'sig rel err %.2e' % (np.abs(s - fx['sigma']) / fx['sigma']).max(),
                  {k: st[k] for k in ('restarts', 'block_applications', 'max_residual', 'stagnated', 'ms_total')})
