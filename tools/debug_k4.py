import sys, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from conftest import load_fixture, fixture_layers
from oracle import n2v2r_oracle as orc
from node2vec2rank_amd import _lib
fx = load_fixture('k4_strategies'); layers = fixture_layers(fx)
dims=[int(x) for x in fx['dims']]; metrics=[str(x) for x in fx['metrics']]
e=_lib.Engine(0); e.set_layers(layers); st=e.uase(6, seed=7); print(st)
Y=e.embedding().astype(np.float64); Ya=orc.align_signs(Y, fx['Y'])
print('Yerr', np.abs(Ya-fx['Y']).max()/np.abs(fx['Y']).max())
e.rank('sequential', dims, metrics)
D=e.distances(0); Dref=fx['sequential/1/D']
Dy=orc.rank_distances(Y, dims, metrics, 'sequential')['1'][1]
cols=[str(c) for c in fx['sequential/1/cols']]
for c in range(D.shape[1]):
    print(cols[c], np.nanmax(np.abs(D[:,c]-Dref[:,c])), np.nanmax(np.abs(Dy[:,c]-Dref[:,c])), np.nanmax(np.abs(D[:,c]-Dy[:,c])))
print('sigma', e.singular_values(), fx['sigma'])
