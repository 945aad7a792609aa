import sys, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from conftest import load_fixture, fixture_layers
from node2vec2rank_amd.model import N2V2R
name = sys.argv[1]; strategy = sys.argv[2]
fx = load_fixture(name); layers = fixture_layers(fx)
cfg = dict(embed_dimensions=[int(x) for x in fx["dims"]], distance_metrics=[str(x) for x in fx["metrics"]],
           seed=int(fx["seed"]), comp_strategy=strategy, verbose=1, save_dir=None)
m = N2V2R(graphs=layers, nodes=[str(x) for x in fx["nodes"]], config=cfg)
r = m.fit_transform_rank(); a = m.aggregate_transform()
out = {'Y': m.node_embeddings}
for k in r: out[f'D/{k}'] = r[k].to_numpy(); out[f'B/{k}'] = a[k]['borda_ranks'].to_numpy()
np.savez(f'gpurun_out/dump_{name}_{strategy}.npz', **out)
print(m.eig_stats)
