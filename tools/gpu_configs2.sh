# every single-GPU config once (bench lines), cfg4 twice-step for timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cfgs
mkdir -p $O
for c in cfg1 cfg3 cfg4; do
  st=3; [ $c = cfg4 ] && st=2
  timeout -k 10 400 python -u bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { echo "$c failed"; tail -5 $O/$c.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); g=d['eig']
print('$c', d['ms_per_step'], 'ms', d['value'], 'nodes/s cycles', g['restarts'], 'apps', g['block_applications'], 'res %.2e' % g['max_residual'])
"
done
