# full GPU suite + cfg2 bench (two runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sb
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/sb/tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/sb/tests.log; exit 1; }
tail -1 gpurun_out/sb/tests.log
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sb/b.json 2> gpurun_out/sb/b.err || { tail -3 gpurun_out/sb/b.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/sb/b.json').read().strip().splitlines()[-1])
print('%8.3f ms  apps %d  res %.3e' % (d['ms_per_step'], d['eig']['block_applications'], d['eig']['max_residual']))"
done
