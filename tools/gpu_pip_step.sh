# fused PIP pass: probe (full run + phases), solver GPU tests, cfg2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/pip_probe.txt
for k in 0 4 5 6; do
  echo "== N2V2R_PIP_STOP=$k" >> gpurun_out/pip_probe.txt
  N2V2R_PIP_STOP=$k timeout -k 10 60 ./tools/pip_probe >> gpurun_out/pip_probe.txt 2>&1 || { cat gpurun_out/pip_probe.txt; exit 1; }
done
grep -E "==|local|applied  1:|applied  7|all" gpurun_out/pip_probe.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_poison.py tests/test_gpu_dist.py -k "uase or lean or reorth or band or poison or dist or rank_deficient or redo or end_to_end" > gpurun_out/ab_tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -3 gpurun_out/b.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1])
print('%8.3f ms  apps %d  res %.3e' % (d['ms_per_step'], d['eig']['block_applications'], d['eig']['max_residual']))"
done
