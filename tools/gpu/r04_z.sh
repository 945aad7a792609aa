#!/bin/bash
# Round 4 (session 2): keep 21d/16 by default -- the whole GPU suite + smoke, then bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04_final_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || exit $?
cat gpurun_out/r04_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_cfg4.json 2> gpurun_out/r04_bench_cfg4.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 > gpurun_out/r04_bench_cfg2.json 2> gpurun_out/r04_bench_cfg2.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg1 --steps 20 --warmup 3 > gpurun_out/r04_bench_cfg1.json 2> gpurun_out/r04_bench_cfg1.err || exit $?
for c in 4 2 1; do python -c "
import json; d=json.load(open('gpurun_out/r04_bench_cfg$c.json')); print('cfg$c', d['ms_per_step'], d['value'], d['device_resident'], d['eig']['block_applications'], d['eig']['restarts'], d['eig']['max_residual'])"; done
