#!/bin/bash
# Round 4 (session 2) closing run on the final build: GPU suite + smoke, bench lines (cfg4 = the
# default, cfg3, cfg2, cfg1), cfg4 and cfg3 kernel traces
set -o pipefail
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/close_heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04_final_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || exit $?
cat gpurun_out/r04_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_cfg4.json 2> gpurun_out/r04_bench_cfg4.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 > gpurun_out/r04_bench_cfg3.json 2> gpurun_out/r04_bench_cfg3.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 > gpurun_out/r04_bench_cfg2.json 2> gpurun_out/r04_bench_cfg2.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg1 --steps 20 --warmup 3 > gpurun_out/r04_bench_cfg1.json 2> gpurun_out/r04_bench_cfg1.err || exit $?
for c in 4 3 2 1; do python -c "
import json; d=json.load(open('gpurun_out/r04_bench_cfg$c.json')); print('cfg$c', d['ms_per_step'], d['value'], d['device_resident']['ms_per_step'], d['eig']['block_applications'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_close_cfg4 -o cfg4 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_close_cfg4.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_close_cfg4.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_close_cfg3 -o cfg3 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_close_cfg3.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_close_cfg3.err || exit $?
echo done
