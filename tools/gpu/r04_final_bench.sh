#!/bin/bash
# Round 4, final build (rerun in the second session): closing bench lines (cfg4 = the default, cfg3, cfg2, cfg1) and the cfg4
# kernel trace of a one-step bench (csv stats)
set -o pipefail
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/final_bench_heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_cfg4.json 2> gpurun_out/r04_bench_cfg4.err || exit $?
cut -c1-300 gpurun_out/r04_bench_cfg4.json
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 > gpurun_out/r04_bench_cfg3.json 2> gpurun_out/r04_bench_cfg3.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 > gpurun_out/r04_bench_cfg2.json 2> gpurun_out/r04_bench_cfg2.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg1 --steps 20 --warmup 3 > gpurun_out/r04_bench_cfg1.json 2> gpurun_out/r04_bench_cfg1.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_cfg4_prof -o cfg4 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_cfg4_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_cfg4_prof.err || exit $?
echo done
