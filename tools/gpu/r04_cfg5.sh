#!/bin/bash
# Round 4 (session 2): cfg5 (N = 10M, degree 30, d = 128) on ONE GPU through the partitioned path
# (RCCL world 1) on the final build
set -o pipefail
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/cfg5_heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 0 --no-cpu-baseline > gpurun_out/r04_bench_cfg5_1gpu.json 2> gpurun_out/r04_bench_cfg5_1gpu.err || exit $?
cut -c1-600 gpurun_out/r04_bench_cfg5_1gpu.json
