#!/bin/bash
# Round 6: bench lines on the current library: cfg4 at N = 1 (the driver's headline) and the N > 1
# API path rehearsed over a repeated device (N2V2R_BENCH_DEVICES=0,0: the thread communicator)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_i
mkdir -p $O
timeout -k 10 400 python -u bench.py --config cfg4 --steps 5 --warmup 2 > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed rc=$?"; tail -20 $O/cfg4.err; exit 1; }
N2V2R_BENCH_DEVICES=0,0 timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline --resident-steps 0 > $O/cfg4_dev00.json 2> $O/cfg4_dev00.err || { echo "dev00 failed rc=$?"; tail -20 $O/cfg4_dev00.err; exit 1; }
echo done
