#!/bin/bash
# Round 4 (session 2): cfg4 PMC of the current tiled SpMM (kernel trace, FETCH_SIZE, WRITE_SIZE,
# L2 hit passes) -- the `traffic` record bench.py reads (profiles/spmm_traffic.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof5
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B4="bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
K4="spmm8_flat_kernel"
run kt4 400 --kernel-trace --stats -d $O/cfg4/kt -o run -- python -u $B4
run p4f 400 --pmc FETCH_SIZE --kernel-include-regex "$K4" -d $O/cfg4/fetch -o run -- python -u $B4
run p4w 400 --pmc WRITE_SIZE --kernel-include-regex "$K4" -d $O/cfg4/write -o run -- python -u $B4
run p4h 400 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K4" -d $O/cfg4/hit -o run -- python -u $B4
echo done
