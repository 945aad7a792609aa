#!/bin/bash
# Round 5: cfg4 kernel trace + PMC passes of the tiled SpMM (window offsets, segment fold) in the
# bench's own fits: FETCH_SIZE, WRITE_SIZE, and the fabric-request pass (TCC_EA0_RDREQ: one
# 128-B request per L2 miss for this access shape, profiles/r04_fabric_req_calibration.md) --
# each pass a run of its own (rocprofv3 does not split counters over passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_r05
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B4="bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 0 --no-cpu-baseline"
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
K4="spmm8_flat_kernel"
run kt4 300 --kernel-trace --stats -d $O/cfg4/kt -o run -- python -u $B4
run p4f 300 --pmc FETCH_SIZE --kernel-include-regex "$K4" -d $O/cfg4/fetch -o run -- python -u $B4
run p4w 300 --pmc WRITE_SIZE --kernel-include-regex "$K4" -d $O/cfg4/write -o run -- python -u $B4
run p4r 300 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex "$K4" -d $O/cfg4/rdreq -o run -- python -u $B4
echo done
