#!/bin/bash
# Round 6 measurement set on the current library: bench lines cfg1, cfg2, cfg4, cfg5 (one GPU);
# cfg4 kernel trace + PMC passes of the tiled SpMM (FETCH_SIZE, WRITE_SIZE, fabric requests),
# each pass a run of its own
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_j
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for c in cfg1 cfg2 cfg4; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed rc=$?"; tail -20 $O/bench_$c.err; exit 1; }
done
timeout -k 10 600 python -u bench.py --config cfg5 --steps 2 --warmup 1 --resident-steps 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo "bench cfg5 failed rc=$?"; tail -20 $O/bench_cfg5.err; exit 1; }
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
