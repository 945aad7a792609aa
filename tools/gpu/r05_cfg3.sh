#!/bin/bash
# Round 5, BASELINE cfg3 (dense |corr| layers, N = 20k, d = 256): kernel trace of the bench's own
# fit (the Rayleigh-Ritz per cycle: rr_tridiag_coop_kernel, sharded grid barrier), the same with
# the one-counter barrier (N2V2R_RR_TRI_BAR=single), then counter passes for the dense SpMM
# (dense_tn_kernel: MFMA busy vs waits, HBM fetch) -- each pass a run of its own
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_r05c3
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B3="bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 0 --no-cpu-baseline"
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
K="dense_tn_kernel"
run kt 300 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python -u $B3
N2V2R_RR_TRI_BAR=single run kts 300 --kernel-trace --stats --output-format csv -d $O/kt_single -o run -- python -u $B3
run m 300 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d $O/mfma -o run -- python -u $B3
run f 300 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $O/fetch -o run -- python -u $B3
echo done
