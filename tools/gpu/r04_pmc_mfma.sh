# MFMA counters for the TSQR-side MFMA kernels (Ritz products ritz_nn_kernel, general panel
# products ts_nn_kernel) at cfg4 and cfg3, with the kernel trace and HBM bytes of the same run:
# one rocprofv3 pass per counter group
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcm
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B4="bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
B3="bench.py --config cfg3 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
K="ritz_nn_kernel|ts_nn_kernel"
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
run c4kt 400 --kernel-trace --stats --output-format csv -d $O/cfg4/kt -o run -- python -u $B4
run c4m 400 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d $O/cfg4/mfma -o run -- python -u $B4
run c4f 400 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $O/cfg4/fetch -o run -- python -u $B4
run c3kt 300 --kernel-trace --stats --output-format csv -d $O/cfg3/kt -o run -- python -u $B3
run c3m 300 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d $O/cfg3/mfma -o run -- python -u $B3
echo done
