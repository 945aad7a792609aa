# Round-3 profiles: kernel-trace stats of the cfg4 / cfg2 / cfg3 bench commands, then separate
# PMC passes (FETCH_SIZE; WRITE_SIZE; L2 hit; MFMA busy) for the dominant kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B4="bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
B2="bench.py --config cfg2 --steps 3 --warmup 1 --resident-steps 3 --no-cpu-baseline"
B3="bench.py --config cfg3 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
run() {  # name, limit, rocprofv3 args..., -- , command
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
run kt4 400 --kernel-trace --stats -d $O/cfg4/kt -o run -- python -u $B4
run kt2 300 --kernel-trace --stats -d $O/cfg2/kt -o run -- python -u $B2
run kt3 300 --kernel-trace --stats -d $O/cfg3/kt -o run -- python -u $B3
K4="spmm8_tile_kernel|spmm8_flat_kernel"
run p4f 400 --pmc FETCH_SIZE --kernel-include-regex "$K4" -d $O/cfg4/fetch -o run -- python -u $B4
run p4w 400 --pmc WRITE_SIZE --kernel-include-regex "$K4" -d $O/cfg4/write -o run -- python -u $B4
run p4h 400 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K4" -d $O/cfg4/hit -o run -- python -u $B4
K3="dense_gemm_kernel|ritz_nn_kernel"
run p3f 300 --pmc FETCH_SIZE --kernel-include-regex "$K3" -d $O/cfg3/fetch -o run -- python -u $B3
run p3w 300 --pmc WRITE_SIZE --kernel-include-regex "$K3" -d $O/cfg3/write -o run -- python -u $B3
run p3m 300 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE --kernel-include-regex "$K3" -d $O/cfg3/mfma -o run -- python -u $B3
echo done
