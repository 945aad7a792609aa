# cfg4 PMC passes for the orthogonalisation kernels of the final build (paired-pass Gram, LDS
# streaming Gram, fused PIP): kernel trace + FETCH_SIZE / WRITE_SIZE / L2 hit, one pass each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcg
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B4="bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
K="ts_tn_stream2_kernel|ts_tn_stream_lds_kernel|pip_fused_kernel"
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
run kt 400 --kernel-trace --stats -d $O/kt -o run -- python -u $B4
run fetch 400 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/fetch -o run -- python -u $B4
run write 400 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/write -o run -- python -u $B4
run hit 400 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" -d $O/hit -o run -- python -u $B4
echo done
