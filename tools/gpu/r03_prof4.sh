# cfg4 profile of the default (flat-window) tiled SpMM: kernel trace + FETCH / WRITE / L2-hit
# passes; cfg2 with the column blocks forced on (A/B against its row kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof4
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B4="bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline"
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
K4="spmm8_tile_kernel|spmm8_flat_kernel"
run kt4 400 --kernel-trace --stats -d $O/cfg4/kt -o run -- python -u $B4
run p4f 400 --pmc FETCH_SIZE --kernel-include-regex "$K4" -d $O/cfg4/fetch -o run -- python -u $B4
run p4w 400 --pmc WRITE_SIZE --kernel-include-regex "$K4" -d $O/cfg4/write -o run -- python -u $B4
run p4h 400 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K4" -d $O/cfg4/hit -o run -- python -u $B4
for cb in 0 1; do
  N2V2R_SPMM_CB=$cb timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 --resident-steps 10 --no-cpu-baseline > $O/cfg2_cb$cb.json 2> $O/cfg2_cb$cb.err || { echo cfg2-fail-$cb; exit 1; }
done
echo done
