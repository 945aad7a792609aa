#!/bin/bash
# Round 4 (session 2): what the L2's fabric read counters count for 32-B gathers -- the gather
# microbenchmark at 2 / 32 / 320 MB panels (every access form, 100M entries per launch) and the
# flat tiled SpMM at cfg4's size (one layer, 16 column blocks), one --pmc pass each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/cal
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || { echo "counter list failed"; tail -5 $O/counters.txt; exit 1; }
C=""
for c in TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_DRAM TCC_MISS; do
  if grep -q "\b$c\b" $O/counters.txt; then C="$C ${c}_sum"; fi
done
echo "counters:$C"
[ -n "$C" ] || exit 1
run() {
  local name=$1 lim=$2; shift 2
  timeout -s KILL $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
for mb in 2 32 320; do
  run g$mb 90 --pmc $C --output-format csv -d $O/g$mb -o run -- $GRAFT_REPO_ROOT/tools/gather_ceiling 100 3 $mb 32
done
run flat 240 --pmc $C --kernel-include-regex spmm8_flat --output-format csv -d $O/flat -o run -- python3 -u tools/tile_nb_probe.py 1000000 50 16
echo done
