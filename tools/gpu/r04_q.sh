# L2 hit rates: the gather microbenchmark at a 2 MB panel (32-B rows) against the flat tiled
# SpMM's cfg4 layer launches (16 column blocks = 2 MB panel blocks), one --pmc pass each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcq
mkdir -p $O
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/$name.log; exit 1; }
}
run gkt 120 --kernel-trace --stats --output-format csv -d $O/gather/kt -o run -- $GRAFT_REPO_ROOT/tools/gather_ceiling 100 5 2 32
run ghit 120 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/gather/hit -o run -- $GRAFT_REPO_ROOT/tools/gather_ceiling 100 5 2 32
run skt 300 --kernel-trace --stats --output-format csv -d $O/flat/kt -o run -- python3 -u tools/flat_knob_probe.py --fits 0 --modes 1 --reps 5
run shit 300 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex spmm8_flat --output-format csv -d $O/flat/hit -o run -- python3 -u tools/flat_knob_probe.py --fits 0 --modes 1 --reps 5
run greq 120 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d $O/gather/req -o run -- $GRAFT_REPO_ROOT/tools/gather_ceiling 100 5 2 32
run sreq 300 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --kernel-include-regex spmm8_flat --output-format csv -d $O/flat/req -o run -- python3 -u tools/flat_knob_probe.py --fits 0 --modes 1 --reps 5
echo done
