# L2 hit rate vs gather rate in the microbenchmark: 4 and 8 MB panels (32-B rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcr
mkdir -p $O
for mb in 4 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g$mb/kt -o run -- $GRAFT_REPO_ROOT/tools/gather_ceiling 100 5 $mb 32 > $O/kt$mb.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/g$mb/hit -o run -- $GRAFT_REPO_ROOT/tools/gather_ceiling 100 5 $mb 32 > $O/hit$mb.log 2>&1 || exit 1
done
echo done
