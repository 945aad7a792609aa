# A/B of one cfg4 fit-and-rank under env settings: AB="ENV=V;ENV=V ENV=V ..." (space-separated
# sets, ';'-joined assignments)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg4ab
export TMPDIR=/tmp
rm -f gpurun_out/cfg4ab/sweep.log
for set in ${AB:-NONE=0}; do
  echo "== $set" >> gpurun_out/cfg4ab/sweep.log
  env ${set//;/ } timeout -k 10 200 python -u bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline >> gpurun_out/cfg4ab/sweep.log 2>> gpurun_out/cfg4ab/err.log || { echo bench-fail; exit 1; }
done
