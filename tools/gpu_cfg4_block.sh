# cfg4 fit-and-rank at Krylov block widths 8 / 16 / 32 (one step each)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg4b
export TMPDIR=/tmp
rm -f gpurun_out/cfg4b/sweep.log
for blk in 8 16 32; do
  echo "== block $blk" >> gpurun_out/cfg4b/sweep.log
  timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline --eig "{\"block\": $blk}" >> gpurun_out/cfg4b/sweep.log 2>> gpurun_out/cfg4b/err.log || { echo bench-fail; exit 1; }
done
