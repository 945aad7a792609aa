# column-block SpMM: new GPU tests, then cfg4 one-step A/B (row SpMM vs column blocks)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cb
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "column_blocks or spmm" tests/test_gpu_dist.py > gpurun_out/cb/tests.log 2>&1 || { echo tests-fail; exit 1; }
for set in N2V2R_SPMM_CB=0 N2V2R_SPMM_CB=1; do
  echo "== $set" >> gpurun_out/cb/ab.log
  env $set timeout -k 10 200 python -u bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline >> gpurun_out/cb/ab.log 2>> gpurun_out/cb/err.log || { echo bench-fail; exit 1; }
done
