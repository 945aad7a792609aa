# stage-2 running reduce on the side stream: column-block tests, cfg4 A/B (overlap off / on)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cbo2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -k "column_blocks or spmm" > gpurun_out/cbo2/tests.log 2>&1 || { echo tests-fail; exit 1; }
for set in N2V2R_CB_OVERLAP=0 NONE=0 N2V2R_CB_OVERLAP=0 NONE=0; do
  echo "== $set" >> gpurun_out/cbo2/ab.log
  env $set timeout -k 10 200 python -u bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/cbo2/ab.log 2>> gpurun_out/cbo2/err.log || { echo bench-fail; exit 1; }
done
