# column-block SpMM: stage-1 reduce overlap on a side stream (N2V2R_CB_OVERLAP=1), tests + cfg4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cbo
export TMPDIR=/tmp
N2V2R_CB_OVERLAP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "column_blocks" > gpurun_out/cbo/tests.log 2>&1 || { echo tests-fail; exit 1; }
for set in NONE=0 N2V2R_CB_OVERLAP=1 NONE=0 N2V2R_CB_OVERLAP=1; do
  echo "== $set" >> gpurun_out/cbo/ab.log
  env $set timeout -k 10 200 python -u bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline >> gpurun_out/cbo/ab.log 2>> gpurun_out/cbo/err.log || { echo bench-fail; exit 1; }
done
