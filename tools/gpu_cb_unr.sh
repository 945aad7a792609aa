# cb_row_accumulate A/B (two index group-widths per gather round) + column-block tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cbu
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -k "column_blocks" > gpurun_out/cbu/tests.log 2>&1 || { echo tests-fail; exit 1; }
for set in N2V2R_CB_UNR=0 NONE=0 N2V2R_CB_RPW=8 N2V2R_CB_WGS=8192; do
  echo "== $set" >> gpurun_out/cbu/sweep.log
  env $set timeout -k 10 100 python -u tools/cb_probe.py 300000:30 1000000:50 3000000:30 >> gpurun_out/cbu/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
done
