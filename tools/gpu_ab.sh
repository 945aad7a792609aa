# A/B timing of one cfg2 fit under env settings: AB="ENV=V;ENV=V ENV=V ..." (space-separated sets,
# ';'-joined assignments); runs the uase GPU tests first (TESTK selects, default "uase").
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
rm -f gpurun_out/ab/sweep.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "${TESTK:-uase}" --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { echo tests-fail; exit 1; }
for set in ${AB:-NONE=0}; do
  echo "== $set" >> gpurun_out/ab/sweep.log
  env ${set//;/ } timeout -k 10 200 python -u tools/sweep_eig.py 100000 64 20 "${CFGS:-[[0,0,0,0]]}" >> gpurun_out/ab/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
done
