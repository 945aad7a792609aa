set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "restart_overlap or fallbacks" > gpurun_out/new_tests.log 2>&1 || { echo tests-fail; tail -40 gpurun_out/new_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/new_tests.log | tail -8
