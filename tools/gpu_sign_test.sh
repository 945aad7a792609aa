set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "sign_convention" > gpurun_out/sign.log 2>&1 || { tail -30 gpurun_out/sign.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/sign.log
