set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
N2V2R_TRACE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s -k "${TESTK:-rank_deficient}" --timeout 120 --timeout-method thread > gpurun_out/one.log 2>&1
