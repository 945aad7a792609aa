set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
N2V2R_TRACE=1 timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/tests_trace.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 300 python -u tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" > gpurun_out/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
timeout -k 10 300 python -u tools/sweep_eig.py 200000 128 30 "[[0,0,0,0]]" >> gpurun_out/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
