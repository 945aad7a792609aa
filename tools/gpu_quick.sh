set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/tests.log; exit 1; }
timeout -k 10 300 python -u tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" > gpurun_out/sweep.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profq -o run -- python3 tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" > gpurun_out/profq.log 2>&1 || exit 1
find gpurun_out/profq -name "*kernel_trace.csv" -delete
