set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/check
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/check/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/check/prof_bench.json 2> gpurun_out/check/prof_bench.err || { echo "prof rc=$?"; exit 1; }
find gpurun_out/check/prof -name "*kernel_trace.csv" -delete
echo done
