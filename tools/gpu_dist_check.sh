# distances kernels: parity tests, bench, per-kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dc
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -k "distances or end_to_end or model or dist or demo or pairwise or borda" > gpurun_out/dc/tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/dc/tests.log; exit 1; }
tail -1 gpurun_out/dc/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dc/t -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dc/b.json 2> gpurun_out/dc/b.err || { echo trace-fail; exit 1; }
find gpurun_out/dc/t -name "*kernel_trace.csv" -delete
f=$(find gpurun_out/dc/t -name "*kernel_stats.csv" | head -1)
grep -iE "distances|borda_init" $f | cut -c1-160
