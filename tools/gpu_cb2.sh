# column-block SpMM: GPU tests, cfg4 bench line (with CPU baseline), cfg4 rocprofv3 stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cb2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -k "column_blocks or spmm" > gpurun_out/cb2/tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg4 --steps 2 --warmup 1 > gpurun_out/cb2/bench_cfg4.json 2> gpurun_out/cb2/bench_cfg4.err || { echo bench-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cb2/prof -o run -- python3 bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/cb2/prof_bench.json 2> gpurun_out/cb2/prof_bench.err || { echo prof-fail; exit 1; }
find gpurun_out/cb2/prof -name "*kernel_trace.csv" -delete
