# round-end check after the overlap change: full GPU suite, smoke, cfg4 bench line + rocprofv3 stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/final2/tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg4 --steps 2 --warmup 1 > gpurun_out/final2/bench_cfg4.json 2> gpurun_out/final2/bench_cfg4.err || { echo bench4-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final2/prof4 -o run -- python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/final2/prof4_bench.json 2> gpurun_out/final2/prof4_bench.err || { echo prof4-fail; exit 1; }
find gpurun_out/final2 -name "*kernel_trace.csv" -delete
