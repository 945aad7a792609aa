# full GPU suite + smoke + default bench (cfg2) + cfg4 bench and rocprofv3 stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/round
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/round/tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/round/bench_cfg2.json 2> gpurun_out/round/bench_cfg2.err || { echo bench-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/round/prof4 -o run -- python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/round/prof4_bench.json 2> gpurun_out/round/prof4_bench.err || { echo prof-fail; exit 1; }
find gpurun_out/round -name "*kernel_trace.csv" -delete
