# round-2 baseline at HEAD: full GPU suite, smoke, default bench (cfg2), rocprofv3 kernel stats of cfg2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02base
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo tests-fail; tail -30 $O/tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo bench-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2_bench.json 2> $O/prof2_bench.err || { echo prof-fail; exit 1; }
find $O -name "*kernel_trace.csv" -delete
tail -3 $O/tests.log; cat $O/smoke.log $O/bench_cfg2.json
