# HEAD check: GPU suite, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/head
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo tests-fail; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo bench-fail; tail $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
