# iteration check: full GPU suite, smoke, cfg2 bench line, cfg2 rocprofv3 kernel stats
# usage: TAG=name bash tools/gpu_iter.sh   (outputs under gpurun_out/$TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-iter}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo tests-fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; cat $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo bench-fail; tail $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2_bench.json 2> $O/prof2_bench.err || { echo prof-fail; exit 1; }
find $O -name "*kernel_trace.csv" -delete
