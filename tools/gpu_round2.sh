# round-2 record: full GPU suite, smoke, default bench (cfg2, with CPU baseline), rocprofv3 kernel
# stats of cfg2 and cfg4, cfg1/cfg3/cfg4 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02rec
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo tests-fail; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo bench-fail; tail $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2_bench.json 2> $O/prof2_bench.err || { echo prof2-fail; exit 1; }
for c in cfg1 cfg3 cfg4; do
  st=5; [ $c = cfg4 ] && st=2; [ $c = cfg3 ] && st=3
  timeout -k 10 400 python -u bench.py --config $c --steps $st --warmup 1 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "$c failed"; tail -5 $O/bench_$c.err; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o run -- python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof4_bench.json 2> $O/prof4_bench.err || { echo prof4-fail; exit 1; }
find $O -name "*kernel_trace.csv" -delete
echo done
