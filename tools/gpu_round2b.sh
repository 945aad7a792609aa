# round-2 record (final build), part A: full GPU suite, smoke, default bench (cfg2, CPU baseline),
# rocprofv3 kernel stats of the cfg2 bench, SpMM PMC passes (FETCH_SIZE / WRITE_SIZE / trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j
mkdir -p $O gpurun_out/meas
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo tests-fail; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo bench-fail; tail $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2_bench.json 2> $O/prof2_bench.err || { echo prof2-fail; exit 1; }
find $O -name "*kernel_trace.csv" -delete
M=gpurun_out/meas
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $M/fetch -o run -- python3 tools/spmm_probe.py > $M/fetch.log 2>&1 || { echo fetch-fail; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $M/write -o run -- python3 tools/spmm_probe.py > $M/write.log 2>&1 || { echo write-fail; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $M/ptrace -o run -- python3 tools/spmm_probe.py > $M/ptrace.log 2>&1 || { echo ptrace-fail; exit 1; }
find $M -name "*kernel_trace.csv" -delete
echo done
