# Final build check: smoke, the whole GPU suite, cfg5 on one GPU (32 column blocks), cfg2 / cfg4
# device-resident fits (two-block Gram folding one right-hand side at a time).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final3
mkdir -p $O
export TMPDIR=/tmp
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider --durations=5 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 --resident-steps 20 --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo cfg2-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 3 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo cfg4-fail; exit 1; }
timeout -k 10 700 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > $O/bench_cfg5_1gpu.json 2> $O/bench_cfg5_1gpu.err || { echo cfg5-fail; exit 1; }
echo done
