# Round-3 closing lines on the final build: smoke, bench default (cfg4 + CPU baseline), cfg2,
# cfg3, cfg1, API breakdown cfg4.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final4
mkdir -p $O
export TMPDIR=/tmp
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo cfg4-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg2 --steps 10 --warmup 2 --resident-steps 10 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo cfg2-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg3 --steps 3 --warmup 1 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { echo cfg3-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg1 --steps 20 --warmup 2 --resident-steps 20 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || { echo cfg1-fail; exit 1; }
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg4 > $O/breakdown_cfg4.json 2>&1 || { echo bd4-fail; exit 1; }
echo done
