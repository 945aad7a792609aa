# Round-3 final lines on the final build: bench default (cfg4 + CPU baseline), cfg2, cfg3, cfg1,
# cfg5 on one GPU, API breakdowns, and the cfg4 kernel trace of the bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final2
mkdir -p $O
export TMPDIR=/tmp
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u bench.py > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo cfg4-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg2 --steps 10 --warmup 2 --resident-steps 10 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo cfg2-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg3 --steps 3 --warmup 1 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { echo cfg3-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg1 --steps 20 --warmup 2 --resident-steps 20 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || { echo cfg1-fail; exit 1; }
for c in cfg2 cfg4 cfg3; do
  timeout -k 10 300 python -u tools/api_breakdown.py --config $c > $O/breakdown_$c.json 2>&1 || { echo bd-$c-fail; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt4 -o run -- python -u bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > $O/kt4.log 2>&1 || { echo kt4-fail; exit 1; }
timeout -k 10 700 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > $O/bench_cfg5_1gpu.json 2> $O/bench_cfg5_1gpu.err || { echo cfg5-fail; exit 1; }
echo done
