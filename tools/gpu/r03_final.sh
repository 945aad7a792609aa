# Round-3 bench lines (default cfg4 with the CPU baseline, cfg2, cfg3, cfg1) and API wall times.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u bench.py > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo cfg4-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg2 --steps 10 --warmup 2 --resident-steps 10 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo cfg2-fail; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg3 --steps 3 --warmup 1 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { echo cfg3-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg1 --steps 20 --warmup 2 --resident-steps 20 > $O/bench_cfg1.json 2> $O/bench_cfg1.err || { echo cfg1-fail; exit 1; }
timeout -k 10 200 python -u tools/api_wall.py --config cfg2 --reps 3 > $O/api_cfg2.json 2>&1 || { echo api2-fail; exit 1; }
timeout -k 10 300 python -u tools/api_wall.py --config cfg4 --reps 2 > $O/api_cfg4.json 2>&1 || { echo api4-fail; exit 1; }
timeout -k 10 400 python -u tools/probe_block.py --config cfg4 --blocks 8 --sweep 144:0 192:0 224:0 160:448 160:384 192:448 > $O/sweep_cfg4.jsonl 2> $O/sweep_cfg4.err || { echo sweep-fail; exit 1; }
echo done
