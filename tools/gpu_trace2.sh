# cfg2 kernel trace (per-launch durations in launch order) for tools/trace_split.py
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/trace2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo trace-fail; exit 1; }
ls -R $O
