# kernel trace of a short cfg2 bench (timeline analysis of the restart overlap)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/traceov
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo trace-fail; tail -3 $O/b.err; exit 1; }
ls $O
