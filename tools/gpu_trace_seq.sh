# kernel trace of one cfg2 fit (warmup 1, steps 1): per-launch durations and gaps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tseq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b.json 2> $O/b.err || { echo trace-fail; tail $O/b.err; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1)
python3 tools/trace_seq.py $f 60 > $O/seq.txt
python3 tools/trace_split.py $f > $O/split.txt && python3 tools/trace_gaps.py $f > $O/gaps.txt
rm -f $f
