# round-2 record (final build), part B: cfg1/cfg3/cfg4 bench lines, rocprofv3 stats of cfg4,
# fit-level PMC of the cfg2 orthogonalisation kernels (separate passes, counters alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i
mkdir -p $O
export TMPDIR=/tmp
for c in cfg1 cfg3 cfg4; do
  st=5; [ $c = cfg4 ] && st=2; [ $c = cfg3 ] && st=3
  timeout -k 10 400 python -u bench.py --config $c --steps $st --warmup 1 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "$c failed"; tail -5 $O/bench_$c.err; exit 1; }
  tail -1 $O/bench_$c.json | cut -c1-200
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o run -- python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof4_bench.json 2> $O/prof4_bench.err || { echo prof4-fail; exit 1; }
find $O -name "*kernel_trace.csv" -delete
P=gpurun_out/pmc
mkdir -p $P
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "ts_tn_stream|pip_fused|spmm8_pipe|reduce_cols" --output-format csv -d $P/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/p$i.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $P/p$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "ts_tn_stream|pip_fused|spmm8_pipe|reduce_cols" --output-format csv -d $P/kt -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/kt.log 2>&1 || { echo trace-fail; exit 1; }
echo done
