# kernel traces of a short cfg2 bench under two settings of one env switch (VAR, A, B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in $A $B; do
  O=gpurun_out/traceab/$v
  mkdir -p $O
  env $VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo trace-fail; tail -3 $O/b.err; exit 1; }
done
