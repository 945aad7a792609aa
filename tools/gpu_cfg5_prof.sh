# cfg5 on one GPU: rocprofv3 kernel stats of one fit (no warmup)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5p
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5p/prof -o run -- python3 -u bench.py --config cfg5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c5p/b.json 2> gpurun_out/c5p/b.err || { tail -5 gpurun_out/c5p/b.err; exit 1; }
find gpurun_out/c5p -name "*kernel_trace.csv" -delete
echo ok
