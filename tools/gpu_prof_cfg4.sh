# rocprofv3 kernel stats of one cfg4 fit-and-rank (N = 1M, d = 128)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg4prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg4prof -o run -- python3 bench.py --config cfg4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/cfg4prof/bench.json 2> gpurun_out/cfg4prof/bench.err || { echo prof-fail; exit 1; }
find gpurun_out/cfg4prof -name "*kernel_trace.csv" -delete
