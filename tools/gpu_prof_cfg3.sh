set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 bench.py --config cfg3 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof3/bench.json 2> gpurun_out/prof3/bench.err
find gpurun_out/prof3 -name "*kernel_trace.csv" -delete
