set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof2/bench.json 2> gpurun_out/prof2/bench.err
echo "exit=$?" >> gpurun_out/prof2/bench.err
find gpurun_out/prof2 -name "*kernel_trace.csv" -delete
