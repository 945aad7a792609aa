set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run -- python3 bench.py --config cfg5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof5/bench.json 2> gpurun_out/prof5/bench.err
echo "exit=$?" >> gpurun_out/prof5/bench.err
find gpurun_out/prof5 -name "*kernel_trace.csv" -delete
