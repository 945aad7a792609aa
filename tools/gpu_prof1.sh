set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
echo "exit=$?" >> gpurun_out/prof/bench.err
find gpurun_out/prof -name "*.csv" | head -20 >> gpurun_out/prof/bench.err
