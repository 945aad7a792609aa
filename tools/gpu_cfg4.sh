set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err
echo "exit=$?" >> gpurun_out/cfg4.err
