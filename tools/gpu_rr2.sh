set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "rayleigh" > gpurun_out/rr.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/t1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2>/dev/null || exit 1
mkdir -p gpurun_out/prof2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof2/bench.json 2> gpurun_out/prof2/bench.err
find gpurun_out/prof2 -name "*kernel_trace.csv" -delete
