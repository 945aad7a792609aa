set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/t1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
N2V2R_TRACE=1 timeout -k 10 1000 python tools/sweep_big.py 10000000 30 128 "[[160,512]]" 150 > gpurun_out/sweep_big5.log 2>&1
