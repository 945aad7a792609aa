set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
N2V2R_TRACE=1 timeout -k 10 900 python bench.py --config cfg5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || exit 1
timeout -k 10 600 python bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err
