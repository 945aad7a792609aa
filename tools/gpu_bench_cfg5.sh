set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --mode partitioned --no-cpu-baseline > gpurun_out/bench_cfg2p.json 2> gpurun_out/bench_cfg2p.err || exit 1
timeout -k 10 900 python bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err
