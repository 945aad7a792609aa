# bench lines for the non-default configs (cfg3 dense, cfg4 N=1M, cfg5 N=10M on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfgs
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfgs/cfg4.json 2> gpurun_out/cfgs/cfg4.err || { echo cfg4-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfgs/cfg3.json 2> gpurun_out/cfgs/cfg3.err || { echo cfg3-fail; exit 1; }
timeout -k 10 500 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/cfgs/cfg5.json 2> gpurun_out/cfgs/cfg5.err || { echo cfg5-fail; exit 1; }
