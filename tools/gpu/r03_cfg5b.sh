# cfg5 on one GPU with the flat tiled form by default (64 blocks of 5 MB) vs 32 blocks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5b
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/c5b/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > gpurun_out/c5b/cfg5_default.json 2> gpurun_out/c5b/cfg5_default.err || { echo default-fail; exit 1; }
N2V2R_SPMM_TILE_NB=32 timeout -k 10 600 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > gpurun_out/c5b/cfg5_nb32.json 2> gpurun_out/c5b/cfg5_nb32.err || { echo nb32-fail; exit 1; }
echo done
