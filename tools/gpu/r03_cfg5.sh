# cfg5 on one GPU (partitioned path, W = 1): the row kernel (320 MB panel, default) vs the flat
# tiled form with the column-block window opened to 400 MB (32 blocks of 10 MB).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/c5/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
N2V2R_CB_MAX_MB=400 timeout -k 10 500 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > gpurun_out/c5/cfg5_flat.json 2> gpurun_out/c5/cfg5_flat.err || { echo flat-fail; exit 1; }
timeout -k 10 500 python -u bench.py --config cfg5 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > gpurun_out/c5/cfg5_row.json 2> gpurun_out/c5/cfg5_row.err || { echo row-fail; exit 1; }
echo done
