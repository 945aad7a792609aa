# tiled SpMM: column blocks per layer (panel block vs 4 MB L2) x row-group / flat forms.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nb
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/nb/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ingest_device.py tests/test_gpu_configs.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider -k "borda or ingest or large_directed or cfg2 or cfg4_api" > gpurun_out/nb/tests.log 2>&1 || { echo tests-failed; exit 1; }
for v in "1 16" "1 32" "0 16" "1 8"; do
  set -- $v
  N2V2R_TILE_FLAT=$1 N2V2R_SPMM_TILE_NB=$2 timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/nb/cfg4_f$1_nb$2.json 2> gpurun_out/nb/cfg4_f$1_nb$2.err || { echo bench-fail-$1-$2; exit 1; }
done
echo done
