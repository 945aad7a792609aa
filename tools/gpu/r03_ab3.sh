# tiled SpMM row-group forms (N2V2R_TILE_PAIR 0/1/2) + the regression tests pending since ab2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/ab3/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for pr in 0 1 2; do
  N2V2R_TILE_PAIR=$pr timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/ab3/cfg4_p$pr.json 2> gpurun_out/ab3/cfg4_p$pr.err || { echo bench-fail-$pr; exit 1; }
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ingest_device.py tests/test_gpu_writer.py tests/test_gpu_dist.py tests/test_ingest.py -v -rf -s --durations=15 --timeout 700 --timeout-method thread -p no:cacheprovider -k "large_dimension or sturm_failure or loose or column_blocks or cfg4 or cfg5 or ingest or writer or dist or partition or gather or projection" > gpurun_out/ab3/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab3/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
echo done
