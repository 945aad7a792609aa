# packed flat-window tiled SpMM: parity tests, then cfg4 bench flat vs row groups.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/flat
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/flat/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "column_blocks or spectral" > gpurun_out/flat/tests1.log 2>&1 || { echo small-tests-failed; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dist.py -v -rf -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "cfg4 or cfg5 or partitioned" > gpurun_out/flat/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/flat/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
for f in 1 0; do
  N2V2R_TILE_FLAT=$f timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/flat/cfg4_f$f.json 2> gpurun_out/flat/cfg4_f$f.err || { echo bench-fail-$f; exit 1; }
done
echo done
