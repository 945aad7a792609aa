# dense GEMM (LDS-staged, batched loads) + tiled SpMM block counts + new regression tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py tests/test_gpu_ingest_device.py tests/test_gpu_parity.py tests/test_gpu_writer.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "dense or cfg3 or ingest or large_dimension or sturm_failure or loose or random_starts or fallbacks or writer or output or agg or edited or column_blocks" > gpurun_out/ab2/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab2/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/ab2/cfg3.json 2> gpurun_out/ab2/cfg3.err || { echo bench-cfg3-fail; exit 1; }
for nb in 4 8; do
  N2V2R_SPMM_TILE_NB=$nb timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/ab2/cfg4_nb$nb.json 2> gpurun_out/ab2/cfg4_nb$nb.err || { echo bench-fail-$nb; exit 1; }
done
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg4 > gpurun_out/ab2/breakdown_cfg4.json 2>&1 || { echo breakdown-fail; exit 1; }
echo done
