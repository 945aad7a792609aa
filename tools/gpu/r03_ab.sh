# cfg4 SpMM form A/B (tiled, 8/16/32 blocks; partials form), dense GEMM tests + cfg3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py tests/test_gpu_dist.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "dense or cfg3 or cfg4_full or cfg5 or partitioned or rccl" > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
for nb in 16 8 32; do
  N2V2R_SPMM_TILE_NB=$nb timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/ab/cfg4_nb$nb.json 2> gpurun_out/ab/cfg4_nb$nb.err || { echo bench-fail-$nb; exit 1; }
done
timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/ab/cfg3.json 2> gpurun_out/ab/cfg3.err || { echo bench-cfg3-fail; exit 1; }
echo done
