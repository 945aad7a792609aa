# dense GEMM (cfg3): X staged transposed (16-B operand reads) vs k-major.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dg2
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/dg2/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -v -rf -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "dense or cfg3" > gpurun_out/dg2/tests.log 2>&1 || { echo tests-failed; exit 1; }
for v in 1 0; do
  N2V2R_DG_XT=$v timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/dg2/cfg3_xt$v.json 2> gpurun_out/dg2/cfg3_xt$v.err || { echo bench-fail-$v; exit 1; }
done
timeout -k 10 400 python -u tools/probe_block.py --config cfg4 --blocks 8 16 > gpurun_out/dg2/probe_block.jsonl 2> gpurun_out/dg2/probe_block.err || { echo probe-fail; exit 1; }
echo done
