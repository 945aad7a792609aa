# int32 block row pointers: column-block tests, SpMM probe, cfg4 one-step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cbr
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -k "column_blocks or spmm" > gpurun_out/cbr/tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 100 python -u tools/cb_probe.py 300000:30 1000000:50 3000000:30 > gpurun_out/cbr/probe.log 2>&1 || { echo probe-fail; exit 1; }
timeout -k 10 200 python -u bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/cbr/cfg4.json 2> gpurun_out/cbr/cfg4.err || { echo bench-fail; exit 1; }
