set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_dense.py -q -x > gpurun_out/dense.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/dense.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config cfg3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err
