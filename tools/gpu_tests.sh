set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/debug_conv.py > gpurun_out/conv.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py -q -x > gpurun_out/dist.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/dist.log
timeout -k 10 900 python -m pytest tests -q -m gpu --deselect tests/test_gpu_dist.py > gpurun_out/t1.log 2>&1
rc2=$?; echo "exit=$rc2" >> gpurun_out/t1.log
[ $rc -eq 0 ] && [ $rc2 -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
