#!/bin/bash
# Round 4: the whole GPU suite on the current build, the gather ceiling microbenchmark, a cfg3
# kernel trace (csv) and the cfg4 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 tools/gather_ceiling 100 20 > gpurun_out/r04_gather_ceiling.jsonl 2>&1
rc=$?; cat gpurun_out/r04_gather_ceiling.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_prof2 -o cfg3 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench2.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench2.err
rc=$?; cut -c1-300 $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench2.json; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r04_bench_cfg4.json 2> gpurun_out/r04_bench_cfg4.err
rc=$?; cut -c1-400 gpurun_out/r04_bench_cfg4.json; exit $rc
