#!/bin/bash
# Round 4: multi-workgroup tridiagonalisation (targeted tests + cfg3 kernel trace), the gather
# ceiling microbenchmark, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "rayleigh_ritz_stage or cfg3 or block_widths or large_dimension" \
  > gpurun_out/r04_rr_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_rr_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_prof -o cfg3 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench.err
rc=$?; cut -c1-600 $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench.json; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && timeout -k 10 180 tools/gather_ceiling 100 20 > gpurun_out/r04_gather_ceiling.jsonl 2>&1
rc=$?; cat gpurun_out/r04_gather_ceiling.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04_gpu_tests.log; exit $rc
