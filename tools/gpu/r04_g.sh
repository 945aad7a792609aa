#!/bin/bash
# Round 4: register-per-entry Cholesky in pip_chol (8 < b <= 32): the wide-block tests, cfg3
# bench + kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "block_widths or large_dimension or cfg3 or dense or rayleigh" \
  > gpurun_out/r04_g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_g_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_prof3 -o cfg3 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench3.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench3.err
rc=$?; cut -c1-300 $GRAFT_REPO_ROOT/gpurun_out/r04_cfg3_bench3.json; exit $rc
