#!/bin/bash
# Round 4 (session 2): gather ceiling with wider index loads (dword / dwordx2 per lane handed to
# the lane pairs by ds_bpermute); cfg4 API breakdown; Rayleigh-Ritz back-transform with the
# T factors precomputed (stage tests, cfg3 bench + kernel trace)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/gather_ceiling 100 20 2 32 > gpurun_out/r04_gather_wide.jsonl || exit $?
cat gpurun_out/r04_gather_wide.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_dense.py -k "rayleigh_ritz_stage or dense" > gpurun_out/r04_t_tests.log 2>&1 || { tail -30 gpurun_out/r04_t_tests.log; exit 1; }
tail -3 gpurun_out/r04_t_tests.log
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04_t_cfg3.json 2> gpurun_out/r04_t_cfg3.err || exit $?
cut -c1-400 gpurun_out/r04_t_cfg3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_t_cfg3_prof -o cfg3 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/gpurun_out/r04_t_cfg3_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04_t_cfg3_prof.err || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg4 > gpurun_out/r04_api_breakdown_cfg4.json 2> gpurun_out/r04_api_breakdown_cfg4.err || exit $?
cat gpurun_out/r04_api_breakdown_cfg4.json
