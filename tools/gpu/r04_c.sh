#!/bin/bash
# Round 4: cfg4-grid convergence trace, the tests that failed, the RR stage tests (granule
# hand-off), the gather ceiling, a cfg3 kernel trace (csv) and the cfg4 bench line
set -o pipefail
mkdir -p gpurun_out
N2V2R_TRACE=1 timeout -k 10 200 python -u tools/trace_fit.py 100000 50 128 > gpurun_out/r04_trace_cfg4g.json 2> gpurun_out/r04_trace_cfg4g.err
rc=$?; tail -3 gpurun_out/r04_trace_cfg4g.err; cut -c1-400 gpurun_out/r04_trace_cfg4g.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider -k "rayleigh_ritz_stage or cfg3 or end_to_end or large_dimension or block_widths or cfg4_grid or lean or uase_residuals" \
  > gpurun_out/r04_c_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04_c_tests.log; [ $rc -eq 0 ] || exit $rc
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
