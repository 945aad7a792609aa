#!/bin/bash
# Round 4: dense_tn_kernel with its loads pinned in batches (sched_barrier) -- tests, A/B of the
# three forms vs the LDS-staged GEMM; the 16-bit index stream in the gather microbenchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "dense_gemm" > gpurun_out/r04_j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_j_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dense_tn_probe.py --fits 0 > gpurun_out/r04_dense_tn3.jsonl 2> gpurun_out/r04_dense_tn3.err
rc=$?; cat gpurun_out/r04_dense_tn3.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 tools/gather_ceiling 100 20 > gpurun_out/r04_gather_ceiling_u16.jsonl 2>&1
rc=$?; grep -E '"panel_MB": (1|2),' gpurun_out/r04_gather_ceiling_u16.jsonl; exit $rc
