#!/bin/bash
# Round 4: dense_tn_kernel depth / occupancy forms vs the LDS-staged GEMM (cfg3 size)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "dense_gemm" > gpurun_out/r04_i_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_i_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dense_tn_probe.py --fits 0 > gpurun_out/r04_dense_tn2.jsonl 2> gpurun_out/r04_dense_tn2.err
rc=$?; cat gpurun_out/r04_dense_tn2.jsonl; exit $rc
