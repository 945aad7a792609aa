#!/bin/bash
# Round 4 (session 2): the dense product with an LDS-DMA ring (N2V2R_DENSE_GLDS=1): bit-identity
# tests, then one-layer launches and cfg3 fits against dense_tn_kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_dense.py -k "glds" > gpurun_out/r04_x_tests.log 2>&1 || { tail -30 gpurun_out/r04_x_tests.log; exit 1; }
tail -3 gpurun_out/r04_x_tests.log
timeout -k 10 400 python -u tools/dense_glds_probe.py > gpurun_out/r04_dense_glds.jsonl 2> gpurun_out/r04_dense_glds.err || exit $?
cat gpurun_out/r04_dense_glds.jsonl
