#!/bin/bash
# Round 4 (session 2): embedding capture at d = 60 / 100 beside 64 / 128
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "lean_check_bit_identical" > gpurun_out/r04_ycap_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r04_ycap_tests.log
exit $rc
