#!/bin/bash
# Round 4: full GPU suite (prints kept: Kendall taus, residuals), log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04_gpu_tests.log
exit $rc
