#!/bin/bash
# Round 4, final build: the whole GPU suite (prints kept: taus, residuals) + smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=5 --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r04_final_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04_final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
rc=$?; cat gpurun_out/r04_smoke.log; exit $rc
