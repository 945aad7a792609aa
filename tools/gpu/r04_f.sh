#!/bin/bash
# Round 4: tiled SpMM tests with the non-temporal index stream (now default), the phase-barrier
# A/B, then the MFMA counter passes for ritz_nn / ts_nn (r04_pmc_mfma.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "spmm or cfg4_end or paired" \
  > gpurun_out/r04_f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/flat_knob_probe.py --var N2V2R_FLAT_BAR --fits 2 > gpurun_out/r04_flat_bar.jsonl 2> gpurun_out/r04_flat_bar.err
rc=$?; cat gpurun_out/r04_flat_bar.jsonl; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r04_pmc_mfma.sh
