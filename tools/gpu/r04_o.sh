#!/bin/bash
# Round 4: tiled SpMM bounded-skew phase sync (N2V2R_FLAT_SYNC=2) -- SpMM tests under it, then
# the sync A/B (layer launches and cfg4 fits)
set -o pipefail
mkdir -p gpurun_out
N2V2R_FLAT_SYNC=2 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "spmm_tiled or cfg4_full" > gpurun_out/r04_o_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/flat_knob_probe.py --var N2V2R_FLAT_SYNC --modes 1 2 --fits 2 \
  > gpurun_out/r04_flat_sync.jsonl 2> gpurun_out/r04_flat_sync.err
rc=$?; cat gpurun_out/r04_flat_sync.jsonl; exit $rc
