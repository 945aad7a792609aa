#!/bin/bash
# Round 4: non-temporal index stream (microbenchmark + flat kernel A/B), cfg2 API trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 tools/gather_ceiling 100 20 > gpurun_out/r04_gather_ceiling_nt.jsonl 2>&1
rc=$?; grep -E '"panel_MB": (2|4|8),' gpurun_out/r04_gather_ceiling_nt.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/flat_nt_probe.py > gpurun_out/r04_flat_nt.jsonl 2> gpurun_out/r04_flat_nt.err
rc=$?; cat gpurun_out/r04_flat_nt.jsonl; [ $rc -eq 0 ] || exit $rc
N2V2R_TRACE=1 timeout -k 10 200 python -u tools/api_breakdown.py --config cfg2 > gpurun_out/r04_api_cfg2.json 2> gpurun_out/r04_api_cfg2.err
rc=$?; cat gpurun_out/r04_api_cfg2.json; exit $rc
