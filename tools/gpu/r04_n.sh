#!/bin/bash
# Round 4: cfg3 basis / keep sweep (dense Rayleigh-Ritz cost vs block applications)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/sweep_cfg3.py > gpurun_out/r04_cfg3_sweep.jsonl 2> gpurun_out/r04_cfg3_sweep.err
rc=$?; cat gpurun_out/r04_cfg3_sweep.jsonl; exit $rc
