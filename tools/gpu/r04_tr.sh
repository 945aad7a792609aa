#!/bin/bash
# Round 4 (session 2): per-cycle convergence trace of the bench's cfg4 graph and cfg2 (how much of
# the last cycle a mid-cycle stop could save)
set -o pipefail
mkdir -p gpurun_out
N2V2R_TRACE=1 timeout -k 10 200 python -u tools/trace_fit.py 1000000 50 128 1000 > gpurun_out/r04_trace_cfg4.txt 2>&1 || exit $?
N2V2R_TRACE=1 timeout -k 10 200 python -u tools/trace_fit.py 100000 20 64 1000 > gpurun_out/r04_trace_cfg2.txt 2>&1 || exit $?
grep -v "host: rr start" gpurun_out/r04_trace_cfg4.txt | tail -30
