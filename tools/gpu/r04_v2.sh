#!/bin/bash
# Round 4 (session 2): cProfile of a cfg2 API call (where its 7 ms beside the fit go)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/api_profile.py --config cfg2 > gpurun_out/r04_api_profile_cfg2.txt 2>&1 || exit $?
head -45 gpurun_out/r04_api_profile_cfg2.txt
