#!/bin/bash
# Round 4 (session 2): where the host side of a cfg4 API call goes (cProfile)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/api_profile.py --config cfg4 > gpurun_out/r04_api_profile_cfg4.txt 2>&1 || exit $?
head -60 gpurun_out/r04_api_profile_cfg4.txt
