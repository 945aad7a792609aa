#!/bin/bash
# Round 6: the paired full passes' Gram (ts_tn_stream2_kernel) at 4 waves per SIMD
# (__launch_bounds__(256, 4): 128 VGPRs) instead of 3: kernel trace of cfg4 and cfg5 fits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_aa
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python -u tools/probe_block16.py 1000000 50 128 8:0:0,8:0:0 > $O/cfg4.log 2>&1 || { echo "cfg4 failed rc=$?"; tail -5 $O/cfg4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt5 -o run -- python -u tools/probe_block16.py 10000000 30 128 8:0:0 > $O/cfg5.log 2>&1 || { echo "cfg5 failed rc=$?"; tail -5 $O/cfg5.log; exit 1; }
echo done
