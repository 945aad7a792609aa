#!/bin/bash
# Round 6: per-cycle residual history of the default fits at cfg4 and cfg5 (N2V2R_TRACE=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_y
mkdir -p $O
N2V2R_TRACE=1 timeout -k 10 120 python -u tools/probe_block16.py 1000000 50 128 8:0:0 > $O/cfg4.jsonl 2> $O/cfg4.trace || { echo "cfg4 failed rc=$?"; tail -5 $O/cfg4.trace; exit 1; }
N2V2R_TRACE=1 timeout -k 10 300 python -u tools/probe_block16.py 10000000 30 128 8:0:0 > $O/cfg5.jsonl 2> $O/cfg5.trace || { echo "cfg5 failed rc=$?"; tail -5 $O/cfg5.trace; exit 1; }
echo done
