#!/bin/bash
# Round 6: the flat tiled SpMM at b = 16 against b = 8 at BASELINE cfg5's size (one ER layer,
# N = 10M, degree 30): ms per layer launch over column-block counts, the b = 16 result vs scipy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_a
mkdir -p $O
timeout -k 10 500 python -u tools/probe_spmm16.py 10000000 30 8:64:0,16:64:0,16:32:0,16:16:0 > $O/spmm16_cfg5.jsonl 2>&1 || { echo "probe failed rc=$?"; tail -5 $O/spmm16_cfg5.jsonl; exit 1; }
echo done
