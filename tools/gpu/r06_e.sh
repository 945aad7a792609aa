#!/bin/bash
# Round 6: b = 16 flat tiled SpMM with 2048-row tiles, one workgroup per CU (libn2v2r_hip_w1.so,
# -DN2V2R_SPMM16_WPC=1) against the 1024-row, two-per-CU form, at cfg4's and cfg5's layer sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_e
mkdir -p $O
timeout -k 10 150 python -u tools/probe_spmm16.py 1000000 50 8:16:0,16:16:0,16:32:0 > $O/cfg4_w2.jsonl 2>&1 || { echo "w2 cfg4 failed"; tail -5 $O/cfg4_w2.jsonl; exit 1; }
N2V2R_LIB=node2vec2rank_amd/lib/libn2v2r_hip_w1.so timeout -k 10 150 python -u tools/probe_spmm16.py 1000000 50 16:16:0,16:32:0,16:8:0 > $O/cfg4_w1.jsonl 2>&1 || { echo "w1 cfg4 failed"; tail -5 $O/cfg4_w1.jsonl; exit 1; }
N2V2R_LIB=node2vec2rank_amd/lib/libn2v2r_hip_w1.so timeout -k 10 400 python -u tools/probe_spmm16.py 10000000 30 16:32:0,16:64:0,16:16:0 > $O/cfg5_w1.jsonl 2>&1 || { echo "w1 cfg5 failed"; tail -5 $O/cfg5_w1.jsonl; exit 1; }
echo done
