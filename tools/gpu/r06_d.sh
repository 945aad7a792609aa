#!/bin/bash
# Round 6: paired-panel mode, first run: cfg2-size graph with the tiled SpMM forced (traced),
# then cfg4's graph, 8-wide vs paired fits
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_d
mkdir -p $O
N2V2R_SPMM_CB=1 N2V2R_TRACE=1 timeout -k 10 120 python -u tools/probe_pair.py 100000 20 64 1 16,8 > $O/cfg2.jsonl 2> $O/cfg2.err || { echo "cfg2 failed rc=$?"; tail -30 $O/cfg2.err; exit 1; }
timeout -k 10 300 python -u tools/probe_pair.py 1000000 50 128 2 8,16 > $O/cfg4.jsonl 2> $O/cfg4.err || { echo "cfg4 failed rc=$?"; tail -30 $O/cfg4.err; exit 1; }
echo done
