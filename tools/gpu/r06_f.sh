#!/bin/bash
# Round 6: paired-panel fits with the 64-B-row column-block rule: cfg4 (32 blocks) and cfg5 on
# one GPU (16 blocks), each against the 8-wide fit
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_f
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 200 python -u tools/probe_pair.py 1000000 50 128 1 16 > $O/cfg4.jsonl 2> $O/cfg4.err || { echo "cfg4 failed rc=$?"; tail -30 $O/cfg4.err; exit 1; }
timeout -k 10 400 python -u tools/probe_pair.py 10000000 30 128 1 16,8 > $O/cfg5.jsonl 2> $O/cfg5.err || { echo "cfg5 failed rc=$?"; tail -30 $O/cfg5.err; exit 1; }
echo done
