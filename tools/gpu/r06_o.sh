#!/bin/bash
# Round 6: block applications against basis size and kept vectors (b = 8) at cfg4 and cfg5;
# bases past 640 take the dense Rayleigh-Ritz, so only their application counts matter here
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_o
mkdir -p $O
timeout -k 10 120 python -u tools/probe_block16.py 1000000 50 128 8:0:640,8:0:768,8:224:768 > $O/basis_cfg4.jsonl 2>&1 || { echo "cfg4 probe failed rc=$?"; tail -5 $O/basis_cfg4.jsonl; exit 1; }
timeout -k 10 600 python -u tools/probe_block16.py 10000000 30 128 8:0:640,8:0:768,8:224:640 > $O/basis_cfg5.jsonl 2>&1 || { echo "cfg5 probe failed rc=$?"; tail -5 $O/basis_cfg5.jsonl; exit 1; }
echo done
