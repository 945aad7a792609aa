#!/bin/bash
# Round 5, BASELINE cfg2 (2-layer ER N = 100k, d = 64): kernel trace of the bench's own fits, to
# count the launches per block application and their gaps (the launch-bound part of the fit);
# before it, fit time and applications against the basis size
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_r05c2
mkdir -p $O
timeout -k 10 200 python -u tools/probe_block16.py 100000 20 64 8:0:0,8:0:0,8:0:320,8:0:448,8:0:512,8:0:576,8:0:640,8:0:0,8:0:448,8:0:512 > $O/basis.jsonl 2>&1 || { echo "basis probe failed rc=$?"; tail -5 $O/basis.jsonl; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python -u bench.py --config cfg2 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/kt.log 2>&1 || { echo "kt failed rc=$?"; tail -5 $O/kt.log; exit 1; }
echo done
