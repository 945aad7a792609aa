#!/bin/bash
# Round 5, BASELINE cfg2 (2-layer ER N = 100k, d = 64): kernel trace of the bench's own fits, to
# count the launches per block application and their gaps (the launch-bound part of the fit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_r05c2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python -u bench.py --config cfg2 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/kt.log 2>&1 || { echo "kt failed rc=$?"; tail -5 $O/kt.log; exit 1; }
echo done
