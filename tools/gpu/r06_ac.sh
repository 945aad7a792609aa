#!/bin/bash
# Round 6: cfg4-shape kept set / basis sensitivity over four graphs (seed bases 1000 = the
# bench's, 2000, 3000, 4000): block applications and fit seconds per combination
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_ac
mkdir -p $O
for sd in 1000 2000 3000 4000; do
  PROBE_SEED=$sd timeout -k 10 200 python -u tools/probe_block16.py 1000000 50 128 8:168:640,8:168:704,8:168:768,8:160:640,8:176:640,8:184:704,8:168:576 > $O/seed$sd.jsonl 2>&1 || { echo "seed $sd failed rc=$?"; tail -5 $O/seed$sd.jsonl; exit 1; }
done
echo done
