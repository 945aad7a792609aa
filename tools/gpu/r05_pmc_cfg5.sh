#!/bin/bash
# Round 5: L2 hits / misses and fabric read requests of the tiled SpMM at cfg5 size (one ER layer,
# N = 10M, degree 30; 32 vs 64 column blocks, 64-row windows), one rocprofv3 --pmc run per block
# count (tools/tile_nb_probe.py: 2 rounds x 11 launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof_r05c5
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for nb in 32 64; do
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex spmm8_flat_kernel --output-format csv -d $O/nb$nb -o run -- python -u tools/tile_nb_probe.py 10000000 30 $nb 6 > $O/nb$nb.log 2>&1 || { echo "nb$nb failed rc=$?"; tail -5 $O/nb$nb.log; exit 1; }
done
echo done
