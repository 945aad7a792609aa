#!/bin/bash
# Round 6: L2 hits / misses and fabric read requests of the cfg5-sized tiled SpMM at 64 blocks
# (64-row windows) and 128 blocks (128-row windows): is the 128-block form's loss an L2 matter?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_u
mkdir -p $O
for cfg in "64 6" "128 7"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex spmm8_flat_kernel --output-format csv -d $O/nb$1 -o run -- python -u tools/tile_nb_probe.py 10000000 30 $1 $2 > $O/nb$1.log 2>&1 || { echo "nb$1 failed rc=$?"; tail -5 $O/nb$1.log; exit 1; }
done
echo done
