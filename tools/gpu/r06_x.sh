#!/bin/bash
# Round 6 diagnostic: L2 hit rate of the flat tiled SpMM against rounds of tiles and block size
# (N = 1M / 4M / 10M, degree 30; 16 / 64 column blocks): is cfg5's 0.25 a matter of rounds,
# of phase length or of block size?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_x
mkdir -p $O
for cfg in "1000000 16" "1000000 64" "4000000 64" "4000000 32"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex spmm8_flat_kernel --output-format csv -d $O/n$1_nb$2 -o run -- python -u tools/tile_nb_probe.py $1 30 $2 6 > $O/n$1_nb$2.log 2>&1 || { echo "n$1 nb$2 failed rc=$?"; tail -5 $O/n$1_nb$2.log; exit 1; }
done
echo done
