#!/bin/bash
# Round 6: the persistent tile-synced flat SpMM (launches of more than one round of resident
# workgroups): tests (bit-identical to the one-round form), cfg5-sized layer launch with / without
# it, and its L2 hit rate
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "tile_sync or (test_spmm_tiled_flat_blocks and 6)" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
N2V2R_SPMM_TSYNC=0 timeout -k 10 200 python -u tools/tile_nb_probe.py 10000000 30 64,32 6 > $O/nb_off.jsonl 2>&1 || { echo "probe off failed rc=$?"; tail -5 $O/nb_off.jsonl; exit 1; }
timeout -k 10 200 python -u tools/tile_nb_probe.py 10000000 30 64,32,128 6 > $O/nb_on.jsonl 2>&1 || { echo "probe on failed rc=$?"; tail -5 $O/nb_on.jsonl; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex spmm8_flat_kernel --output-format csv -d $O/pmc_on -o run -- python -u tools/tile_nb_probe.py 10000000 30 64 6 > $O/pmc_on.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $O/pmc_on.log; exit 1; }
echo done
