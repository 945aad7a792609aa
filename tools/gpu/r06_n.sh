#!/bin/bash
# Round 6: 128 column blocks (2.5 MB panel blocks at cfg5: inside one XCD's 4 MB L2 beside the
# index stream) against 64, windows of 64 / 128 rows, one cfg5-sized layer
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_n
mkdir -p $O
timeout -k 10 500 python -u tools/tile_nb_probe.py 10000000 30 64,128 6,7 > $O/tile_cfg5.jsonl 2>&1 || { echo "probe failed rc=$?"; tail -5 $O/tile_cfg5.jsonl; exit 1; }
echo done
