#!/bin/bash
# Round 4 (session 2): tiled SpMM column-block count at cfg5's size (one layer, N = 10M, degree 30)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u tools/tile_nb_probe.py 10000000 30 8,16,32,64 > gpurun_out/r04_tile_nb_cfg5.jsonl 2>&1
