#!/bin/bash
# Round 4 (session 2): cfg2 basis around the new keep (two graphs); cfg5 one GPU at the new default
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04_keep_sweep2.jsonl
: > $O
for sb in 2000 3000 4000; do
  timeout -k 10 200 python -u tools/sweep_big.py 100000 20 64 '[[88,384],[88,352],[88,320],[96,352],[96,416],[104,416],[80,320]]' 60 $sb >> $O 2>> gpurun_out/r04_keep_sweep2.err || exit $?
done
cat $O
timeout -k 10 400 python -u tools/sweep_big.py 10000000 30 128 '[[168,512]]' 60 2000 >> $O 2>> gpurun_out/r04_keep_sweep2.err || exit $?
tail -1 $O
