#!/bin/bash
# Round 4 (session 2): keep / basis on the current build -- cfg4 (two graphs), cfg2 (two graphs),
# cfg5 at one GPU (keep 160 vs 176)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04_keep_sweep.jsonl
: > $O
for sb in 2000 3000; do
  timeout -k 10 300 python -u tools/sweep_big.py 1000000 50 128 '[[160,512],[168,512],[176,512],[184,512],[176,480],[160,512],[176,512]]' 60 $sb >> $O 2>> gpurun_out/r04_keep_sweep.err || exit $?
  timeout -k 10 200 python -u tools/sweep_big.py 100000 20 64 '[[80,384],[88,384],[96,384],[88,424],[80,384],[88,384]]' 60 $sb >> $O 2>> gpurun_out/r04_keep_sweep.err || exit $?
done
cat $O
timeout -k 10 400 python -u tools/sweep_big.py 10000000 30 128 '[[160,512],[176,512]]' 60 2000 >> $O 2>> gpurun_out/r04_keep_sweep.err || exit $?
tail -2 $O
