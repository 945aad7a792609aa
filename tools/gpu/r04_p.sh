#!/bin/bash
# Round 4: cfg3 basis / keep candidates on two more members of the graph family
set -o pipefail
mkdir -p gpurun_out
for sb in 100 200; do
  timeout -k 10 300 python -u tools/sweep_cfg3.py --seed-base $sb --reps 1 \
    --pairs 320:768 288:704 320:640 352:768 288:640 320:704 >> gpurun_out/r04_cfg3_sweep2.jsonl 2> gpurun_out/r04_cfg3_sweep2.err || exit $?
done
cat gpurun_out/r04_cfg3_sweep2.jsonl
