#!/bin/bash
# Round 4 (session 2): lean images (default) against every image kept (N2V2R_LEAN_W=0) at cfg4
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 1 0; do
    N2V2R_LEAN_W=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --resident-steps 3 > gpurun_out/r04_lean_$v.$rep.json 2> gpurun_out/r04_lean_$v.$rep.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/r04_lean_$v.$rep.json')); print('cfg4 lean=$v', d['ms_per_step'], d['device_resident']['ms_per_step'], d['eig']['block_applications'], d['eig']['restarts'])"
  done
done
