#!/bin/bash
# Round 4 (session 2): the tiled SpMM with the next phase's panel block prefetched into L2
# (N2V2R_FLAT_PF=1): tiled-SpMM tests under it, then cfg4 A/B (alternating on one box)
set -o pipefail
mkdir -p gpurun_out
N2V2R_FLAT_PF=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "tiled_flat or column_blocks" > gpurun_out/r04_w_tests.log 2>&1 || { tail -30 gpurun_out/r04_w_tests.log; exit 1; }
tail -3 gpurun_out/r04_w_tests.log
for rep in 1 2; do
  for pv in 0 1; do
    N2V2R_FLAT_PF=$pv timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
      --resident-steps 3 > gpurun_out/r04_w_pf$pv.$rep.json 2> gpurun_out/r04_w_pf$pv.$rep.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/r04_w_pf$pv.$rep.json')); print('pf', $pv, d['ms_per_step'], d['device_resident']['ms_per_step'], d['roofline']['avg_launch_ms'], d['eig']['block_applications'])"
  done
done
