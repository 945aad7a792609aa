#!/bin/bash
# Round 4 (session 2): non-temporal basis loads in the paired Gram and the fused PIP pass
# (N2V2R_BASIS_NT: unset = auto, nt beyond 256 MB of basis) -- cfg4 auto vs plain, cfg2 auto vs
# forced nt, alternating on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "paired_full_passes or column_blocks_er_20k" > gpurun_out/r04_nt_tests.log 2>&1 || { tail -20 gpurun_out/r04_nt_tests.log; exit 1; }
tail -2 gpurun_out/r04_nt_tests.log
for rep in 1 2; do
  for v in 0 auto; do
    if [ $v = auto ]; then unset N2V2R_BASIS_NT; else export N2V2R_BASIS_NT=$v; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --resident-steps 3 > gpurun_out/r04_nt4_$v.$rep.json 2> gpurun_out/r04_nt4_$v.$rep.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/r04_nt4_$v.$rep.json')); print('cfg4 nt=$v', d['ms_per_step'], d['device_resident']['ms_per_step'], d['eig']['block_applications'])"
  done
  for v in 1 auto; do
    if [ $v = auto ]; then unset N2V2R_BASIS_NT; else export N2V2R_BASIS_NT=$v; fi
    timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline --steps 10 --warmup 2 --resident-steps 10 > gpurun_out/r04_nt2_$v.$rep.json 2> gpurun_out/r04_nt2_$v.$rep.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/r04_nt2_$v.$rep.json')); print('cfg2 nt=$v', d['ms_per_step'], d['device_resident']['ms_per_step'], d['eig']['block_applications'])"
  done
done
unset N2V2R_BASIS_NT
