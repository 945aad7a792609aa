#!/bin/bash
# Round 4 (session 2): fused PIP pass against pip_chol + the apply (N2V2R_PIP_FUSED=0) at cfg4 and
# cfg5-size rows, alternating on one box (the fused form repeats the Gram staging and the 8 x 8
# Cholesky in every workgroup)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 1 0; do
    N2V2R_PIP_FUSED=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --resident-steps 3 > gpurun_out/r04_pf2_$v.$rep.json 2> gpurun_out/r04_pf2_$v.$rep.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/r04_pf2_$v.$rep.json')); print('cfg4 fused=$v', d['ms_per_step'], d['device_resident']['ms_per_step'], d['eig']['block_applications'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_pf2_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/trace_fit.py 1000000 50 128 1000 > /dev/null 2>&1 || exit $?
N2V2R_PIP_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04_pf2_prof0 -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/trace_fit.py 1000000 50 128 1000 > /dev/null 2>&1 || exit $?
echo fused-prof-ok
