#!/bin/bash
# Round 4 (session 2): the flat SpMM with one 8-B index load per lane (N2V2R_FLAT_X2=1):
# bit-identity tests, then cfg4 A/B (alternating on one box); dense GEMM 2x-MFMA probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "flat_x2 or tiled_flat or column_blocks" > gpurun_out/r04_u_tests.log 2>&1 || { tail -30 gpurun_out/r04_u_tests.log; exit 1; }
tail -3 gpurun_out/r04_u_tests.log
for rep in 1 2; do
  for xv in 0 1; do
    N2V2R_FLAT_X2=$xv timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
      --resident-steps 3 > gpurun_out/r04_u_x2$xv.$rep.json 2> gpurun_out/r04_u_x2$xv.$rep.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/r04_u_x2$xv.$rep.json')); print('x2', $xv, d['ms_per_step'], d['device_resident']['ms_per_step'], d['roofline']['avg_launch_ms'], d['eig']['block_applications'])"
  done
done
# dense GEMM: 2x MFMAs per streamed byte (bytes- or MFMA-bound? VERDICT r03 item 4)
timeout -k 10 200 python -u tools/dense_dup_probe.py > gpurun_out/r04_dense_dup.jsonl 2> gpurun_out/r04_dense_dup.err || exit $?
cat gpurun_out/r04_dense_dup.jsonl
