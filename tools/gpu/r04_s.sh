#!/bin/bash
# Round 4 (session 2): gather ceiling with the index stream software-pipelined; the pipelined
# flat SpMM (N2V2R_FLAT_PIPE=1) -- bit-identity tests, then cfg4 A/B (alternating, one box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/gather_ceiling 100 20 2 32 > gpurun_out/r04_gather_pipe.jsonl || exit $?
timeout -k 10 120 tools/gather_ceiling 100 20 8 32 >> gpurun_out/r04_gather_pipe.jsonl || exit $?
cat gpurun_out/r04_gather_pipe.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "flat_pipe or tiled_flat" > gpurun_out/r04_s_tests.log 2>&1 || { tail -30 gpurun_out/r04_s_tests.log; exit 1; }
tail -3 gpurun_out/r04_s_tests.log
for rep in 1 2; do
  for pv in 0 1; do
    N2V2R_FLAT_PIPE=$pv timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
      --resident-steps 3 > gpurun_out/r04_s_pipe$pv.$rep.json 2> gpurun_out/r04_s_pipe$pv.$rep.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/r04_s_pipe$pv.$rep.json')); print('pipe', $pv, d['ms_per_step'], d['device_resident']['ms_per_step'], d['roofline']['avg_launch_ms'], d['eig']['block_applications'])"
  done
done
