#!/bin/bash
# Round 4: dense_tn default -- dense / cfg3 tests, fit A/B against the LDS-staged GEMM, cfg3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "dense or cfg3 or block_widths" \
  > gpurun_out/r04_k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dense_tn_probe.py --fits 2 > gpurun_out/r04_dense_tn4.jsonl 2> gpurun_out/r04_dense_tn4.err
rc=$?; cat gpurun_out/r04_dense_tn4.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r04_bench_cfg3_k.json 2> gpurun_out/r04_bench_cfg3_k.err
rc=$?; cut -c1-300 gpurun_out/r04_bench_cfg3_k.json; exit $rc
