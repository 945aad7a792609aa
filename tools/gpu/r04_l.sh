#!/bin/bash
# Round 4: dense_tn_kernel without the mid-loop exit (next half's loads no longer sunk below the
# MFMAs) -- dense tests, A/B, cfg3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "dense or cfg3" > gpurun_out/r04_l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dense_tn_probe.py --fits 2 > gpurun_out/r04_dense_tn5.jsonl 2> gpurun_out/r04_dense_tn5.err
rc=$?; cat gpurun_out/r04_dense_tn5.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r04_bench_cfg3_l.json 2> gpurun_out/r04_bench_cfg3_l.err
rc=$?; cut -c1-300 gpurun_out/r04_bench_cfg3_l.json; exit $rc
