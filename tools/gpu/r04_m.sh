#!/bin/bash
# Round 4: dense_tn_kernel three stages in flight (triple-buffered loads) --
# dense tests, A/B, cfg3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -p no:cacheprovider -k "dense or cfg3" > gpurun_out/r04_m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dense_tn_probe.py --fits 2 > gpurun_out/r04_dense_tn6.jsonl 2> gpurun_out/r04_dense_tn6.err
rc=$?; cat gpurun_out/r04_dense_tn6.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r04_bench_cfg3_m.json 2> gpurun_out/r04_bench_cfg3_m.err
rc=$?; cut -c1-300 gpurun_out/r04_bench_cfg3_m.json; exit $rc
