#!/bin/bash
# Round 4: wave-span tiled SpMM + multi-workgroup pip_chol: the tests that exercise them, the
# span/window A/B (layer launches and fits), cfg3 and cfg4 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --maxfail=3 --timeout 400 \
  --timeout-method thread -p no:cacheprovider \
  -k "spmm or block_widths or large_dimension or cfg3 or cfg4 or partitioned or rccl or paired" \
  > gpurun_out/r04_d_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r04_d_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/spmm_tiled_probe.py > gpurun_out/r04_span_ab.jsonl 2> gpurun_out/r04_span_ab.err
rc=$?; cat gpurun_out/r04_span_ab.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r04_bench_cfg3_d.json 2> gpurun_out/r04_bench_cfg3_d.err
rc=$?; cut -c1-300 gpurun_out/r04_bench_cfg3_d.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r04_bench_cfg4_d.json 2> gpurun_out/r04_bench_cfg4_d.err
rc=$?; cut -c1-400 gpurun_out/r04_bench_cfg4_d.json; exit $rc
