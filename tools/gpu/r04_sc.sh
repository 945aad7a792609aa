#!/bin/bash
# Round 4 (session 2): streaming-read ceiling (plain / nt / LDS-DMA) for the orthogonalisation passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/stream_ceiling 2 10 > gpurun_out/r04_stream_ceiling.jsonl || exit $?
cat gpurun_out/r04_stream_ceiling.jsonl
