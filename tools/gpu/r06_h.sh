#!/bin/bash
# Round 6: the new GPU tests (paired mode, chunked reduce-scatter), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py "tests/test_gpu_dist.py::test_rs_chunks_bit_identical" -x -v -s --timeout 180 --timeout-method thread > $O/new_tests.log 2>&1 || { echo "new tests failed rc=$?"; tail -40 $O/new_tests.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "suite failed rc=$?"; tail -40 $O/gpu_suite.log; exit 1; }
tail -3 $O/gpu_suite.log
