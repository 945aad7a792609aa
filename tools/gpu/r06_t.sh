#!/bin/bash
# Round 6: the paired full passes' two-block Gram at N = 10M (chunk partials sized for it): the
# cfg5 tests, the cfg5 bench line, a cfg5 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 400 --timeout-method thread -k "cfg5" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
bash tools/gpu/steps.sh $O bench:cfg5 kt:cfg5
