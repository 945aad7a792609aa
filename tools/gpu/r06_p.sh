#!/bin/bash
# Round 6: kept sets past the reducing band path's arrow on the lean Sturm path (dense
# Rayleigh-Ritz from the expanded band as its fallback): the new tests, then block applications
# and fit time over keep at cfg5 (N = 10M) and at N = 3M
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "sturm_failure or large_kept" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
bash tools/gpu/steps.sh $O basis:3000000:30:128:8:0:640,8:224:640 basis:10000000:30:128:8:0:640,8:200:640,8:224:640,8:256:640
