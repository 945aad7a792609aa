#!/bin/bash
# Round 6: bases up to 768 columns on the lean fused banded path: the new tests, then block
# applications and fit time over keep x basis at cfg4 and cfg5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "sturm_failure or large_kept or basis_768" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
bash tools/gpu/steps.sh $O basis:1000000:50:128:8:0:640,8:0:768,8:224:768,8:256:768 basis:10000000:30:128:8:224:768,8:256:768,8:288:768
