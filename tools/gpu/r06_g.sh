#!/bin/bash
# Round 6: multi-GPU API tests (host row slices for symmetric and directed layers, the per-rank
# upload counter, a rank failing alone), then the paired-panel fits at cfg4 and cfg5 (r06_f.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -x -v -s --timeout 180 --timeout-method thread > $O/multi_tests.log 2>&1 || { echo "multi tests failed rc=$?"; tail -40 $O/multi_tests.log; exit 1; }
bash tools/gpu/r06_f.sh
