#!/bin/bash
# Round 6: two register windows per wave (N2V2R_SPMM_NVW=2) against one: tests (bit-identical),
# cfg5-sized layer A/B, cfg5 fits A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_af
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "register_windows" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
timeout -k 10 200 python -u tools/spmm_env_ab.py 10000000 30 N2V2R_SPMM_NVW 1,2 3 > $O/layer_ab.jsonl 2>&1 || { echo "layer ab failed rc=$?"; tail -5 $O/layer_ab.jsonl; exit 1; }
timeout -k 10 400 python -u tools/probe_env_ab.py 10000000 30 N2V2R_SPMM_NVW 1,2 1 > $O/fit_ab.jsonl 2>&1 || { echo "fit ab failed rc=$?"; tail -5 $O/fit_ab.jsonl; exit 1; }
echo done
