#!/bin/bash
# Round 6: register-window tiles of the flat SpMM (each wave also keeps one 64-row window in
# VGPRs; more rows in flight per round): tests (bit-identical), cfg5-sized layer A/B, its L2
# hit rate, then cfg5 fits A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_ae
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "register_windows or test_spmm_tiled_flat_blocks" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
timeout -k 10 200 python -u tools/spmm_env_ab.py 10000000 30 N2V2R_SPMM_VW 0,1 3 > $O/layer_ab.jsonl 2>&1 || { echo "layer ab failed rc=$?"; tail -5 $O/layer_ab.jsonl; exit 1; }
N2V2R_SPMM_VW=1 timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex spmm8_flat_kernel --output-format csv -d $O/pmc_vw -o run -- python -u tools/tile_nb_probe.py 10000000 30 64 6 > $O/pmc_vw.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $O/pmc_vw.log; exit 1; }
timeout -k 10 400 python -u tools/probe_env_ab.py 10000000 30 N2V2R_SPMM_VW 0,1 1 > $O/fit_ab.jsonl 2>&1 || { echo "fit ab failed rc=$?"; tail -5 $O/fit_ab.jsonl; exit 1; }
echo done
