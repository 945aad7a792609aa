#!/bin/bash
# Round 6: paired mode against the reference fixtures (er_cfg2, er_cfg4g); fabric read requests
# of the b = 16 and b = 8 tiled SpMM at cfg5's layer size (one PMC pass, both kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair.py -x -v -s --timeout 300 --timeout-method thread > $O/pair_tests.log 2>&1 || { echo "pair tests failed rc=$?"; tail -30 $O/pair_tests.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex "spmm(8|16)_flat_kernel" --output-format csv -d $O/pmc -o run -- python -u tools/probe_spmm16.py 10000000 30 8:64:0,16:16:0 > $O/pmc.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $O/pmc.log; exit 1; }
echo done
