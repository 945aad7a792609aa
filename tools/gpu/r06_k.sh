#!/bin/bash
# Round 6: the symmetric dense form (dense_sym_kernel) -- numerics, then cfg3 fits A/B against
# the full-matrix dense_tn form, then the cfg3 kernel trace with it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 120 --timeout-method thread -k "sym or dense_gemm" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
for v in 1 0 1 0; do
  N2V2R_DENSE_SYM=$v timeout -k 10 200 python -u tools/probe_cfg3.py cfg3 >> $O/ab.txt 2>&1 || { echo "cfg3 probe failed"; tail -20 $O/ab.txt; exit 1; }
  echo "^ N2V2R_DENSE_SYM=$v" >> $O/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python -u tools/probe_cfg3.py cfg3 > $O/kt.log 2>&1 || { echo "kt failed rc=$?"; tail -5 $O/kt.log; exit 1; }
echo done
