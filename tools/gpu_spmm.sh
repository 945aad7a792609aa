set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spmm" --timeout 120 --timeout-method thread > gpurun_out/spmm_t.log 2>&1 || { echo spmm-fail; exit 1; }
timeout -k 10 120 python -u tools/spmm_probe.py > gpurun_out/probe_v2.log 2>&1 || exit 1
N2V2R_SPMM_V1=1 timeout -k 10 120 python -u tools/spmm_probe.py > gpurun_out/probe_v1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" > gpurun_out/sweep.log 2>&1 || exit 1
N2V2R_SPMM_V1=1 timeout -k 10 300 python -u tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" >> gpurun_out/sweep.log 2>&1 || exit 1
