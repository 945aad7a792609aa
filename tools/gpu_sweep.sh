set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profeig
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "band_stage" --timeout 120 --timeout-method thread > gpurun_out/band.log 2>&1 || { echo band-fail; exit 1; }
timeout -k 10 300 python -u tools/sweep_eig.py 100000 64 20 "[[0,0,0,0],[0,0,0,2],[0,256,0,0]]" > gpurun_out/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
timeout -k 10 300 python -u tools/sweep_eig.py 200000 128 30 "[[0,0,0,0],[0,0,0,2]]" >> gpurun_out/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profeig -o run -- python3 tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" > gpurun_out/profeig/sweep.log 2>&1 || { echo prof-fail; exit 1; }
find gpurun_out/profeig -name "*kernel_trace.csv" -delete
