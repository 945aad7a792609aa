set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace1 -o run -- python3 tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" > gpurun_out/trace1/sweep.log 2>&1
