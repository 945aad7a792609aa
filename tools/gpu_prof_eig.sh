set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profeig
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profeig -o run -- python3 tools/sweep_eig.py 100000 64 20 "${SWEEP:-[[8,256,80,0]]}" > gpurun_out/profeig/sweep.log 2>&1
rc=$?
find gpurun_out/profeig -name "*kernel_trace.csv" -delete
exit $rc
