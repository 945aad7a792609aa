set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rr
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rr/prof -o run -- python3 tools/bench_rr.py ${RRARGS:-384 80 88 5} > gpurun_out/rr/bench.log 2>&1 || { echo rr-fail; exit 1; }
find gpurun_out/rr/prof -name "*kernel_trace.csv" -delete
