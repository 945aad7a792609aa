set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- python3 tools/spmm_probe.py > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o run -- python3 tools/spmm_probe.py > gpurun_out/pmc/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/trace -o run -- python3 tools/spmm_probe.py > gpurun_out/pmc/trace.log 2>&1
