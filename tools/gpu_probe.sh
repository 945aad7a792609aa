set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe -o run -- python3 tools/spmm_probe.py > gpurun_out/probe/probe.log 2>&1
