set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/t1.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/t1.log; exit $rc
