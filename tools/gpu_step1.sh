set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/t1.log 2>&1
echo "exit=$?" >> gpurun_out/t1.log
