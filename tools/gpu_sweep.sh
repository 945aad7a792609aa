set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep_eig.py 100000 64 20 "[[8,256,80,0],[8,256,80,1],[8,320,80,0],[8,320,80,1],[8,384,80,0],[8,224,80,0]]" > gpurun_out/sweep.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
echo "exit=$?" >> gpurun_out/tests.log
