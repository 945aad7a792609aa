set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/t1.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/sweep_eig.py 100000 64 20 "[[8,256,80],[8,192,72],[8,192,80],[8,224,80],[8,256,72],[8,256,96],[8,320,80],[8,160,72]]" > gpurun_out/sweep.log 2>&1
echo "exit=$?" >> gpurun_out/sweep.log
