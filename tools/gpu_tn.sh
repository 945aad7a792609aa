set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tn
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "uase" --timeout 120 --timeout-method thread > gpurun_out/tn/tests.log 2>&1 || { echo tests-fail; exit 1; }
for cfg in "lines 2048" "stream 2048" "stream 4096" "stream 8192" "stream 1024"; do
  set -- $cfg
  echo "== $1 $2" >> gpurun_out/tn/sweep.log
  N2V2R_TN_FORM=$1 N2V2R_TN_WAVES=$2 timeout -k 10 200 python -u tools/sweep_eig.py 100000 64 20 "[[0,0,0,0]]" >> gpurun_out/tn/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
done
