# poison test + the full GPU suite three times with every eigensolver stage checked for
# non-finite output (hunting the intermittent b = 16 non-finite Ritz value; the first stage
# that produces one is named in the log)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/flake2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_poison.py tests/test_gpu_parity.py -m gpu > $O/poison.log 2>&1 || { echo poison-fail; tail -30 $O/poison.log; exit 1; }
tail -2 $O/poison.log
for i in 1 2 3; do
  N2V2R_DEBUG_FINITE=1 timeout -k 10 400 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests -m gpu > $O/suite$i.log 2>&1
  rc=$?
  echo "suite $i rc=$rc $(tail -1 $O/suite$i.log)"
  grep -h "non-finite\|WARNING" $O/suite$i.log | head -5
  if [ $rc -gt 1 ]; then exit $rc; fi
done
