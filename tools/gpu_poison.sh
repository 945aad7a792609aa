# hunt uninitialised / stale reads: GPU parity + dense tests with NaN-poisoned allocations and
# scratch, every eigensolver stage checked for non-finite output (N2V2R_DEBUG_FINITE)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/poison
mkdir -p $O
export TMPDIR=/tmp
export N2V2R_POISON=1 N2V2R_DEBUG_FINITE=1
timeout -k 10 600 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dense.py -m gpu > $O/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 $O/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/stress_b16.py 3 > $O/stress.log 2>&1 || { echo stress-fail; tail -20 $O/stress.log; exit 1; }
tail -5 $O/stress.log
