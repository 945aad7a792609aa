# hunt the intermittent block-16 non-convergence: the test selection it appeared in, N times
# in fresh processes, with the solver trace on (stderr kept in the log)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/flake
export TMPDIR=/tmp
for i in $(seq 1 ${FLAKE_N:-5}); do
  N2V2R_TRACE=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x -s -k "${TESTK:-band_stage or uase or rayleigh}" --timeout 120 --timeout-method thread > gpurun_out/flake/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc" >> gpurun_out/flake/summary.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
