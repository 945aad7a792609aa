# Final verification: smoke(), the whole GPU suite, API breakdowns (cfg2, cfg4).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/verify
mkdir -p $O
export TMPDIR=/tmp
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider --durations=10 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg2 > $O/breakdown_cfg2.json 2>&1 || { echo bd2-fail; exit 1; }
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg4 > $O/breakdown_cfg4.json 2>&1 || { echo bd4-fail; exit 1; }
echo verify-done
