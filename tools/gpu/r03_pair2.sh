# Paired full passes on by default: smoke, the whole GPU suite, cfg2 trace (fixup kernel), cfg2
# and cfg4 bench lines with the pairing on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pair2
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-fail; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider --durations=5 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
B2="bench.py --config cfg2 --steps 3 --warmup 1 --resident-steps 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2 -o run -- python -u $B2 > $O/kt2.log 2>&1 || { echo kt2-fail; exit 1; }
for v in 1 0; do
  N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg2 --steps 10 --warmup 2 --resident-steps 10 --no-cpu-baseline > $O/cfg2_d$v.json 2> $O/cfg2_d$v.err || { echo cfg2-fail-$v; exit 1; }
  N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg4_d$v.json 2> $O/cfg4_d$v.err || { echo cfg4-fail-$v; exit 1; }
done
echo done
