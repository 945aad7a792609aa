# Whole GPU suite + rank-agreement probe, then the round-3 bench lines and API wall times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/full
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/full/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider --durations=10 > gpurun_out/full/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/full/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
timeout -k 10 400 python -u tools/parity_probe.py > gpurun_out/full/parity.jsonl 2> gpurun_out/full/parity.err || { echo parity-fail; exit 1; }
bash tools/gpu/r03_final.sh || exit 1
echo full-done
