# Kernel-trace profile of the b = 16 cfg4 fit (where its non-SpMM time goes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/b16
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python -u tools/probe_block.py --config cfg4 --blocks 16 > $O/kt.log 2>&1 || { echo b16-prof-fail; exit 1; }
echo b16-done
