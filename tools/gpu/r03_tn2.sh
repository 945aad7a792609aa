# Two-block Gram with Z rows staged through LDS: tests touching the paired passes, cfg4 / cfg2
# kernel traces (ts_tn_stream2_kernel average against 353 / 26 us before), cfg4 / cfg2 fits.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tn2
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "paired or uase or cfg4 or cfg5 or dist or partition" > $O/tests.log 2>&1 || { echo tests-failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt4 -o run -- python -u bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > $O/kt4.log 2>&1 || { echo kt4-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2 -o run -- python -u bench.py --config cfg2 --steps 3 --warmup 1 --resident-steps 3 --no-cpu-baseline > $O/kt2.log 2>&1 || { echo kt2-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 3 --no-cpu-baseline > $O/cfg4.json 2> $O/cfg4.err || { echo cfg4-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg2 --steps 3 --warmup 1 --resident-steps 20 --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.err || { echo cfg2-fail; exit 1; }
echo done
