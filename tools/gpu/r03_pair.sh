# Paired full passes: kernel traces of cfg2 / cfg4 fits with N2V2R_REORTH_DEFER=1 (pair Gram)
# and with the two passes one by one, the default beside them; the GPU tests under the switch;
# cfg3 API breakdown (sampled density test).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pair
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
B2="bench.py --config cfg2 --steps 3 --warmup 1 --resident-steps 3 --no-cpu-baseline"
N2V2R_REORTH_DEFER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2p -o run -- python -u $B2 > $O/kt2p.log 2>&1 || { echo kt2p-fail; exit 1; }
N2V2R_REORTH_DEFER=1 N2V2R_REORTH_PAIR=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2e -o run -- python -u $B2 > $O/kt2e.log 2>&1 || { echo kt2e-fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2d -o run -- python -u $B2 > $O/kt2d.log 2>&1 || { echo kt2d-fail; exit 1; }
for v in 1 0; do
  N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg4_d$v.json 2> $O/cfg4_d$v.err || { echo cfg4-fail-$v; exit 1; }
done
N2V2R_REORTH_DEFER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_defer.log 2>&1
echo "pytest rc=$?" >> $O/tests_defer.log
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg3 > $O/breakdown_cfg3.json 2>&1 || { echo bd3-fail; exit 1; }
echo done
