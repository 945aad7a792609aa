# Deferred full passes (N2V2R_REORTH_DEFER=1, numerics of a paired full pass): cfg2 / cfg4
# applications, residuals and time vs the default; parity subset under the switch; cfg3 API
# breakdown with the pinned staged upload on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/defer
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
N2V2R_REORTH_DEFER=1 N2V2R_REORTH_PAIR=0 timeout -k 10 300 python -u bench.py --config cfg2 --steps 5 --warmup 1 --resident-steps 5 --no-cpu-baseline > $O/cfg2_pair0.json 2> $O/cfg2_pair0.err || { echo cfg2-pair0-fail; exit 1; }
for v in 1 0; do
  N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg2 --steps 5 --warmup 1 --resident-steps 5 --no-cpu-baseline > $O/cfg2_d$v.json 2> $O/cfg2_d$v.err || { echo cfg2-fail-$v; exit 1; }
done
for v in 1 0; do
  N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg4_d$v.json 2> $O/cfg4_d$v.err || { echo cfg4-fail-$v; exit 1; }
done
N2V2R_REORTH_DEFER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "uase or end_to_end or cfg4_full" > $O/tests_defer.log 2>&1
echo "pytest rc=$?" >> $O/tests_defer.log
for v in 1 0; do
  N2V2R_H2D_STAGED=$v timeout -k 10 300 python -u tools/api_breakdown.py --config cfg3 > $O/breakdown_cfg3_h$v.json 2>&1 || { echo bd3-fail-$v; exit 1; }
done
echo done
