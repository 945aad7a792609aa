# Streaming Gram with LDS-staged Z rows (N2V2R_TN_LDS=1, default) vs unstaged: GPU suite,
# cfg4 kernel traces both ways, cfg4 / cfg2 fits both ways.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tnlds
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo tests-failed; exit 1; }
for v in 1 0; do
  N2V2R_TN_LDS=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt4_$v -o run -- python -u bench.py --config cfg4 --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline > $O/kt4_$v.log 2>&1 || { echo kt4-fail-$v; exit 1; }
done
for v in 1 0 1 0; do
  N2V2R_TN_LDS=$v timeout -k 10 300 python -u bench.py --config cfg2 --steps 1 --warmup 1 --resident-steps 20 --no-cpu-baseline > $O/cfg2_$v.$RANDOM.json 2> $O/cfg2_$v.err || { echo cfg2-fail-$v; exit 1; }
done
for v in 1 0; do
  N2V2R_TN_LDS=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 3 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || { echo cfg4-fail-$v; exit 1; }
done
echo done
