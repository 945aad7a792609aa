# Fused PIP with 512-row workgroups (N2V2R_PIP_ROWS=512) vs 256: tests under the switch, cfg4 / cfg2
# fits alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pip
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
N2V2R_PIP_ROWS=512 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "uase or cfg4_full or paired" > $O/tests.log 2>&1 || { echo tests-failed; exit 1; }
for v in 512 256 512 256; do
  N2V2R_PIP_ROWS=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg4_$v.$RANDOM.json 2> $O/cfg4_$v.err || { echo cfg4-fail-$v; exit 1; }
done
for v in 512 256; do
  N2V2R_PIP_ROWS=$v timeout -k 10 300 python -u bench.py --config cfg2 --steps 1 --warmup 1 --resident-steps 20 --no-cpu-baseline > $O/cfg2_$v.json 2> $O/cfg2_$v.err || { echo cfg2-fail-$v; exit 1; }
done
echo done
