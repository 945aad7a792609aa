# flat SpMM window scheduling A/B (N2V2R_FLAT_SCHED 0..3: static / per-phase counter / rp
# prefetch / both), one layer at cfg4 size, then cfg4 fits for 0 and 3; staged (pinned,
# threaded) host -> HBM uploads: ingest / dense tests and cfg3 / cfg4 API time A/B; cfg5 test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sched
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest_device.py tests/test_gpu_dense.py tests/test_ingest.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_ingest.log 2>&1 || { echo ingest-tests-failed; exit 1; }
for v in 0 1 2 3; do
  N2V2R_FLAT_SCHED=$v timeout -k 10 300 python -u tools/spmm16_probe.py --widths 8 > $O/probe_s$v.jsonl 2> $O/probe_s$v.err || { echo probe-fail-$v; exit 1; }
done
for v in 1 0; do
  N2V2R_H2D_STAGED=$v timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 1 --no-cpu-baseline > $O/cfg3_h$v.json 2> $O/cfg3_h$v.err || { echo cfg3-fail-$v; exit 1; }
done
for v in 3 0; do
  N2V2R_FLAT_SCHED=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg4_s$v.json 2> $O/cfg4_s$v.err || { echo bench-fail-$v; exit 1; }
done
timeout -k 10 300 python -u tools/api_breakdown.py --config cfg4 > $O/breakdown_cfg4.json 2>&1 || { echo bd4-fail; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -v -rf -s --timeout 280 --timeout-method thread -p no:cacheprovider -k "cfg5" > $O/tests.log 2>&1 || { echo tests-failed; exit 1; }
echo done
