# flat SpMM workgroup size A/B: 1024 threads (2 per CU) vs 512 (4 per CU, half the tile rows);
# dense GEMM with two A tiles in flight (N2V2R_DG_PD=2) vs one.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wg
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 ./tools/graph_probe > $O/graph_probe.txt 2>&1 || { echo graph-probe-fail; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider -k "tiled_flat_widths or paired" > $O/tests_new.log 2>&1 || { echo new-tests-failed; exit 1; }
for v in 512 1024 512; do
  N2V2R_FLAT_WG=$v timeout -k 10 300 python -u tools/spmm16_probe.py --widths 8 > $O/probe_$v.$RANDOM.jsonl 2> $O/probe_$v.err || { echo probe-fail-$v; exit 1; }
done
for v in 512 1024; do
  N2V2R_FLAT_WG=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 3 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || { echo cfg4-fail-$v; exit 1; }
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_dense.log 2>&1 || { echo dense-tests-failed; exit 1; }
N2V2R_DG_PD=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_dense_pd2.log 2>&1 || { echo dense-pd2-tests-failed; exit 1; }
for v in 2 1 2 1; do
  N2V2R_DG_PD=$v timeout -k 10 300 python -u bench.py --config cfg3 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg3_pd$v.$RANDOM.json 2> $O/cfg3_pd$v.err || { echo cfg3-fail-$v; exit 1; }
done
echo done
