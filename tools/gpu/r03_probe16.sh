# b = 16 flat SpMM probe (vs b = 8; fold-skipped timing variant), cfg3 dense GEMM with X
# prefetched, then smoke + the GPU suite and the b = 16 fit profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/p16
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u tools/spmm16_probe.py > $O/probe.jsonl 2> $O/probe.err || { echo probe-fail; exit 1; }
N2V2R_FLAT_NOFOLD=1 timeout -k 10 300 python -u tools/spmm16_probe.py > $O/probe_nofold.jsonl 2> $O/probe_nofold.err || { echo probe-nofold-fail; exit 1; }
N2V2R_T16_ROWS=512 timeout -k 10 300 python -u tools/spmm16_probe.py > $O/probe_t512.jsonl 2> $O/probe_t512.err || { echo probe-t512-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg3.json 2> $O/cfg3.err || { echo cfg3-fail; exit 1; }
echo probes-done
