# flat-window SpMM: non-temporal index stream A/B at cfg4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nt
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/nt/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for v in 1 0 1; do
  N2V2R_FLAT_NT=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/nt/cfg4_nt$v.$RANDOM.json 2> gpurun_out/nt/cfg4_nt$v.err || { echo bench-fail-$v; exit 1; }
done
echo done
