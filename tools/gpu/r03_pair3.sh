# Paired full passes A/B on one box, alternating: cfg2 (basis in the Infinity Cache) and cfg4
# (basis in HBM), device-resident fits.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pair3
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for rep in 1 2; do
  for v in 1 0; do
    N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg2 --steps 1 --warmup 1 --resident-steps 20 --no-cpu-baseline > $O/cfg2_d${v}_r$rep.json 2> $O/cfg2_d${v}_r$rep.err || { echo cfg2-fail-$v; exit 1; }
  done
done
for rep in 1 2; do
  for v in 1 0; do
    N2V2R_REORTH_DEFER=$v timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 3 --no-cpu-baseline > $O/cfg4_d${v}_r$rep.json 2> $O/cfg4_d${v}_r$rep.err || { echo cfg4-fail-$v; exit 1; }
  done
done
echo done
