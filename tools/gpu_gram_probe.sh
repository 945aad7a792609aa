# orthogonalisation Gram timing: per-kernel stats of the probe, then env variants (event time)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gram
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- ./tools/gram_probe > $O/prof.log 2>&1 || { cat $O/prof.log; exit 1; }
find $O -name "*kernel_trace.csv" -delete
cat $O/prof.log | grep "us per"
python3 -c "
import csv,glob
f=glob.glob('$O/prof/**/run_kernel_stats.csv', recursive=True)+glob.glob('$O/prof/run_kernel_stats.csv')
for r in csv.DictReader(open(f[0])): print('%-60s %5s calls %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
for v in "N2V2R_TN_WAVES=2048" "N2V2R_TN_WAVES=8192" "N2V2R_TN_U=8" "N2V2R_TN_MINROWS=128" "N2V2R_TN_MINROWS=416" "N2V2R_REDUCE=wave"; do
  echo "== $v"
  env $v timeout -k 10 60 ./tools/gram_probe || exit 1
done
