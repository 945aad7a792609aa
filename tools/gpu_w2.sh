set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/w2
mkdir -p $O
export TMPDIR=/tmp
for v in "X=0" "N2V2R_EXPERIMENT_W2=1"; do
  env $v timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 tools/w2_probe.py > $O/log 2>&1 || { echo fail; tail $O/log; exit 1; }
  echo "== $v"; tail -1 $O/log
  python3 -c "
import csv
for r in list(csv.DictReader(open('$O/$v/run_kernel_stats.csv')))[:7]:
    print('  %8.2f ms %6s x %8.2f us  %s' % (float(r['TotalDurationNs'])/1e6/3, r['Calls'], float(r['AverageNs'])/1e3, r['Name'][:50]))
"
done
find $O -name "*kernel_trace.csv" -delete
