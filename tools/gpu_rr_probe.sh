set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rrprobe
mkdir -p $O
export TMPDIR=/tmp
for kp in 0 80; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$kp -o run -- python3 tools/rr_probe.py 384 $kp 5 > $O/p$kp.log 2>&1 || { echo fail; tail $O/p$kp.log; exit 1; }
  cat $O/p$kp.log | tail -1
  python3 -c "
import csv
for r in csv.DictReader(open('$O/p$kp/run_kernel_stats.csv')):
    print('  %8.1f us x %s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:60]))
"
done
find $O -name "*kernel_trace.csv" -delete
