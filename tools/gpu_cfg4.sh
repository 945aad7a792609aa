# cfg4 (N = 1M, column-block SpMM) bench line + rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cfg4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo "cfg4 failed"; tail -5 $O/b.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); g=d['eig']
print('cfg4', d['ms_per_step'], 'ms', d['value'], 'nodes/s cycles', g['restarts'], 'apps', g['block_applications'], 'res %.2e' % g['max_residual'])
"
if [ -n "$PROF" ]; then
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config cfg4 --steps 1 --warmup 1 --no-cpu-baseline > $O/p.json 2> $O/p.err || { echo prof-fail; exit 1; }
find $O -name "*kernel_trace.csv" -delete
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in rows[:10]:
    print(f"{float(r['TotalDurationNs'])/1e6/2:9.1f} ms/fit {int(r['Calls'])/2:7.1f} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
fi
