# rocprofv3 kernel stats of a short cfg2 bench (TAG names the output dir; extra env via ENVV)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-profq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo prof-fail; tail $O/bench.err; exit 1; }
find $O -name "*kernel_trace.csv" -delete
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6/4:8.2f} ms/step {int(r['Calls'])/4:7.1f} calls {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:70]}")
PY
