# kernel traces of one cfg2 fit with the lean restart overlap on (80 inverse-iteration CUs) and off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 80 off; do
  O=gpurun_out/tlo_$v
  mkdir -p $O
  if [ $v = off ]; then export N2V2R_LEAN_OVERLAP=0; else export N2V2R_INV_CUS=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo trace-fail; tail $O/b.err; exit 1; }
  f=$(find $O -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_gaps.py $f 12 > $O/gaps.txt
  python3 - "$f" > $O/cycle.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("fill_normal")]
fit = rows[st[-1]:]
t0 = int(fit[0]["Start_Timestamp"])
# around the 3rd inverse iteration of the fit: 25 launches before, 30 after
inv = [i for i, r in enumerate(fit) if r["Kernel_Name"].startswith("rr_sturm_inviter")]
i = inv[2]
for r in fit[i - 8:i + 30]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:10.2f} {(e - t0) / 1e3:10.2f} {(e - s) / 1e3:8.2f}  q{r.get('Queue_Id', '?'):>3s} {r['Kernel_Name'][:60]}")
PY
  rm -f $f
done
