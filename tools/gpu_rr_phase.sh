# Rayleigh-Ritz stage timing: rocprofv3 kernel stats of a short cfg2 bench with the inverse
# iteration cut after phase k (N2V2R_INVITER_STOP=k; the cut sets the error flag, so the
# reducing fallback runs after it -- only the inviter kernel's own time is read here)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/rrphase
mkdir -p $O
export TMPDIR=/tmp
for k in ${STOPS:-1 2 3 4 5 0}; do
  N2V2R_INVITER_STOP=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$k -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b$k.json 2> $O/b$k.err || { echo "prof-fail $k"; tail -3 $O/b$k.err; exit 1; }
  find $O/p$k -name "*kernel_trace.csv" -delete
  python3 - "$O/p$k/run_kernel_stats.csv" "$k" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r['Name'].startswith(('rr_sturm_inviter', 'rr_msect_kernel', 'rr_sturm_prep')):
        print(f"stop={sys.argv[2]} {r['Name'][:30]:30s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
done
