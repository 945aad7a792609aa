# cfg2 step time at panel width 16 (dense Rayleigh-Ritz) vs the b = 8 default, plus one kernel
# profile of the b = 16 fit
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/b16
mkdir -p $O
export TMPDIR=/tmp
for e in '{}' '{"block": 16}' '{"block": 16, "max_basis": 320}' '{"block": 16, "max_basis": 384}' '{"block": 16, "keep": 96, "max_basis": 384}'; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --eig "$e" > $O/b.json 2> $O/b.err || { echo "fail $e"; tail -3 $O/b.err; continue; }
  python3 -c "
import json,sys
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); g=d['eig']
print('%-45s %8.2f ms  cycles %3d apps %4d basis %d res %.2e' % (sys.argv[1], d['ms_per_step'], g['restarts'], g['block_applications'], g['basis'], g['max_residual']))
" "$e"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --eig '{"block": 16}' > $O/prof.log 2>&1 || { echo prof-fail; tail -5 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/b16/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6s} {float(r['TotalDurationNs'])/1e6:9.2f} {float(r['AverageNs'])/1e3:8.1f}")
PY
