# cfg2 step time vs Krylov basis size / kept vectors (bench --eig); stops at a crash or timeout
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/basis2
mkdir -p $O
for e in '{}' '{"max_basis": 320}' '{"max_basis": 448}' '{"max_basis": 512}' '{"keep": 72}' '{"keep": 88}' '{"keep": 96}' '{"keep": 96, "max_basis": 448}' '{"keep": 104, "max_basis": 512}' '{"keep": 88, "max_basis": 448}'; do
  timeout -k 10 200 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --eig "$e" > $O/b.json 2> $O/b.err
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "fail rc=$rc $e"; tail -2 $O/b.err
    if [ $rc -ge 124 ]; then exit 1; fi
    continue
  fi
  python3 -c "
import json,sys
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); g=d['eig']
print('%-40s %8.2f ms  cycles %3d apps %4d basis %d res %.2e' % (sys.argv[1], d['ms_per_step'], g['restarts'], g['block_applications'], g['basis'], g['max_residual']))
" "$e"
done
