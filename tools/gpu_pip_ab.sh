# PIP apply variants: rows per workgroup x blocks in flight (cfg2 bench step time)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pipab
mkdir -p $O
timeout -k 10 200 python -u -m pytest -q -x --timeout 120 tests/test_gpu_parity.py -k "uase_matches or residuals or rank_deficient or redo" > $O/t.log 2>&1 || { echo tests-fail; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in "N2V2R_PIP_ROWS=256 N2V2R_PIP_QB=4" "N2V2R_PIP_ROWS=128 N2V2R_PIP_QB=8" "N2V2R_PIP_ROWS=128 N2V2R_PIP_QB=4" "N2V2R_PIP_ROWS=256 N2V2R_PIP_QB=4"; do
  env $v timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo "fail $v"; tail -3 $O/b.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('%-40s %8.3f ms' % (sys.argv[1], d['ms_per_step']))
" "$v"
done
