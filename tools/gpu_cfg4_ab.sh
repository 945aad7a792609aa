# cfg4 A/B of one env switch: AB="VAR=a VAR=b" (each once, steps 2 warmup 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cfg4ab
mkdir -p $O
for v in $AB; do
  env $v timeout -k 10 400 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo "fail $v"; tail -3 $O/b.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('%-34s %9.1f ms  apps %d' % (sys.argv[1], d['ms_per_step'], d['eig']['block_applications']))
" "$v"
done
