# generic env A/B on the cfg2 bench: AB="VAR=a VAR=b ..." (each a separate run, twice; join
# several variables of one run with +, e.g. AB="A=1+B=2 A=0")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab
mkdir -p $O
for rep in 1 2; do
for v in $AB; do
  env ${v//+/ } timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo "fail $v"; tail -3 $O/b.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('%-34s %8.3f ms  apps %d' % (sys.argv[1], d['ms_per_step'], d['eig']['block_applications']))
" "$v"
done
done
