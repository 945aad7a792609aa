set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/cfg3_sweep.log
for e in '{}' '{"block":32,"max_basis":512}' '{"block":64,"max_basis":768}' '{"block":64,"max_basis":640}' '{"block":16,"max_basis":768}' '{"block":32,"max_basis":640,"keep":288}'; do
  timeout -k 10 300 python bench.py --config cfg3 --steps 1 --warmup 1 --no-cpu-baseline --eig "$e" >> gpurun_out/cfg3_sweep.log 2>> gpurun_out/cfg3_sweep.err || exit 1
done
