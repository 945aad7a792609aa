# cfg5 (ER N=10M, deg 30, d=128) on ONE GPU through the partitioned path (world 1), round-2 build;
# progress lines every cycle on stderr (N2V2R_TRACE) so the run is seen alive
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
N2V2R_TRACE=1 timeout -k 10 1000 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5/bench_cfg5.json 2> gpurun_out/c5/bench_cfg5.err || { tail -5 gpurun_out/c5/bench_cfg5.err; exit 1; }
cut -c1-400 gpurun_out/c5/bench_cfg5.json
