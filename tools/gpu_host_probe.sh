set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp
for v in 1 0; do
N2V2R_TRACE=1 N2V2R_LEAN_OVERLAP=$v N2V2R_INV_CUS=80 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/hp/b$v.json 2> gpurun_out/hp/e$v.txt || exit 1
done
