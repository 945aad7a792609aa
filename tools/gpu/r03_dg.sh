# dense GEMM (cfg3): X operands in registers vs LDS, workgroup counts; fp64 projection test.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dg
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/dg/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_ingest.py tests/test_gpu_dense.py -v -rf -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dg/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/dg/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
for v in "1 0" "0 0" "1 512" "1 768" "1 1024" "0 768"; do
  set -- $v
  N2V2R_DG_XREG=$1 N2V2R_DG_SPLIT=$2 timeout -k 10 300 python -u bench.py --config cfg3 --steps 2 --warmup 1 --resident-steps 2 --no-cpu-baseline > gpurun_out/dg/cfg3_x$1_s$2.json 2> gpurun_out/dg/cfg3_x$1_s$2.err || { echo bench-fail-$1-$2; exit 1; }
done
echo done
