# column-block SpMM tuning: RPW / workgroup sweeps at N = 300k and 1M; L2 hit rate by PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cbt
export TMPDIR=/tmp
for set in NONE=0 N2V2R_CB_RPW=8 N2V2R_CB_RPW=4 N2V2R_CB_WGS=1024 N2V2R_CB_WGS=4096 N2V2R_CB_WGS=8192; do
  echo "== $set" >> gpurun_out/cbt/sweep.log
  env $set timeout -k 10 100 python -u tools/cb_probe.py 300000:30 1000000:50 >> gpurun_out/cbt/sweep.log 2>&1 || { echo sweep-fail; exit 1; }
done
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/cbt/pmc -o run -- python3 tools/cb_probe.py 1000000:50 > gpurun_out/cbt/pmc.log 2>&1 || { echo pmc-fail; exit 1; }
