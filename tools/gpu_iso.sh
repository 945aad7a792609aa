# isolate an intermittent GPU test failure: the same selection under several env settings
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/iso
export TMPDIR=/tmp
i=0
for set in ${ISO:-NONE=0}; do
  i=$((i+1))
  env ${set//;/ } timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x -k "${TESTK:-uase}" --timeout 120 --timeout-method thread > gpurun_out/iso/r$i.log 2>&1
  echo "$set rc=$?" >> gpurun_out/iso/r$i.log
done
