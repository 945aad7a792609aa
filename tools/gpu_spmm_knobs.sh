# SpMM b = 8 knob sweep on the locality probe graphs (+ SpMM parity under the lane kernel)
cd $GRAFT_REPO_ROOT
set -o pipefail
N2V2R_SPMM8=lane timeout -k 10 100 python -u -m pytest -q -x tests/test_gpu_parity.py -k "spmm_matches or spmm_b8" 2>&1 | tail -2 || exit 1
for v in "" "N2V2R_SPMM8=lane" "N2V2R_SPMM8=lane N2V2R_SPMM_RPW=8" "N2V2R_SPMM8=lane N2V2R_SPMM_RPW=2"; do
  echo "== $v"
  env $v timeout -k 10 100 python -u tools/spmm_locality.py || exit 1
done
