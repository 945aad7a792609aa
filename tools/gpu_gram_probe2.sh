# orthogonalisation Gram timing, env variants (event time per Gram + reduce), two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in "N2V2R_NONE=1" "N2V2R_REDUCE=wave" "N2V2R_REDUCE=wave N2V2R_TN_MINROWS=416" "N2V2R_TN_MINROWS=416" "N2V2R_REDUCE=wave N2V2R_TN_U=8"; do
  echo "== $v"
  env $v timeout -k 10 60 ./tools/gram_probe || exit 1
done
done
