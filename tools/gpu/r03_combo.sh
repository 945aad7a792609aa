# dense A/B + block-width probe, then the profile passes (one box).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r03_dg2.sh || exit 1
bash tools/gpu/r03_prof.sh || exit 1
echo combo-done
