# local-pass Gram chunk size (rows per chunk at least N2V2R_TN_MINROWS): cfg2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
AB="N2V2R_TN_MINROWS=256 N2V2R_TN_MINROWS=416 N2V2R_TN_MINROWS=832" bash tools/gpu_ab_env.sh
