# lean-image restart overlap: parity subset, then cfg2 A/B (overlap off / plain streams / CU masks)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out


AB="N2V2R_LEAN_OVERLAP=0 N2V2R_LEAN_OVERLAP=1" bash tools/gpu_ab_env.sh
