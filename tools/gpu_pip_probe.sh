# fused PIP pass phase timing: the probe with every phase after k skipped (N2V2R_PIP_STOP=k)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/pip_probe.txt
for k in 0 1 2 3 4 5 6; do
  echo "== N2V2R_PIP_STOP=$k" >> gpurun_out/pip_probe.txt
  N2V2R_PIP_STOP=$k timeout -k 10 60 ./tools/pip_probe >> gpurun_out/pip_probe.txt 2>&1 || { cat gpurun_out/pip_probe.txt; exit 1; }
done
cat gpurun_out/pip_probe.txt
