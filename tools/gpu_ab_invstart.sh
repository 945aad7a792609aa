# inverse-iteration start vectors (kept Ritz vector vs random): parity subset, second-solve counts, cfg2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_poison.py -k "uase or lean or reorth or band or sturm or poison" > gpurun_out/ab_tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
N2V2R_TRACE=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep -E "second solve|true max_res" > gpurun_out/inv_trace.txt || true
cat gpurun_out/inv_trace.txt
AB="N2V2R_INV_START=rand N2V2R_INV_START=warm" bash tools/gpu_ab_env.sh
