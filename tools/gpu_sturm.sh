# Sturm Rayleigh-Ritz: stage tests (both forms), then the solver tests and a cfg2 bench pair
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sturm
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "band_stage" > $O/stage.log 2>&1
echo "stage rc=$?"; tail -25 $O/stage.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo tests-fail; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
N2V2R_TRACE=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_sturm.json 2> $O/bench_sturm.err || { echo bench-fail; tail $O/bench_sturm.err; exit 1; }
N2V2R_RR=band timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_band.json 2> $O/bench_band.err || { echo bench2-fail; exit 1; }
python - <<'PY'
import json
for f in ["sturm", "band"]:
    d = json.loads(open(f"gpurun_out/sturm/bench_{f}.json").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["value"], d["eig"]["restarts"], d["eig"]["block_applications"], d["eig"]["max_residual"])
PY
grep -c "Sturm Rayleigh-Ritz failed" $O/bench_sturm.err || true
