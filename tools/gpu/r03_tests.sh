# GPU suite (no -x: every failure listed), rank agreement probe, API wall times, cfg4 bench A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t/tests.log
case $rc in 0|1) ;; *) echo "pytest crashed rc=$rc"; exit 1;; esac
timeout -k 10 400 python -u tools/parity_probe.py > gpurun_out/t/parity.jsonl 2> gpurun_out/t/parity.err || { echo parity-fail; exit 1; }
timeout -k 10 200 python -u tools/api_wall.py --config cfg2 --reps 3 > gpurun_out/t/api_cfg2.json 2>&1 || { echo api2-fail; exit 1; }
timeout -k 10 300 python -u tools/api_wall.py --config cfg4 --reps 2 > gpurun_out/t/api_cfg4.json 2>&1 || { echo api4-fail; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/t/bench_cfg4_tile.json 2> gpurun_out/t/bench_cfg4_tile.err || { echo bench-tile-fail; exit 1; }
N2V2R_SPMM_TILE=0 timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/t/bench_cfg4_cb.json 2> gpurun_out/t/bench_cfg4_cb.err || { echo bench-cb-fail; exit 1; }
echo done
