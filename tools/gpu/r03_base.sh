# Round-3 baseline on one MI355X: GPU suite, end-to-end rank agreement, API wall times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/base
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/base/tests.log 2>&1 || { echo tests-fail; exit 1; }
timeout -k 10 300 python -u tools/parity_probe.py > gpurun_out/base/parity.jsonl 2> gpurun_out/base/parity.err || { echo parity-fail; exit 1; }
timeout -k 10 200 python -u tools/api_wall.py --config cfg2 --reps 3 > gpurun_out/base/api_cfg2.json 2>&1 || { echo api2-fail; exit 1; }
timeout -k 10 300 python -u tools/api_wall.py --config cfg4 --reps 2 > gpurun_out/base/api_cfg4.json 2>&1 || { echo api4-fail; exit 1; }
echo done
