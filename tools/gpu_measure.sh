set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/meas
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/meas/bench.json 2> gpurun_out/meas/bench.err || { echo bench-fail; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/meas/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/meas/prof_bench.json 2> gpurun_out/meas/prof_bench.err || { echo prof-fail; exit 1; }
find gpurun_out/meas/prof -name "*kernel_trace.csv" -delete
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/meas/fetch -o run -- python3 tools/spmm_probe.py > gpurun_out/meas/fetch.log 2>&1 || { echo fetch-fail; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/meas/write -o run -- python3 tools/spmm_probe.py > gpurun_out/meas/write.log 2>&1 || { echo write-fail; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/meas/ptrace -o run -- python3 tools/spmm_probe.py > gpurun_out/meas/ptrace.log 2>&1 || { echo ptrace-fail; exit 1; }
