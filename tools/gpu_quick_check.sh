# model / sign-convention tests + cfg2 bench (two runs) + kernel trace split of one fit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qc
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_dense.py -k "uase or end_to_end or model or dist or dense or demo or dedi" > gpurun_out/qc/tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/qc/tests.log; exit 1; }
tail -1 gpurun_out/qc/tests.log
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/qc/b.json 2> gpurun_out/qc/b.err || { tail -3 gpurun_out/qc/b.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/qc/b.json').read().strip().splitlines()[-1])
print('%8.3f ms  apps %d  res %.3e' % (d['ms_per_step'], d['eig']['block_applications'], d['eig']['max_residual']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qc/t -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/qc/tb.json 2> gpurun_out/qc/tb.err || { echo trace-fail; exit 1; }
f=$(find gpurun_out/qc/t -name "*kernel_trace.csv" | head -1)
python3 tools/trace_split.py $f > gpurun_out/qc/split.txt
rm -f $f
grep -E "colmax|distances|borda|radix|scale_cols|spmm_csr|inverse_perm" gpurun_out/qc/split.txt | head -12
