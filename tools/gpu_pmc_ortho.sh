# PMC passes (one counter group per run) over a short cfg2 bench: HBM fetch/write and L2 hits of
# the orthogonalisation kernels (Gram, PIP) and the SpMM
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc
mkdir -p $O
export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "ts_tn_stream|pip_fused|spmm8_pipe|reduce_chunks" --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $O/p$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "ts_tn_stream|pip_fused|spmm8_pipe|reduce_chunks" --output-format csv -d $O/kt -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1 || { echo trace-fail; exit 1; }
ls -R $O | head -30
