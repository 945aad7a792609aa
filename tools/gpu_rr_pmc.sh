set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rrpmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/rrpmc -o run -- python3 tools/bench_rr.py 384 80 88 2 > gpurun_out/rrpmc/log 2>&1
