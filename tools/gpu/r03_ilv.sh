# Flat SpMM stage 1 with the layers walked in the same phases (N2V2R_FLAT_ILV=1) vs the default:
# parity tests under the switch, cfg4 fits at 16 / 32 column blocks both ways.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ilv
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
N2V2R_FLAT_ILV=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "column_blocks or cfg4 or tiled" > $O/tests_ilv.log 2>&1 || { echo ilv-tests-failed; exit 1; }
for v in "1 16" "0 16" "1 32" "0 16" "1 16"; do
  set -- $v
  N2V2R_FLAT_ILV=$1 N2V2R_SPMM_TILE_NB=$2 timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 --resident-steps 2 --no-cpu-baseline > $O/cfg4_i$1_nb$2.$RANDOM.json 2> $O/cfg4_i$1_nb$2.err || { echo cfg4-fail-$1-$2; exit 1; }
done
echo done
