#!/bin/bash
# GPU measurement steps, run through gpurun from the repo root:
#   bash tools/gpu/steps.sh OUTDIR STEP [STEP ...]
# Steps (each GPU step under its own time limit; the first failure ends the script):
#   tests         the whole GPU suite (pytest -m gpu) + __graft_entry__.smoke()
#   bench:CFG     one bench.py line for cfg1 / cfg2 / cfg3 / cfg4 (5 steps) or cfg5 (2 steps)
#   kt:CFG        rocprofv3 kernel trace + stats of one bench step of CFG
#   pmc4          the cfg4 tiled SpMM's counter passes (FETCH_SIZE, WRITE_SIZE, fabric read
#                 requests + L2 hits / misses), each pass a run of its own
#   pmc3          the cfg3 dense product's counter passes (MFMA busy / waits, FETCH_SIZE)
#   pmc5          fabric read requests + L2 hits / misses of the cfg5-sized tiled SpMM
#                 (one ER layer, N = 10M, degree 30: tools/tile_nb_probe.py)
#   nb5:LIST      cfg5-sized tiled SpMM ms per launch over column-block counts (e.g. nb5:64,128)
#   basis:N:DEG:D:COMBOS  block applications over b:keep:basis combos (tools/probe_block16.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$1
shift
mkdir -p "$O"
( while true; do date +%T >> "$O/heartbeat.txt"; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT

fail() { echo "$1 failed rc=$2"; tail -30 "$3"; exit 1; }
prof() {  # prof NAME LIMIT rocprofv3-args... (the program directly after --)
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" rocprofv3 "$@" > "$O/$name.log" 2>&1 || fail "$name" $? "$O/$name.log"
}
bench_args() {  # the bench command line of one step of CFG, no CPU baseline
  echo "bench.py --config $1 --steps 1 --warmup 1 --resident-steps 0 --no-cpu-baseline"
}

for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$O/gpu_suite.log" 2>&1 || fail tests $? "$O/gpu_suite.log"
      tail -2 "$O/gpu_suite.log"
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$O/smoke.log" 2>&1 || fail smoke $? "$O/smoke.log"
      ;;
    bench:cfg5)
      timeout -k 10 600 python -u bench.py --config cfg5 --steps 2 --warmup 1 --resident-steps 1 \
        > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err" || fail "bench cfg5" $? "$O/bench_cfg5.err"
      ;;
    bench:*)
      c=${step#bench:}
      timeout -k 10 400 python -u bench.py --config "$c" --steps 5 --warmup 2 \
        > "$O/bench_$c.json" 2> "$O/bench_$c.err" || fail "bench $c" $? "$O/bench_$c.err"
      ;;
    kt:*)
      c=${step#kt:}
      prof "kt_$c" 400 --kernel-trace --stats --output-format csv -d "$O/kt_$c" -o run -- python -u $(bench_args "$c")
      ;;
    pmc4)
      K="spmm8_flat_kernel"
      B=$(bench_args cfg4)
      prof p4f 300 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/cfg4/fetch" -o run -- python -u $B
      prof p4w 300 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/cfg4/write" -o run -- python -u $B
      prof p4r 300 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex "$K" --output-format csv -d "$O/cfg4/rdreq" -o run -- python -u $B
      ;;
    pmc3)
      K="dense_tn_kernel"
      B=$(bench_args cfg3)
      prof p3m 300 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d "$O/cfg3/mfma" -o run -- python -u $B
      prof p3f 300 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/cfg3/fetch" -o run -- python -u $B
      ;;
    pmc5)
      prof p5r 400 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex spmm8_flat_kernel --output-format csv -d "$O/cfg5/rdreq" -o run -- python -u tools/tile_nb_probe.py 10000000 30 0 6
      ;;
    nb5:*)
      timeout -k 10 500 python -u tools/tile_nb_probe.py 10000000 30 "${step#nb5:}" 6 \
        > "$O/nb5.jsonl" 2>&1 || fail nb5 $? "$O/nb5.jsonl"
      ;;
    basis:*)
      IFS=: read -r _ n deg d combos <<< "$step"
      timeout -k 10 900 python -u tools/probe_block16.py "$n" "$deg" "$d" "$combos" \
        > "$O/basis_$n.jsonl" 2>&1 || fail basis $? "$O/basis_$n.jsonl"
      ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
