#!/bin/bash
# Round 4 (session 2) probe (N2V2R_TN_SMALL_WAVES, removed after it): wave target of the streaming
# Gram for <= 4 blocks (the local pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r04_tw
mkdir -p $R
for w in 1024 2048 4096 8192; do
  for cfg in cfg4 cfg2; do
    N2V2R_TN_SMALL_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$cfg.$w -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 1 --warmup 0 --resident-steps 1 --no-cpu-baseline \
      > $R/$cfg.$w.json 2> $R/$cfg.$w.err || exit $?
    python3 - <<PY
import csv, glob
f = glob.glob("$R/$cfg.$w/**/run_kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(f))}
for k in ("void ts_tn_stream_lds_kernel<4>", "reduce_chunks_kernel", "reduce_cols_kernel"):
    r = rows.get(k)
    if r: print("$cfg", $w, k, r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total", round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
  done
done
