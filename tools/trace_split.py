"""Split a rocprofv3 kernel trace (csv) of one bench step by kernel and launch shape.

    python tools/trace_split.py gpurun_out/trace2/run_kernel_trace.csv [--last-steps 1]

Prints per (kernel, grid) the call count, total and mean duration, plus the idle time between
consecutive launches on the GPU (gaps)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the timed step is the second half (warmup 1 + steps 1): take launches after the midpoint fit
half = len(rows) // 2
rows = rows[half:]
agg = defaultdict(lambda: [0, 0.0, []])
gap = 0.0
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev_end is not None and s > prev_end:
        gap += s - prev_end
    prev_end = max(prev_end or 0, e)
    name = r["Kernel_Name"].split("(")[0][:48]
    key = (name, r["Grid_Size_X"], r["Grid_Size_Y"])
    a = agg[key]
    a[0] += 1
    a[1] += (e - s) / 1e3
    a[2].append((e - s) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
print(f"launches {len(rows)}  span {span:.2f} ms  gaps {gap / 1e6:.2f} ms")
by_name = defaultdict(float)
for (n, gx, gy), (c, t, _) in agg.items():
    by_name[n] += t
for n, t in sorted(by_name.items(), key=lambda x: -x[1]):
    print(f"{t / 1e3:8.2f} ms  {n}")
print()
for (n, gx, gy), (c, t, ds) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    ds.sort()
    print(f"{t / 1e3:7.2f} ms {c:5d} x {t / c:7.2f} us (min {ds[0]:6.2f} max {ds[-1]:7.2f})  grid {gx}x{gy}  {n}")
