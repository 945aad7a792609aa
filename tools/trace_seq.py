"""Print a window of consecutive kernels of a rocprofv3 kernel trace (csv) with each launch's
duration and the idle gap before it, from the middle of the last fit.

    python tools/trace_seq.py run_kernel_trace.csv [count] [offset]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
count = int(sys.argv[2]) if len(sys.argv) > 2 else 40
off = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows) * 3 // 4
prev = None
tot_gap = tot_dur = 0.0
for r in rows[off:off + count]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev) / 1e3 if prev is not None else 0.0
    prev = e
    tot_gap += max(g, 0)
    tot_dur += (e - s) / 1e3
    print(f"gap {g:7.2f} us  dur {(e - s) / 1e3:8.2f} us  grid {r['Grid_Size_X']:>7s}x{r['Grid_Size_Y']:<4s} {r['Kernel_Name'][:60]}")
print(f"sum: busy {tot_dur:.1f} us, idle {tot_gap:.1f} us")
