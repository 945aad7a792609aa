"""Idle gaps of the GPU inside the last fit of a rocprofv3 kernel trace (csv): the largest
gaps with the kernels on either side, and the total idle time between the last fit's first and
last launch.

    python tools/trace_gaps.py run_kernel_trace.csv [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
# the last fit: from the last fill_normal (start block) to the Borda sum after it
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("fill_normal")]
i0 = starts[-1] if starts else 0
ends = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("borda_sum") and i > i0]
fit = rows[i0:(ends[0] + 1) if ends else len(rows)]
gaps = []
idle = 0.0
for a, b in zip(fit, fit[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if g > 0:
        idle += g
    gaps.append((g, a["Kernel_Name"][:50], b["Kernel_Name"][:50]))
span = (int(fit[-1]["End_Timestamp"]) - int(fit[0]["Start_Timestamp"])) / 1e3
print(f"last fit: {len(fit)} launches, span {span:.1f} us, idle {idle:.1f} us")
for g, a, b in sorted(gaps, reverse=True)[:top]:
    print(f"{g:9.2f} us  after {a:50s} before {b}")
