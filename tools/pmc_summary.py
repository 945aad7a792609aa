"""Summarise the PMC passes of tools/gpu_pmc_ortho.sh into a markdown table: per kernel, the HBM
bytes of the whole cfg2 fit (FETCH_SIZE x 2, the gfx950 correction of MI355X_MICROARCH.md, plus
WRITE_SIZE; both in KiB), the L2 hit rate, the kernel-trace time of the same fit and the
resulting HBM rate.  Usage: python tools/pmc_summary.py gpurun_out/pmc > profiles/r02_pmc_ortho.md"""
import collections
import csv
import sys

d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for p in ("p1", "p2", "p3"):
    for r in csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv")):
        tot[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
ns = collections.defaultdict(float)
cnt = collections.defaultdict(int)
for r in csv.DictReader(open(f"{d}/kt/run_kernel_trace.csv")):
    k = r["Kernel_Name"].split("(")[0]
    ns[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt[k] += 1
print("| kernel | launches | time (ms) | HBM read (MB) | HBM write (MB) | HBM rate (TB/s) | L2 hit |")
print("|---|---|---|---|---|---|---|")
for k, c in sorted(tot.items(), key=lambda kv: -ns[kv[0]]):
    rd = c["FETCH_SIZE"] * 2 * 1024
    wr = c["WRITE_SIZE"] * 1024
    hit = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    t = ns[k] * 1e-9
    rate = (rd + wr) / t / 1e12 if t else float("nan")
    print(f"| `{k}` | {cnt[k]} | {t*1e3:.2f} | {rd/1e6:.0f} | {wr/1e6:.0f} | {rate:.2f} | {hit:.2f} |")
