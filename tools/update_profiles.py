"""Assemble the committed profiles/ artefacts from a tools/gpu_measure.sh run (gpurun_out/meas)."""
import collections
import csv
import json
import os
import shutil
import sys

RUN = sys.argv[1] if len(sys.argv) > 1 else "r01"
M = "gpurun_out/meas"


def load(p):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


fetch = load(f"{M}/fetch/run_counter_collection.csv")
write = load(f"{M}/write/run_counter_collection.csv")
trace = {r["Name"]: r for r in csv.DictReader(open(f"{M}/ptrace/run_kernel_stats.csv"))}
probe = {}
for line in open(f"{M}/ptrace.log"):
    if line.startswith("b="):
        kv = dict(x.split("=") for x in line.split())
        probe[int(kv["b"])] = float(kv["algo_bytes"])
rows = []
traffic = None
for k in fetch:
    if "spmm8_pipe_kernel" in k:
        b = 8
    elif "spmm_csr_panel_kernel" in k:
        b = int(k.split("<")[1].split(",")[0])
    else:
        continue
    fkb, wkb = med(fetch[k]), med(write.get(k, [0.0]))
    hbm = 2 * fkb * 1024 + wkb * 1024
    avg_ns = float(trace[k]["AverageNs"])
    algo = probe[b]
    rows.append((k, avg_ns, fkb, wkb, hbm, algo))
    if b == 8:
        traffic = {"config": "cfg2", "b": 8, "bytes_per_launch": int(hbm),
                   "algo_bytes_per_launch": int(algo), "avg_ns_kernel_trace": avg_ns,
                   "source": f"profiles/{RUN}_spmm_pmc.md (2*FETCH_SIZE+WRITE_SIZE, gfx950 correction)"}
with open(f"profiles/{RUN}_spmm_pmc.md", "w") as f:
    f.write(f"# SpMM HBM traffic, round {RUN[1:]} (rocprofv3 PMC, MI355X)\n\n")
    f.write("Command (tools/gpu_measure.sh; separate passes, counters alone): `rocprofv3 --pmc FETCH_SIZE`, "
            "`rocprofv3 --pmc WRITE_SIZE`, `rocprofv3 --kernel-trace --stats` on `python3 tools/spmm_probe.py` "
            "(cfg2 layer 0: ER N=100k, avg-deg 20, unweighted, 20 timed launches per width).  Per "
            "MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads half of a wide coalesced stream on gfx950, so "
            "read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE exact.  The gathered panel rows (4 b B per nnz) are "
            "an uncalibrated access width: the corrected figure is an upper bound for them.  Algorithmic bytes "
            "= 4 nnz (column indices; the layer is unweighted, so no value stream) + 8 (N+1) + 4 N b (panel) + "
            "4 N b (output).\n\n")
    f.write("| kernel | avg duration (kernel trace) | FETCH_SIZE KB | WRITE_SIZE KB | corrected HBM bytes/launch "
            "| algorithmic bytes/launch | achieved (algorithmic) GB/s |\n|---|---|---|---|---|---|---|\n")
    for k, ns, fkb, wkb, hbm, algo in rows:
        f.write(f"| `{k}` | {ns/1e3:.2f} us | {fkb:.0f} | {wkb:.0f} | {hbm/1e6:.1f} MB | {algo/1e6:.1f} MB | "
                f"{algo/ns:.0f} |\n")
json.dump(traffic, open("profiles/spmm_traffic.json", "w"), indent=1)
shutil.copy(f"{M}/prof/run_kernel_stats.csv", f"profiles/{RUN}_cfg2_bench_kernel_stats.csv")
shutil.copy(f"{M}/bench.json", f"profiles/{RUN}_bench_cfg2.json")
print(open(f"profiles/{RUN}_spmm_pmc.md").read())
print(traffic)
