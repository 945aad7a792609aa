"""Per-launch PMC summary of one kernel family from separate rocprofv3 --pmc passes.

Usage: python tools/pmc_kernel.py DIR REGEX [--alternate N] [--json OUT --config C --stage S]

DIR holds one sub-directory per pass (each with a run_counter_collection.csv somewhere below
it) and `kt/` with the --kernel-trace run of the same command.  For every kernel whose name
matches REGEX: launches, average duration (kernel trace), HBM read = FETCH_SIZE x 2 (the gfx950
correction of MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of wide streaming reads),
HBM write = WRITE_SIZE (both KiB in the CSV), L2 hit rate, and the MFMA counters when present:
busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs).  With --alternate N
the launches of each kernel are split by dispatch order modulo N (the tiled SpMM alternates
stage 1 / stage 2 inside every application of M).  --json writes the per-launch HBM bytes of
phase 0 in the format bench.py reads (profiles/spmm_traffic.json)."""
import argparse
import collections
import csv
import glob
import json
import os
import re


def rows(path):
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("regex")
    ap.add_argument("--alternate", type=int, default=1)
    ap.add_argument("--json")
    ap.add_argument("--config")
    ap.add_argument("--stage")
    ap.add_argument("--algo-bytes", type=float, default=None)
    a = ap.parse_args()
    rx = re.compile(a.regex)

    # counters per (kernel, dispatch)
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for sub in sorted(os.listdir(a.dir)):
        p = os.path.join(a.dir, sub)
        if sub == "kt" or not os.path.isdir(p):
            continue
        for r in rows(p):
            k = r["Kernel_Name"].split("(")[0]
            if not rx.search(k):
                continue
            per[(sub, k)][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    # durations
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "kt", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if rx.search(k):
                dur[k].append((int(r["Dispatch_Id"]),
                               int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))

    kernels = sorted({k for (_, k) in per} | set(dur))
    out = {}
    print("| kernel | phase | launches | avg µs | HBM read / launch (MB) | HBM write / launch (MB)"
          " | HBM rate (TB/s) | L2 hit | MFMA busy |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in kernels:
        for ph in range(a.alternate):
            acc = collections.defaultdict(list)
            for (sub, kk), disp in per.items():
                if kk != k:
                    continue
                ids = sorted(disp)
                for i, d in enumerate(ids):
                    if i % a.alternate != ph:
                        continue
                    for c, v in disp[d].items():
                        acc[c].append(v)
            ds = sorted(dur.get(k, []))
            ts = [t for i, (_, t) in enumerate(ds) if i % a.alternate == ph]
            avg_ns = sum(ts) / len(ts) if ts else float("nan")

            def mean(c):
                v = acc.get(c)
                return sum(v) / len(v) if v else None
            fs, ws = mean("FETCH_SIZE"), mean("WRITE_SIZE")
            rd = fs * 2 * 1024 if fs is not None else None
            wr = ws * 1024 if ws is not None else None
            hit_h, hit_m = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
            hit = hit_h / max(1.0, hit_h + hit_m) if hit_h is not None else None
            busy, act = mean("SQ_VALU_MFMA_BUSY_CYCLES"), mean("GRBM_GUI_ACTIVE")
            mf = busy / (act * 1024) if busy is not None and act else None
            rate = ((rd or 0) + (wr or 0)) / (avg_ns * 1e-9) / 1e12 if ts and rd else None
            f = lambda v, s: "—" if v is None else s.format(v)
            print(f"| `{k}` | {ph} | {len(ts)} | {avg_ns / 1e3:.1f} | {f(rd and rd / 1e6, '{:.1f}')}"
                  f" | {f(wr and wr / 1e6, '{:.1f}')} | {f(rate, '{:.2f}')} | {f(hit, '{:.2f}')}"
                  f" | {f(mf, '{:.3f}')} |")
            out[(k, ph)] = dict(launches=len(ts), avg_ns=avg_ns, read=rd, write=wr, l2_hit=hit,
                                mfma_busy=mf, mops_f32=mean("SQ_INSTS_VALU_MFMA_MOPS_F32"),
                                busy_cycles=busy, gui_active=act)
    if a.json:
        (k, ph), v = next(iter(out.items()))
        rec = dict(config=a.config, stage=a.stage, kernel=k, b=8,
                   bytes_per_launch=(v["read"] or 0) + (v["write"] or 0),
                   read_bytes_per_launch=v["read"], write_bytes_per_launch=v["write"],
                   l2_hit=v["l2_hit"], avg_ns_kernel_trace=v["avg_ns"],
                   source=f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes in {a.dir} "
                          "(2*FETCH_SIZE+WRITE_SIZE, gfx950 correction), phase 0 of "
                          f"{a.alternate} (stage 1 of each application)")
        if a.algo_bytes:
            rec["algo_bytes_per_launch"] = a.algo_bytes
        json.dump(rec, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
