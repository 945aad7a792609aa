"""Per-launch PMC summary of one kernel family from separate rocprofv3 --pmc passes.

Usage: python tools/pmc_kernel.py DIR REGEX [--alternate N] [--json OUT --config C --stage S]
                                  [--stats OUT.csv]

DIR holds one sub-directory per pass and `kt/` with the --kernel-trace run of the same command;
each holds rocprofv3's output (the rocpd SQLite database `*_results.db` that ROCm 7.2 writes
by default, or the CSV files of `--output-format csv`).  For every kernel whose name matches
REGEX: launches, average duration (kernel trace), HBM read = FETCH_SIZE x 2 (the gfx950
correction of MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of wide streaming reads;
Infinity-Cache hits are counted too), HBM write = WRITE_SIZE (both KiB), L2 hit rate, and the
MFMA counters when present: busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x
1024 SIMDs).
With --alternate N the launches of each kernel are split by dispatch order modulo N (the tiled
SpMM alternates stage 1 / stage 2 inside every application of M).  --json writes phase 0's
per-launch bytes in the format bench.py reads (profiles/spmm_traffic.json); --stats writes the
kernel-trace summary of kt/ (every kernel: calls, total / average duration, share)."""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sqlite3


def counter_rows(path):
    """(kernel name, dispatch id, counter, value) of one pass directory."""
    for f in glob.glob(os.path.join(path, "**", "*_results.db"), recursive=True):
        db = sqlite3.connect(f)
        yield from db.execute("select kernel_name, dispatch_id, counter_name, value "
                              "from counters_collection")
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            yield (r["Kernel_Name"], int(r["Dispatch_Id"]), r["Counter_Name"],
                   float(r["Counter_Value"]))


def trace_rows(path):
    """(kernel name, dispatch id, duration ns) of the kernel-trace directory."""
    for f in glob.glob(os.path.join(path, "**", "*_results.db"), recursive=True):
        db = sqlite3.connect(f)
        yield from db.execute("select name, dispatch_id, duration from kernels")
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            yield (r["Kernel_Name"], int(r["Dispatch_Id"]),
                   int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))


def short(name):
    return name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("regex")
    ap.add_argument("--alternate", type=int, default=1)
    ap.add_argument("--json")
    ap.add_argument("--config")
    ap.add_argument("--stage")
    ap.add_argument("--algo-bytes", type=float, default=None)
    ap.add_argument("--stats")
    ap.add_argument("--form", type=int, default=None, help="n2v2r_eig_stats.spmm_form profiled")
    ap.add_argument("--rev", default=None, help="kernel revision tag (bench.SPMM_KERNEL_REV)")
    a = ap.parse_args()
    rx = re.compile(a.regex)

    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for sub in sorted(os.listdir(a.dir)):
        p = os.path.join(a.dir, sub)
        if sub == "kt" or not os.path.isdir(p):
            continue
        for name, disp, cname, val in counter_rows(p):
            k = short(name)
            if rx.search(k):
                per[k][(sub, int(disp))][cname] = float(val)
    dur = collections.defaultdict(list)
    allk = collections.defaultdict(list)
    for name, disp, ns in trace_rows(os.path.join(a.dir, "kt")):
        allk[name].append(ns)
        if rx.search(short(name)):
            dur[short(name)].append((int(disp), ns))

    if a.stats:
        tot = sum(sum(v) for v in allk.values())
        with open(a.stats, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, v in sorted(allk.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 3),
                            round(100.0 * sum(v) / tot, 4)])

    out = {}
    print("| kernel | phase | launches | avg µs | HBM read / launch (MB) | HBM write / launch (MB)"
          " | HBM rate (TB/s) | L2 hit | MFMA busy |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k in sorted(set(per) | set(dur)):
        for ph in range(a.alternate):
            acc = collections.defaultdict(list)
            by_pass = collections.defaultdict(list)
            for (sub, disp), cs in per[k].items():
                by_pass[sub].append((disp, cs))
            for sub, lst in by_pass.items():
                for i, (_, cs) in enumerate(sorted(lst, key=lambda t: t[0])):
                    if i % a.alternate == ph:
                        for c, v in cs.items():
                            acc[c].append(v)
            ts = [t for i, (_, t) in enumerate(sorted(dur.get(k, []))) if i % a.alternate == ph]
            avg_ns = sum(ts) / len(ts) if ts else float("nan")

            def mean(c):
                v = acc.get(c)
                return sum(v) / len(v) if v else None
            fs, ws = mean("FETCH_SIZE"), mean("WRITE_SIZE")
            rd = fs * 2 * 1024 if fs is not None else None
            wr = ws * 1024 if ws is not None else None
            hh, hm = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
            # one fabric read request per L2 miss, a whole 128-B line each, for wide streams
            # and for 32-B gathers alike (profiles/r04_fabric_req_calibration.md)
            rq = mean("TCC_EA0_RDREQ_sum")
            rq_bytes = rq * 128 if rq is not None else None
            hit = hh / max(1.0, hh + hm) if hh is not None else None
            busy, act = mean("SQ_VALU_MFMA_BUSY_CYCLES"), mean("GRBM_GUI_ACTIVE")
            # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (7.0M per 394-us cfg3 dispatch = 8 x
            # 2.2 GHz); SQ_VALU_MFMA_BUSY_CYCLES over the 1024 SIMDs (64 per 32x32x2 f32 MFMA)
            mf = busy * 8 / (act * 1024) if busy is not None and act else None
            rate = ((rd or 0) + (wr or 0)) / (avg_ns * 1e-9) / 1e12 if ts and rd else None
            fmt = lambda v, s: "—" if v is None else s.format(v)
            print(f"| `{k}` | {ph} | {len(ts)} | {avg_ns / 1e3:.1f} | "
                  f"{fmt(rd and rd / 1e6, '{:.1f}')} | {fmt(wr and wr / 1e6, '{:.1f}')} | "
                  f"{fmt(rate, '{:.2f}')} | {fmt(hit, '{:.2f}')} | {fmt(mf, '{:.3f}')} |")
            if rq is not None:
                print(f"|   (fabric read requests) | {ph} | | | {rq / 1e6:.3f} M = "
                      f"{rq_bytes / 1e6:.1f} MB | | | | |")
            out[(k, ph)] = dict(launches=len(ts), avg_ns=avg_ns, read=rd, write=wr, l2_hit=hit,
                                rdreq=rq, rdreq_bytes=rq_bytes,
                                mfma_busy=mf, mops_f32=mean("SQ_INSTS_VALU_MFMA_MOPS_F32"),
                                busy_cycles=busy, gui_active=act)
    if a.json and out:
        (k, ph), v = next(iter(out.items()))
        rec = dict(config=a.config, stage=a.stage, kernel=k, b=8,
                   bytes_per_launch=(v["read"] or 0) + (v["write"] or 0),
                   read_bytes_per_launch=v["read"], write_bytes_per_launch=v["write"],
                   l2_hit=v["l2_hit"], avg_ns_kernel_trace=v["avg_ns"],
                   source=f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({a.dir}), "
                          "2*FETCH_SIZE+WRITE_SIZE (gfx950 correction; Infinity-Cache hits "
                          f"counted), phase 0 of {a.alternate} (stage 1 of each application)")
        if v.get("rdreq") is not None:
            # the calibrated fabric read traffic: TCC_EA0_RDREQ x 128 B (+ WRITE_SIZE) from a
            # pass of its own over the same command; 2 x FETCH_SIZE kept beside it
            rec["fabric_read_requests_per_launch"] = v["rdreq"]
            rec["fetch_size_x2_bytes_per_launch"] = v["read"]
            rec["read_bytes_per_launch"] = v["rdreq_bytes"]
            rec["bytes_per_launch"] = v["rdreq_bytes"] + (v["write"] or 0)
            rec["source"] = (f"rocprofv3 --pmc passes over the same command ({a.dir}): "
                             "TCC_EA0_RDREQ_sum x 128 B (one 128-B fabric request per L2 miss, "
                             "profiles/r04_fabric_req_calibration.md) + WRITE_SIZE; phase 0 of "
                             f"{a.alternate} (stage 1 of each application)")
        if a.rev:
            rec["kernel_rev"] = a.rev
        if a.algo_bytes:
            rec["algo_bytes_per_launch"] = a.algo_bytes
        if a.form is not None:
            rec["spmm_form"] = a.form
        json.dump(rec, open(a.json, "w"), indent=1)
    return out


if __name__ == "__main__":
    main()
