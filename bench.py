"""Benchmark: nodes ranked/s of the fit-and-rank path on MI355X, through the drop-in API.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg4|cfg1|cfg2|cfg3|cfg5]
                    [--mode auto|replicas|partitioned] [--no-cpu-baseline] [--cpu-sample N]

One step = what a caller of the reference does: from host-resident
scipy CSR layers (dense fp32 arrays for cfg3), ``N2V2R(graphs, nodes, config)`` +
``fit_transform_rank()`` + ``aggregate_transform()`` -> host DataFrames of distances and int64
Borda ranks (reference model.py:98-201).  Inside the step: the host->HBM copy of the layers,
the GPU ingest (range check, transpose / symmetry detection), UASE, distances, the device->host
copies, the DataFrames and the Borda of the frames.  ``value`` = nodes ranked/s = N x
comparisons x steps / max-over-ranks wall time.  Default workload: BASELINE cfg4 (2-layer ER
N=1M avg-deg 50, 10-column grid), the largest configuration that fits one GPU.

Extra keys:
  * ``device_resident``: the same work with the layers already in HBM (engine-level loop: UASE,
    distances, Borda, copies of the tables to the host), for comparison;
  * ``roofline``: the dominant kernel of the fit (the SpMM stage launch that takes the most
    device time), timed by HIP events around every SpMM launch of one extra fit on the engine
    stream (solver flag N2V2R_EIG_TIME_SPMM); achieved = SURVEY 8(d) algorithmic bytes per
    launch (for the launch form that runs) / mean launch time; rocprofv3 summaries of the same
    command are committed under profiles/;
  * ``cpu_baseline`` (rank 0, N=1): BASELINE.md 3's faithful CPU restatement (ARPACK svds,
    per-row scipy distances, O(C N^2) list.index Borda over a joblib pool of n_jobs=-2 = the
    CPUs available to the process (its cgroup quota, else its affinity mask) minus one, as the
    reference's model_utils.py:31-32) and its fast variant, on a bounded
    sample of the same graph family; full-size CPU time extrapolated (labelled) from it.

Multi-GPU, --gpus N > 1 (cfg1-4; with or without torchrun): the headline is the SAME drop-in
API call on ONE graph of the workload, row-partitioned over N GPUs by the library itself
(``N2V2R(..., devices=[0..N-1])``: one host thread per GPU inside libn2v2r_hip.so, RCCL over
the N devices), "scaling": "strong".  Under torchrun (the driver's launcher)
rank 0 makes that call and the other ranks wait at the barriers; they then join the side legs:
``replicas`` (every rank its own graph through the API on its own GPU, weak scaling) and
``partitioned_per_process`` (one graph row-partitioned over one process per GPU, RCCL between
processes).  cfg5 (or --mode partitioned) runs one row-partitioned graph with every rank
ingesting only its own rows (one process per GPU under torchrun; the multi-GPU engine without
it).  A gloo group gives the barrier, the max-over-ranks and the RCCL unique id broadcast.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    "cfg1": dict(n=1000, avg_deg=9.99, dims=[8], d=8,
                 desc="cfg1: 2-layer ER N=1000 p=0.01, d=8, cosine+euclidean, sequential"),
    "cfg2": dict(n=100_000, avg_deg=20.0, dims=[64], d=64,
                 desc="cfg2: 2-layer ER N=100k avg-deg 20, d=64, cosine+euclidean, sequential"),
    "cfg3": dict(n=20_000, layers=4, dense=True, dims=[256], d=256, avg_deg=None,
                 desc="cfg3: 4-layer dense |corrcoef| N=20k (N x 200 Gaussian), d=256, "
                      "cosine+euclidean, sequential, dense MFMA path"),
    "cfg4": dict(n=1_000_000, avg_deg=50.0, dims=[8, 16, 32, 64, 128], d=128,
                 desc="cfg4: 2-layer ER N=1M avg-deg 50, dims {8,16,32,64,128} x "
                      "{cosine,euclidean}, sequential"),
    "cfg5": dict(n=10_000_000, avg_deg=30.0, dims=[128], d=128, mode="partitioned",
                 desc="cfg5: 2-layer ER N=10M avg-deg 30, d=128, cosine+euclidean, sequential, "
                      "row-partitioned"),
}
# CPU-baseline sample sizes: ~10-30 s of host work
CPU_SAMPLE = {"cfg1": 1000, "cfg2": 20_000, "cfg3": 2000, "cfg4": 10_000, "cfg5": 10_000}
METRICS = ["cosine", "euclidean"]
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3


def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


class _Group:
    """Control-plane barrier / max over ranks (gloo; the data path has no collective)."""

    def __init__(self, world):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def _reduce(self, x, op):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX) if self.dist else x

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM) if self.dist else x

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def _torch_sync(device=0):
    """torch.cuda.synchronize on this process's own GPU (LOCAL_RANK): under torchrun every
    process touches only its own device, never device 0 of every rank"""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize(device)
    except Exception:
        pass


# BASELINE.json's metric, verbatim
BASELINE_METRIC = "nodes ranked/sec + SpMM HBM GB/s, K-layer N-node graph at 1/2/4/8 GPUs"


def _config(cfg):
    return dict(embed_dimensions=list(cfg["dims"]), distance_metrics=list(METRICS), seed=42,
                comp_strategy="sequential", verbose=-1, save_dir=None)


def api_step(layers, nodes, cfg, device, devices=None):
    """The reference's call sequence on the drop-in API (model.py:18, 98, 149); devices: the
    same call row-partitioned over several GPUs by the library."""
    from node2vec2rank_amd.model import N2V2R
    model = N2V2R(layers, nodes, _config(cfg), device=device, devices=devices)
    ranks = model.fit_transform_rank()
    agg = model.aggregate_transform()
    return model, ranks, agg


def resident_step(eng, cfg, seed=42, flags=0):
    st = eng.uase(cfg["d"], seed=seed, solver_flags=flags)
    ncmp, _ = eng.rank("sequential", cfg["dims"], METRICS)
    out = [(eng.distances(c), eng.borda(c)) for c in range(ncmp)]
    return st, out


def partitioned_step(eng, cfg, rows):
    eng.set_layer_rows(cfg["n"], 2, rows)
    return resident_step(eng, cfg)


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    blas = []
    try:
        from threadpoolctl import threadpool_info
        blas = [f"{d.get('internal_api')}:{d.get('num_threads')}" for d in threadpool_info()]
    except Exception:
        pass
    return model, blas


def host_cpus():
    """CPUs this process may use: the cgroup CPU quota when one is set (the GPU box gives a
    one-GPU job a share of a large host whose os.cpu_count() / affinity list every CPU), else the
    affinity mask."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period))), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    try:
        return len(os.sched_getaffinity(0)), "affinity"
    except AttributeError:
        return os.cpu_count() or 1, "os.cpu_count"


def _sample_layers(cfg, n, seed_base=7000):
    from node2vec2rank_amd import synthetic
    if cfg.get("dense"):
        return synthetic.corr_layers(n, cfg["layers"], seed_base=seed_base)
    return synthetic.er_layers(n, cfg["avg_deg"], 2, seed_base=seed_base)


def cpu_baseline(cfg, n_faithful, workers, blas_threads=1):
    """the repo's faithful CPU restatement of the reference (oracle/, checked
    bit-exact against the reference's outputs) and its fast variant, timed on this host."""
    import scipy.sparse as sp
    from threadpoolctl import threadpool_limits

    from oracle import n2v2r_oracle as orc

    layers = _sample_layers(cfg, n_faithful)
    if cfg.get("dense"):
        layers = [sp.csc_matrix(a) for a in layers]
    with threadpool_limits(blas_threads):
        t0 = time.perf_counter()
        Y, _, _ = orc.uase(layers, cfg["d"], seed=42)
        t_svds = time.perf_counter() - t0
    stages = {}
    for faithful in (True, False):
        with threadpool_limits(blas_threads):
            t1 = time.perf_counter()
            ranks = orc.rank_distances(Y, list(cfg["dims"]), METRICS, "sequential",
                                       faithful=faithful)
            t2 = time.perf_counter()
            for _, (_, D) in ranks.items():
                if faithful:
                    orc.borda_reference_parallel(D, n_jobs=workers)
                else:
                    orc.borda(D)
            t3 = time.perf_counter()
        stages[faithful] = {"svds": t_svds, "distances": t2 - t1, "borda": t3 - t2}
    ncmp = len(ranks)
    fa, fs = stages[True], stages[False]
    n_fast = n_faithful
    tot_fa = sum(fa.values())
    tot_fs = sum(fs.values())
    N = cfg["n"]
    # extrapolation to the bench size (lower bound): svds + distances linear in N (ARPACK's
    # application count only grows with N), Borda O(N^2) for the faithful loop
    r = N / n_faithful
    extra_fa = (fa["svds"] + fa["distances"]) * r + fa["borda"] * r * r
    extra_fs = (fs["svds"] + fs["distances"] + fs["borda"]) * (N / n_fast)
    model, blas = _cpu_info()
    fam = ("{}-layer dense |corrcoef|".format(cfg["layers"]) if cfg.get("dense") else
           f"2-layer ER avg-deg {cfg['avg_deg']:g}")
    return {
        "value": round(n_faithful * ncmp / tot_fa, 1), "unit": "nodes/s", "cores": workers,
        "kind": "port", "blas_threads": blas_threads,
        "sample": (f"{fam} N={n_faithful}, d={cfg['d']}, dims {list(cfg['dims'])} x "
                   f"cosine+euclidean, sequential: oracle faithful mode (ARPACK svds, per-row "
                   f"scipy distances, O(C N^2) list.index Borda over a {workers}-process joblib "
                   f"pool as model_utils.py:31-32), BLAS threads {blas_threads} (ARPACK's dense "
                   f"updates at this size ran slower on more threads)"),
        "stages_s": {k: round(v, 3) for k, v in fa.items()},
        "fast": {"value": round(n_fast * ncmp / tot_fs, 1), "unit": "nodes/s",
                 "sample": f"the same sample and svds: vectorised distances + argsort Borda",
                 "stages_s": {k: round(v, 3) for k, v in fs.items()}},
        "extrapolated_full_size_s": {"faithful_lower_bound": round(extra_fa, 1),
                                     "fast_lower_bound": round(extra_fs, 1),
                                     "note": "svds + distances scaled linearly in N (a lower "
                                             "bound: ARPACK's application count grows with N), "
                                             "faithful Borda as N^2; labelled extrapolated"},
        "host": {"cpu_model": model, "os_cpu_count": os.cpu_count(), "blas": blas},
    }


# ----------------------------------------------------------------------------- roofline
def roofline_from_stats(st, cfg, b, nnz_launch=None, n_launch=None):
    """Dominant SpMM stage of the fit (HIP events around every launch, N2V2R_EIG_TIME_SPMM).
    CSR layers: achieved / frac on BASELINE.md 3's bytes (8 nnz + 4 (N + 1) + 8 N b per layer of
    the launch: nnz_launch entries over n_launch rows); the kernel's own bytes (no value stream
    for unweighted layers, the row pointers it reads) beside them as kernel_bytes."""
    ms = st["gpu_ms_spmm"]
    cnt = st["spmm_timed_launches"]
    by = st["spmm_stage_bytes"]
    j = int(np.argmax(ms))
    if cnt[j] == 0:
        return None
    t = ms[j] / cnt[j]
    bpl = by[j] / cnt[j]
    head = bpl
    if nnz_launch is not None and not cfg.get("dense"):
        head = sum(8.0 * z for z in nnz_launch) + len(nnz_launch) * (4.0 * (n_launch + 1) +
                                                                    8.0 * n_launch * b)
    out = {"bound": "hbm", "achieved": round(head / (t * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
           "unit": "GB/s", "frac": round(head / (t * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
           "traffic": None, "stage": ["Z_k = A_k^T X", "W = sum_k A_k Z_k"][j],
           "avg_launch_ms": round(t, 5), "launches_in_fit": int(cnt[j]),
           "algo_bytes_per_launch": head,
           "algo_bytes_definition": ("BASELINE.md 3 / SURVEY 8(d): 8 nnz + 4 (N + 1) + 8 N b per "
                                     "layer of the launch" if head is not bpl else
                                     "4 N^2 per layer (the dense layer streamed once)"),
           "kernel_bytes": {"bytes_per_launch": bpl,
                            "achieved": round(bpl / (t * 1e-3) / 1e9, 1),
                            "frac": round(bpl / (t * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                            "definition": "what the launch form streams: 4 nnz index words (+4 nnz "
                                          "values for weighted layers) + the window offsets + "
                                          "the panel read and the output written once"},
           "fit_spmm_gpu_ms": [round(x, 2) for x in ms], "fit_spmm_launches": [int(c) for c in cnt]}
    if cfg.get("dense"):
        flops = 2.0 * cfg["n"] * cfg["n"] * b  # one layer's GEMM per launch
        out["kernel"] = ("dense_tn_kernel (A_k X as (B^T X), B streamed from HBM into the MFMA "
                         "B operand, f32 32x32x2)")
        out["mfma_tflops"] = round(flops / (t * 1e-3) / 1e12, 2)
        out["mfma_frac"] = round(flops / (t * 1e-3) / 1e12 / MFMA_F32_PEAK_TFLOPS, 4)
    return out


WATCHDOG_EXIT = 3
GATHER_CEILING_G = 182.1  # G entries/s, profiles/r04_gather_ceiling.jsonl (stream+gather, 2 MB)
# the flat tiled SpMM's revision: a PMC traffic record (profiles/spmm_traffic.json) is attached
# to the line only when it was collected on this revision (round 5: window offsets, segment fold)
SPMM_KERNEL_REV = "r05-window-offsets-w64"


def run_guarded(fn, limit_s, on_timeout):
    """fn() under a watchdog: if it has not returned after limit_s seconds, on_timeout() runs
    (rank 0 prints the bench line there, with the leg marked as timed out) and the process exits
    with status 3 (WATCHDOG_EXIT), so a stalled optional leg neither swallows the line already
    measured nor passes for a clean run with callers that check the exit status."""
    def _fire():
        try:
            on_timeout()
        finally:
            sys.stdout.flush()
            os._exit(WATCHDOG_EXIT)

    timer = threading.Timer(limit_s, _fire)
    timer.daemon = True
    timer.start()
    try:
        return fn()
    finally:
        timer.cancel()


def strong_scaling(group, cfg, args, local, rank, world):
    """One graph of the bench's family row-partitioned over every rank (RCCL), timed like the
    main loop: per step each rank's CSR rows -> HBM, UASE, distances, Borda, tables to host."""
    from node2vec2rank_amd import _lib, synthetic
    uid = group.bcast_bytes(_lib.comm_unique_id() if rank == 0 else None)
    peng = _lib.Engine.rccl(local, rank, world, uid)
    try:
        peng.set_layer_rows(cfg["n"], 2, [])
        _, _, row0, nl = peng.dist_info()
        rows = [synthetic.er_layer_rows(cfg["n"], cfg["avg_deg"], 2000 + k, row0, nl)
                for k in range(2)]
        partitioned_step(peng, cfg, rows)  # warm-up
        peng.synchronize()
        group.barrier()
        t0 = time.perf_counter()
        steps = max(1, args.steps)
        for _ in range(steps):
            st, _ = partitioned_step(peng, cfg, rows)
        peng.synchronize()
        group.barrier()
        t = group.max(time.perf_counter() - t0) / steps
    finally:
        peng.close()
    return {"value": round(cfg["n"] / t, 1), "unit": "nodes/s", "ms_per_step": round(t * 1e3, 3),
            "scaling": "strong", "n_gpus": world, "steps": steps,
            "graph": f"one {cfg['n']}-node graph of the same family (counter-based ER, "
                     f"synthetic.er_layer_rows), rows partitioned over {world} ranks, each "
                     f"rank's CSR rows -> HBM inside the step",
            "block_applications": st.get("block_applications")}


def _local_nnz(layers, row0, nrows):
    """Entries of rows [row0, row0 + nrows) of each CSR layer (one rank's share of a launch)."""
    return [int(a.indptr[row0 + nrows] - a.indptr[row0]) for a in layers]


def replicas_leg(group, cfg, args, local, rank, world):
    """Weak scaling beside the headline (torchrun only): every rank its own graph of the family
    through the one-GPU API on its own GPU, timed like the main loop."""
    from node2vec2rank_amd import synthetic
    layers = synthetic.er_layers(cfg["n"], cfg["avg_deg"], 2, seed_base=1000 + 17 * rank)
    nodes = [f"n{i}" for i in range(cfg["n"])]
    api_step(layers, nodes, cfg, local)  # warm-up
    _torch_sync(local)
    group.barrier()
    t0 = time.perf_counter()
    steps = max(1, args.steps)
    for _ in range(steps):
        api_step(layers, nodes, cfg, local)
    _torch_sync(local)
    group.barrier()
    t = group.max(time.perf_counter() - t0) / steps
    return {"value": round(world * cfg["n"] / t, 1), "unit": "nodes/s",
            "ms_per_step": round(t * 1e3, 3), "scaling": "weak", "n_gpus": world, "steps": steps,
            "graph": "every rank its own graph of the family through the one-GPU API on its own "
                     "GPU (one process per GPU)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg4", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="auto", choices=["auto", "api", "partitioned"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0, help="faithful sample N override")
    ap.add_argument("--resident-steps", type=int, default=3)
    args = ap.parse_args()

    # a progress line on stderr every 45 s (long configurations: cfg5's synthesis and ingest
    # print nothing for minutes)
    import threading
    t_hb = time.perf_counter()

    def _heartbeat():
        while True:
            time.sleep(45)
            print(f"[bench] {args.config}: {time.perf_counter() - t_hb:.0f} s", file=sys.stderr,
                  flush=True)

    threading.Thread(target=_heartbeat, daemon=True).start()

    world, rank, local = _dist_env()
    if world > 1 and world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world} GPUs",
              file=sys.stderr)
    n_gpus = world if world > 1 else max(1, args.gpus)
    group = _Group(world)
    cfg = CONFIGS[args.config]
    mode = args.mode if args.mode != "auto" else cfg.get("mode", "api")
    if cfg.get("dense") and n_gpus > 1:
        mode = "api"
    devices = list(range(n_gpus)) if n_gpus > 1 else None
    if world > 1 and mode == "api" and devices:
        # rank 0 drives every GPU of the node through the library; should a launcher have hidden
        # the other GPUs from it, the same graph is row-partitioned one process per GPU instead
        visible = n_gpus
        if rank == 0:
            try:
                import torch
                visible = torch.cuda.device_count()  # (does not initialise the GPU here)
            except Exception:
                pass
        visible = int(group.bcast_bytes(str(visible).encode() if rank == 0 else None))
        if visible < n_gpus:
            if rank == 0:
                print(f"warning: rank 0 sees {visible} of {n_gpus} GPUs; the graph is "
                      f"row-partitioned one process per GPU instead", file=sys.stderr)
            mode = "partitioned"
            devices = None
    # (rehearsal on a one-GPU box: N2V2R_BENCH_DEVICES=0,0 runs the N > 1 path over a repeated
    # device -- the library's in-process thread communicator instead of RCCL)
    dev_env = os.environ.get("N2V2R_BENCH_DEVICES")
    if dev_env and world == 1:
        devices = [int(v) for v in dev_env.split(",")]
        n_gpus = len(devices)
        if n_gpus == 1:
            devices = None
    # the headline runs in this process: all of it without torchrun, rank 0's share (the whole
    # multi-GPU API call) under torchrun; per-process partitioned runs on every rank
    per_process = mode == "partitioned" and world > 1
    active = per_process or rank == 0

    from node2vec2rank_amd import _lib, synthetic
    t_build = time.perf_counter()
    b = 32 if cfg.get("dense") else 8  # the solver's default panel width
    eng = None
    nnz = None
    if mode == "partitioned":
        if per_process:
            uid = group.bcast_bytes(_lib.comm_unique_id() if rank == 0 else None)
            eng = _lib.Engine.rccl(local, rank, world, uid)
        else:
            eng = _lib.Engine.multi(devices) if devices else _lib.Engine(local)
        if not devices:
            eng.set_layer_rows(cfg["n"], 2, [])  # the partition first
        _, _, row0, n_local = eng.dist_info()
        if devices:  # one process: the global CSR, each GPU uploads its rows (symmetric)
            rows = [synthetic.er_layer_rows(cfg["n"], cfg["avg_deg"], 2000 + k, 0, cfg["n"])
                    for k in range(2)]
            step = lambda: (eng.set_layers(rows, symmetric=_lib.SYM_YES),  # noqa: E731
                            resident_step(eng, cfg))[1]
        else:
            rows = [synthetic.er_layer_rows(cfg["n"], cfg["avg_deg"], 2000 + k, row0, n_local)
                    for k in range(2)]
            step = lambda: partitioned_step(eng, cfg, rows)  # noqa: E731
        nnz = [int(group.sum(float(a.nnz))) if per_process else int(a.nnz) for a in rows]
    elif active:
        if cfg.get("dense"):
            layers = synthetic.corr_layers(cfg["n"], cfg["layers"], seed_base=0)
            nnz = [int(cfg["n"]) ** 2] * cfg["layers"]
        else:
            layers = synthetic.er_layers(cfg["n"], cfg["avg_deg"], 2, seed_base=1000)
            nnz = [int(a.nnz) for a in layers]
        nodes = [f"n{i}" for i in range(cfg["n"])]
        step = lambda: api_step(layers, nodes, cfg, local, devices)  # noqa: E731
    else:
        step = lambda: None  # noqa: E731  (torchrun ranks > 0: the headline runs on rank 0)
    nodes_per_step = float(cfg["n"])  # one graph, ranked once per step
    t_build = time.perf_counter() - t_build

    for _ in range(args.warmup):
        step()
    _torch_sync(local)
    group.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    _torch_sync(local)
    group.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = group.max(elapsed)
    ncmp = 1  # comparisons per step (K - 1 for "sequential" with K = 2; cfg3: 3)
    stats = None
    if active:
        if mode == "partitioned":
            stats = res[0]
        else:
            ncmp = len(res[1])
            stats = res[0].eig_stats
    value = nodes_per_step * ncmp * args.steps / elapsed_max

    # device-resident form of the same work (layers already in HBM), and one instrumented fit
    # for the roofline (HIP events around every SpMM launch; rank 0's launches on N GPUs)
    res_ms = None
    roof = None
    st_t = {}
    if active:
        if mode == "partitioned":
            reng = eng
        else:
            reng = _lib.Engine.multi(devices) if devices else _lib.Engine(local)
            if cfg.get("dense"):
                reng.set_layers(layers, storage="dense", symmetric=1)
            else:
                reng.set_layers(layers)
        if args.resident_steps > 0:
            resident_step(reng, cfg)  # warm-up: a new handle's first fit allocates its workspace
            reng.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.resident_steps):
                resident_step(reng, cfg)
            reng.synchronize()
            res_ms = (time.perf_counter() - t1) / args.resident_steps * 1e3
        st_t, _ = resident_step(reng, cfg, flags=_lib.EIG_TIME_SPMM)
        _, _, row0, nl = reng.dist_info()
        if devices:  # a multi engine reports rank 0's launches: rows [0, ceil(N / n_gpus))
            nl = (cfg["n"] + n_gpus - 1) // n_gpus
            row0 = 0
        if cfg.get("dense"):
            roof = roofline_from_stats(st_t, cfg, b)
        else:
            if mode == "partitioned" and not devices:
                nnz_launch = [int(a.nnz) for a in rows]     # this rank's own rows
            else:
                nnz_launch = _local_nnz(rows if mode == "partitioned" else layers, row0, nl)
            roof = roofline_from_stats(st_t, cfg, b, nnz_launch, nl)
    if res_ms is not None:
        res_ms = group.max(res_ms) if per_process else res_ms
    if roof is not None and not cfg.get("dense"):
        form = int(st_t.get("spmm_form", 0))
        roof["kernel"] = {0: "spmm8_pipe_kernel (b = 8)",
                          1: "spmm8_pipe_kernel (b = 8, layers split over the XCDs)",
                          5: "spmm8_flat_kernel (row tiles x column-block phases, packed flat "
                             "windows located by window offsets, segment fold into LDS "
                             "accumulators, non-temporal index stream)"
                          }.get(form, str(form))
        # one 32-B panel row gathered per stored entry (served by L2 / Infinity Cache): the
        # line-access rate, reported beside the HBM roofline
        ent = float(sum(nnz_launch))
        roof["gathered_entries_per_launch"] = ent
        roof["gather_G_entries_per_s"] = round(ent / (roof["avg_launch_ms"] * 1e-3) / 1e9, 1)
        # the same launch against the measured gather ceiling (tools/gather_ceiling.hip, 32-B
        # rows from a 2 MB L2-resident panel with the 4-B index stream:
        # profiles/r04_gather_ceiling.jsonl)
        roof["gather_ceiling_G_entries_per_s"] = GATHER_CEILING_G
        roof["gather_ceiling_frac"] = round(roof["gather_G_entries_per_s"] / GATHER_CEILING_G, 3)
        if n_gpus > 1:
            roof["per_gpu"] = (f"rank 0's launches ({nl} of {cfg['n']} rows, "
                               f"{int(sum(nnz_launch))} entries per launch)")
    tpath = os.path.join(REPO, "profiles", "spmm_traffic.json")
    if roof is not None and os.path.exists(tpath) and n_gpus == 1:
        try:
            t = json.load(open(tpath))
            # the record must come from the same config, stage, SpMM form and kernel revision
            if (t.get("config") == args.config and t.get("stage") == roof["stage"]
                    and t.get("spmm_form") == int(st_t.get("spmm_form", -1))
                    and t.get("kernel_rev") == SPMM_KERNEL_REV):
                roof["traffic"] = t.get("bytes_per_launch")
                roof["traffic_source"] = t.get("source")
                if t.get("fabric_read_requests_per_launch") is not None:
                    roof["traffic_requests"] = t.get("fabric_read_requests_per_launch")
        except Exception:
            pass

    if mode == "partitioned":
        par = (f"row-partitioned x{n_gpus}, one process per GPU (RCCL)" if per_process else
               f"row-partitioned x{n_gpus}, one process (RCCL over {n_gpus} devices)"
               if devices else "row-partitioned x1")
    else:
        par = (f"row-partitioned x{n_gpus} by the library: N2V2R(..., devices=range({n_gpus})), "
               f"one process, one host thread per GPU, RCCL over the devices" if devices else
               "single GPU")
    result = {
        "metric": BASELINE_METRIC,
        "metric_detail": "nodes ranked/sec (fit_transform_rank + aggregate_transform, host CSR "
                         "in, host DataFrames out); the SpMM GB/s half is roofline.achieved",
        "value": round(value, 1),
        "unit": "nodes/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {"workload": cfg["desc"], "nodes": cfg["n"], "layers": cfg.get("layers", 2),
                   "avg_degree": cfg["avg_deg"], "nnz_per_layer": nnz, "embed_dim": cfg["d"],
                   "columns": len(cfg["dims"]) * len(METRICS), "comparisons": ncmp,
                   "parallelism": par,
                   "timed_path": ("per-rank CSR rows -> HBM + UASE + distances + Borda -> host"
                                  if mode == "partitioned" else
                                  "host CSR -> N2V2R -> fit_transform_rank -> "
                                  "aggregate_transform -> host DataFrames (H2D included)")},
        "roofline": roof,
        # solver counters of the timed fit (ms_spmm / ms_ortho are host-side launch times of
        # asynchronous work, so they are left out; the device time is in roofline)
        "eig": {k: (float(f"{v:.4g}") if isinstance(v, float) else v)
                for k, v in (stats or {}).items() if k not in ("ms_spmm", "ms_ortho")},
        "setup_s": round(t_build, 2),
    }
    if res_ms is not None:
        result["device_resident"] = {"ms_per_step": round(res_ms, 3),
                                     "value": round(nodes_per_step * ncmp / (res_ms * 1e-3), 1)}
    # torchrun at N > 1: side legs beside the headline, each under a watchdog (rank 0 prints the
    # line with a leg marked as timed out and every rank exits with WATCHDOG_EXIT) --
    # N2V2R_BENCH_SIDE=0 skips them
    if (world > 1 and mode == "api" and not cfg.get("dense")
            and os.environ.get("N2V2R_BENCH_SIDE", "1") != "0"):
        limit = float(os.environ.get("N2V2R_BENCH_SIDE_S", "300"))
        legs = [("replicas", replicas_leg)]
        if os.environ.get("N2V2R_BENCH_SIDE") == "all":  # (opt-in: an RCCL world per process)
            legs.append(("partitioned_per_process", strong_scaling))
        for key, fn in legs:
            def _expire(key=key):
                if rank == 0:
                    result[key] = {"error": f"timed out after {limit:g} s"}
                    print(json.dumps(result), flush=True)

            def _leg(fn=fn):
                try:
                    return fn(group, cfg, args, local, rank, world)
                except Exception as e:  # reported in the line; the headline stands
                    return {"error": repr(e)[:300]}

            result[key] = run_guarded(_leg, limit, _expire)
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        avail, how = host_cpus()
        # the reference's pool: joblib n_jobs=-2 = all CPUs but one (model_utils.py:31-32)
        workers = max(1, avail - 1)
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample or CPU_SAMPLE[args.config],
                                              workers)
        result["cpu_baseline"]["host"]["cpus_available"] = avail
        result["cpu_baseline"]["host"]["cpus_available_from"] = how
    if rank == 0:
        print(json.dumps(result), flush=True)
    if eng is not None:
        eng.close()
    elif active:
        reng.close()
    group.close()


if __name__ == "__main__":
    main()
