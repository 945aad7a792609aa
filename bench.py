"""Benchmark: nodes ranked/s of the fit-and-rank path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg1|cfg4|cfg5]
                    [--mode auto|replicas|partitioned]

One step = ``fit_transform_rank()`` + ``aggregate_transform()`` of the engine on one synthetic
2-layer graph whose CSR layers are already resident in HBM: UASE (block Krylov-Schur on the
GPU), distances for every (dim, metric) column, Borda, and the copy of the distance table and
Borda scores back to the host (what the reference API returns).  Default workload is
BASELINE.json configs[1] (cfg2: 2-layer ER N=100k, avg-deg 20, d=64).

Multi-GPU (torchrun, one process per GPU), two modes:
  * replicas (default for cfg1/2/4): every rank ranks its own independent graph (different
    generator seeds), no data-path collective, "scaling": "weak";
  * partitioned (default for cfg5): ONE graph row-partitioned over the ranks (RCCL communicator
    of the engine: panel all-gathers per SpMM stage, all-reduce of the Gram / Rayleigh-Ritz /
    residual reductions), every rank builds only its own rows (counter-based ER generator),
    "scaling": "strong".
A gloo group provides the barrier, the max-over-ranks of the timed region and the broadcast
of the RCCL unique id.

Extra JSON fields: ``roofline`` (SpMM kernel, HIP-event timed on the engine stream at the
Krylov panel width) and ``cpu_baseline`` (the reference algorithm restated in oracle/, on a
bounded sample, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
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
CPU_SAMPLE = {"cfg1": 1000, "cfg2": 50_000, "cfg3": 2_000, "cfg4": 20_000, "cfg5": 20_000}
METRICS = ["cosine", "euclidean"]
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Scattered-line ceiling of the vector memory path: MI355X_MICROARCH.md's indexed-row gather
# (1,152-B rows from an L2-resident table) runs 66-73 GB/s per CU = one 128-B line per ~4.4
# cycles per CU, i.e. 256 CUs x 2.4 GHz / 4.4 = ~140 G lines/s.  A b = 8 SpMM touches one line
# per stored entry (its 32-B panel row), whatever the locality (tools/spmm_locality.py: ER vs
# a 256-wide band graph, 14.5 vs 12.6 us per 2M entries), so this, not HBM, bounds it.
GATHER_LINE_PEAK_GLPS = 256 * 2.4 / 4.4


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

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def _torch_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def run_step(eng, cfg, seed, fetch=True, eig=None):
    st = eng.uase(cfg["d"], seed=seed, **(eig or {}))
    ncmp, _ = eng.rank("sequential", cfg["dims"], METRICS)
    out = []
    if fetch:  # the reference API hands the distance table and the Borda scores to the caller
        for c in range(ncmp):
            out.append((eng.distances(c), eng.borda(c)))
    return st, out


def cpu_baseline(sample_n=20_000, avg_deg=20.0, d=64, dims=(64,), dense_layers=0):
    """Reference algorithm (oracle/, faithful mode) on a bounded sample, 1 thread:
    ARPACK svds + per-row scipy distances + the O(C N^2) list.index Borda."""
    import scipy.sparse as sp
    from threadpoolctl import threadpool_limits

    from node2vec2rank_amd import synthetic
    from oracle import n2v2r_oracle as orc
    if dense_layers:
        layers = [sp.csc_matrix(a) for a in synthetic.corr_layers(sample_n, dense_layers)]
    else:
        layers = synthetic.er_layers(sample_n, avg_deg, 2, seed_base=7000)
    with threadpool_limits(1):
        t0 = time.time()
        Y, _, _ = orc.uase(layers, d, seed=42)
        t1 = time.time()
        ranks = orc.rank_distances(Y, list(dims), METRICS, "sequential", faithful=True)
        t2 = time.time()
        for _, (_, D) in ranks.items():
            orc.borda_reference_loop(D)
        t3 = time.time()
    total = t3 - t0
    fam = (f"{dense_layers}-layer dense |corrcoef| N={sample_n}" if dense_layers else
           f"2-layer ER N={sample_n} avg-deg {avg_deg:g}")
    return {
        "value": sample_n * len(ranks) / total, "unit": "nodes/s", "cores": 1, "kind": "port",
        "sample": (f"{fam}, d={d}, dims {list(dims)} x cosine+euclidean (the bench workload's "
                   f"graph family at fewer nodes; the Borda stage is O(C N^2) so the "
                   f"full-size rate is lower), oracle faithful mode, 1 thread"),
        "stages_s": {"svds": round(t1 - t0, 3), "distances": round(t2 - t1, 3),
                     "borda": round(t3 - t2, 3)},
    }


def _layers_partitioned(cfg, row0, n_local):
    from node2vec2rank_amd import synthetic
    return [synthetic.er_layer_rows(cfg["n"], cfg["avg_deg"], 2000 + k, row0, n_local)
            for k in range(2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "partitioned"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0)
    ap.add_argument("--eig", default="", help='solver knobs as JSON, e.g. {"block": 16, '
                    '"max_basis": 512, "keep": 320} (default: the engine defaults)')
    args = ap.parse_args()

    world, rank, local = _dist_env()
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    group = _Group(world)
    cfg = CONFIGS[args.config]
    mode = args.mode if args.mode != "auto" else cfg.get("mode", "replicas")
    eig = json.loads(args.eig) if args.eig else {}

    from node2vec2rank_amd import _lib, synthetic
    t_build = time.perf_counter()
    if mode == "partitioned":
        if world > 1:
            uid = group.bcast_bytes(_lib.comm_unique_id() if rank == 0 else None)
            eng = _lib.Engine.rccl(local, rank, world, uid)
        else:
            eng = _lib.Engine(local)
        eng.set_layer_rows(cfg["n"], 2, [])  # partition first
        _, _, row0, n_local = eng.dist_info()
        local_layers = _layers_partitioned(cfg, row0, n_local)
        nnz = [int(group.sum(float(a.nnz))) for a in local_layers]
        eng.set_layer_rows(cfg["n"], 2, local_layers)  # local CSR rows -> HBM, untimed
        del local_layers
        seed = 42
        nodes_per_step = float(cfg["n"])  # one graph, ranked once, over all ranks
    elif cfg.get("dense"):
        eng = _lib.Engine(local)
        layers = synthetic.corr_layers(cfg["n"], cfg["layers"], seed_base=17 * rank)
        nnz = [int(cfg["n"]) ** 2] * cfg["layers"]
        eng.set_layers(layers, storage="dense", symmetric=1)  # dense fp32 -> HBM, untimed
        del layers
        seed = 42 + rank
        nodes_per_step = group.sum(float(cfg["n"]))
    else:
        eng = _lib.Engine(local)
        layers = synthetic.er_layers(cfg["n"], cfg["avg_deg"], 2, seed_base=1000 + 17 * rank)
        nnz = [int(a.nnz) for a in layers]
        eng.set_layers(layers)  # CSR -> HBM, untimed (inputs resident when timing starts)
        del layers
        seed = 42 + rank
        nodes_per_step = group.sum(float(cfg["n"]))  # every rank ranks its own graph
    t_build = time.perf_counter() - t_build
    fetch = mode == "replicas" or rank == 0

    for _ in range(args.warmup):
        run_step(eng, cfg, seed, fetch, eig)
    eng.synchronize()
    _torch_sync()
    group.barrier()
    t0 = time.perf_counter()
    stats = None
    for _ in range(args.steps):
        stats, _ = run_step(eng, cfg, seed, fetch, eig)
    eng.synchronize()
    _torch_sync()
    group.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = group.max(elapsed)
    ncmp = eng.ncmp  # comparisons per step (K - 1 for "sequential")
    value = nodes_per_step * ncmp * args.steps / elapsed_max

    # dominant kernel: the CSR x panel SpMM at the Krylov panel width, HIP events on the
    # engine stream (same launch configuration as inside UASE; this rank's rows when
    # partitioned)
    b = int(eig.get("block", 0)) or (32 if cfg.get("dense") else 8)  # the solver's panel width
    X = np.random.default_rng(0).standard_normal((cfg["n"], b)).astype(np.float32)
    col_blocks = (not cfg.get("dense")) and eng.spmm_col_blocks(b)
    nloc_rows = float(eng.dist_info()[3])
    _, spmm_ms, spmm_bytes = eng.bench_spmm(0, X, reps=50, want_y=False)
    del X
    achieved = spmm_bytes / (spmm_ms * 1e-3) / 1e9
    # panel rows gathered per launch (4 b bytes per nnz, served by L2 / Infinity Cache): not
    # HBM bytes, reported beside the roofline
    gathered = (None if cfg.get("dense") else
                4.0 * b * float(nnz[0]) / max(1, world if mode == "partitioned" else 1))
    lines_per_launch = (None if gathered is None else
                        float(nnz[0]) / max(1, world if mode == "partitioned" else 1)
                        * max(1, (4 * b) // 128))
    ms_dist, ms_borda = eng.rank_timing()

    traffic = None
    tpath = os.path.join(REPO, "profiles", "spmm_traffic.json")
    if os.path.exists(tpath) and world == 1:
        try:
            t = json.load(open(tpath))
            if t.get("config") == args.config and int(t.get("b", -1)) == b:
                traffic = t.get("bytes_per_launch")
        except Exception:
            traffic = None

    if mode == "partitioned":
        par = f"row-partitioned x{world} (RCCL)" if world > 1 else "row-partitioned x1"
    else:
        par = f"replicas x{world}" if world > 1 else "single"
    result = {
        "metric": "nodes ranked/sec (fit_transform_rank + aggregate_transform)",
        "value": round(value, 1),
        "unit": "nodes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if mode == "partitioned" else "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {"workload": cfg["desc"], "nodes": cfg["n"], "layers": cfg.get("layers", 2),
                   "avg_degree": cfg["avg_deg"], "nnz_per_layer": nnz, "embed_dim": cfg["d"],
                   "columns": len(cfg["dims"]) * len(METRICS), "comparisons": ncmp,
                   "parallelism": par},
        "roofline": {"bound": "hbm",
                     "kernel": ("dense_gemm_kernel<1> (A_k X, MFMA f32)" if cfg.get("dense")
                                else ("spmm8_cb_kernel<*> + cb_reduce_kernel (b=8, XCD-local "
                                      "column blocks)" if col_blocks
                                      else ("spmm8_pipe_kernel<*> (b=8)" if b == 8
                                            else f"spmm_csr_panel_kernel<{b},*>"))),
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "algo_bytes_per_launch": spmm_bytes, "avg_launch_ms": round(spmm_ms, 5),
                     "gathered_bytes_per_launch": gathered,
                     # column blocks: 8 partial outputs written and re-read by the reduce
                     # (HBM bytes beyond the algorithmic ones)
                     "partial_bytes_per_launch": (2.0 * 8 * 4 * 8 * nloc_rows
                                                  if col_blocks else 0.0),
                     "gather_GBps": (None if gathered is None else
                                     round(gathered / (spmm_ms * 1e-3) / 1e9, 1)),
                     # the bound that applies: 128-B lines touched by the panel-row gathers
                     # (one per stored entry while a panel row fits one line)
                     "gather_lines_per_launch": (None if gathered is None else
                                                 lines_per_launch),
                     "gather_line_rate_Glps": (None if gathered is None else
                                               round(lines_per_launch / (spmm_ms * 1e-3) / 1e9, 1)),
                     "gather_line_peak_Glps": round(GATHER_LINE_PEAK_GLPS, 1),
                     "gather_line_frac": (None if gathered is None else
                                          round(lines_per_launch / (spmm_ms * 1e-3) / 1e9
                                                / GATHER_LINE_PEAK_GLPS, 4))},
        "eig": {k: (float(f"{v:.4g}") if isinstance(v, float) else v) for k, v in stats.items()},
        "eig_options": eig,
        "rank_ms": {"distances": round(ms_dist, 3), "borda": round(ms_borda, 3)},
        "setup_s": round(t_build, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(
            sample_n=args.cpu_sample or CPU_SAMPLE[args.config], avg_deg=cfg["avg_deg"],
            d=cfg["d"], dims=tuple(cfg["dims"]),
            dense_layers=cfg["layers"] if cfg.get("dense") else 0)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    group.close()


if __name__ == "__main__":
    main()
