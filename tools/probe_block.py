"""Block-width probe at a BASELINE config: one fit per block width b, printing wall time,
cycles, block / vector applications, the fit's SpMM device time (HIP events per launch) and the
residual -- the numbers behind the choice of b.

    python tools/probe_block.py [--config cfg4] [--blocks 8 16] [--keep K --basis C]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from node2vec2rank_amd import _lib, synthetic  # noqa: E402

CONFIGS = {"cfg2": (100_000, 20.0, 64), "cfg4": (1_000_000, 50.0, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4", choices=sorted(CONFIGS))
    ap.add_argument("--blocks", type=int, nargs="+", default=[8, 16])
    ap.add_argument("--keep", type=int, default=0)
    ap.add_argument("--basis", type=int, default=0)
    ap.add_argument("--sweep", nargs="*", default=[],
                    help="keep:basis pairs to run at the first block width (0 = default)")
    a = ap.parse_args()
    n, deg, d = CONFIGS[a.config]
    layers = synthetic.er_layers(n, deg, 2, seed_base=1000)
    eng = _lib.Engine(0)
    eng.set_layers(layers)
    runs = [(b, a.keep, a.basis) for b in a.blocks]
    runs += [(a.blocks[0], int(x.split(":")[0]), int(x.split(":")[1])) for x in a.sweep]
    for b, keep, basis in runs:
        a.keep, a.basis = keep, basis
        eng.uase(d, block=b, seed=42, keep=a.keep, max_basis=a.basis)  # warm (allocations)
        eng.synchronize()
        t0 = time.perf_counter()
        st = eng.uase(d, block=b, seed=42, keep=a.keep, max_basis=a.basis)
        eng.synchronize()
        wall = time.perf_counter() - t0
        st_t = eng.uase(d, block=b, seed=42, keep=a.keep, max_basis=a.basis,
                        solver_flags=_lib.EIG_TIME_SPMM)
        print(json.dumps(dict(config=a.config, block=b, keep=keep, basis=basis,
                              wall_ms=round(wall * 1e3, 1),
                              restarts=st["restarts"], block_applications=st["block_applications"],
                              vector_applications=st["block_applications"] * b,
                              max_residual=st["max_residual"], converged=st["converged"],
                              spmm_form=st["spmm_form"],
                              spmm_gpu_ms=st_t["gpu_ms_spmm"],
                              spmm_launches=st_t["spmm_timed_launches"])), flush=True)


if __name__ == "__main__":
    main()
