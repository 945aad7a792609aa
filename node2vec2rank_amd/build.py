"""Build libn2v2r_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the
repository snapshot to the GPU box).

    python -m node2vec2rank_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "lib")
# N2V2R_BUILD_TAG=x: an experimental build beside the product library (lib/libn2v2r_hip_x.so,
# objects in lib/obj_x), loaded only by a process that sets N2V2R_LIB to it (A/B probes)
_TAG = os.environ.get("N2V2R_BUILD_TAG", "")
LIB = os.path.join(OUT_DIR, f"libn2v2r_hip_{_TAG}.so" if _TAG else "libn2v2r_hip.so")
OBJ_DIR = os.path.join(OUT_DIR, f"obj_{_TAG}" if _TAG else "obj")

HIP_SOURCES = ["spmm.hip", "dense.hip", "gemm.hip", "rank.hip", "rr.hip", "rr_band.hip",
               "rr_sturm.hip", "ingest.hip", "pair.hip", "engine.cpp", "layers.cpp", "comm.cpp",
               "solver.cpp", "ranking.cpp", "multi.cpp"]
HOST_SOURCES: list = []
HEADERS = ["common.h", "spmm_args.h", "engine.h", os.path.join("..", "..", "include", "n2v2r.h"),
           os.path.join("..", "..", "include", "n2v2r_diag.h")]
ARCH = os.environ.get("N2V2R_OFFLOAD_ARCH", "gfx950")
# probe builds only (with N2V2R_BUILD_TAG): extra -D flags for the HIP sources
_EXTRA = os.environ.get("N2V2R_EXTRA_HIP_FLAGS", "").split() if _TAG else []


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, h) for h in HEADERS]
    objs, cmds = [], []
    for src in HIP_SOURCES + HOST_SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJ_DIR, src + ".o")
        objs.append(obj)
        if not force and not _newer(obj, [path, __file__] + headers):
            continue
        if src in HIP_SOURCES:
            lang = ["-x", "hip"]
            cmd = [hipcc, *lang, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-munsafe-fp-atomics", *_EXTRA, "-c", path, "-o", obj]
        else:
            cmd = ["g++", "-O3", "-march=x86-64-v3", "-std=c++17", "-fPIC", "-c", path, "-o", obj]
        cmds.append(cmd)
    # the sources compile independently: a few hipcc processes at once
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(8, len(cmds), os.cpu_count() or 1))

    def _run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(_run, cmds))
    if force or _newer(LIB, objs):
        # linked beside the library and renamed over it, so a reader never sees a partial file
        tmp = LIB + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp,
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
