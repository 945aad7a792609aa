"""Multi-process control plane of bench.py (weak-scaling replicas): barrier, max and sum over
ranks with world_size 2 on gloo (CPU)."""
import os
import socket

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    w, r, lr = bench._dist_env()
    g = bench._Group(w)
    g.barrier()
    mx = g.max(float(rank + 1))
    sm = g.sum(100.0 * (rank + 1))
    g.close()
    q.put((r, lr, mx, sm))


def test_bench_group_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [o[0] for o in out] == [0, 1]
    assert all(o[2] == 2.0 for o in out)        # max over ranks
    assert all(o[3] == 300.0 for o in out)      # whole-job sum


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    g = bench._Group(world)
    got = g.bcast_bytes(b"\x00uid\xff" * 25 if rank == 0 else None)
    g.close()
    q.put((rank, got))


def test_bench_unique_id_broadcast_world2():
    """The RCCL unique id (128 opaque bytes) travels from rank 0 over the gloo control plane."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(o[1] == b"\x00uid\xff" * 25 for o in out)
