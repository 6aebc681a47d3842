"""CPU, world_size 2 (gloo): bench.py's multi-rank plumbing — torchrun-style env setup, barrier and the
max-over-ranks step time the whole-job value is computed from."""

import os
import socket
import sys

import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    try:
        os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, repo)
        import bench
        import torch.distributed as dist
        w, r, local = bench.dist_setup(None, backend="gloo")
        assert (w, r, local) == (world, rank, rank)
        bench.barrier(w)
        slowest = bench.max_over_ranks(0.5 + rank, w)     # rank 1 is the slow one
        value = w * 1.0 / slowest                          # bench.py: world * GiB / max step time
        q.put((rank, slowest, value))
        dist.destroy_process_group()
    except Exception as e:  # surfaced in the parent
        q.put((rank, "error", repr(e)))


def test_bench_max_over_ranks_gloo():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] != "error" for r in res), res
    assert sorted(res) == [(0, 1.5, 2 / 1.5), (1, 1.5, 2 / 1.5)]
