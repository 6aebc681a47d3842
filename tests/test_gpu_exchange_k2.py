"""GPU, K = 2 ranks: the real HIP exchange path (HipCodec encode -> all-gather -> fused decode-mean) with two
simulated clients sharing cuda:0 — the reference's packing of two clients per GPU (``NUM_GPUS = 0.5``,
Examples/ray_ad.py:29). RCCL cannot put two ranks on one device, so the rows travel over gloo through
pinned host memory (PeerExchange's host-staged transport); encode and mean are the HIP kernels.

Checked per rank against the oracle (bit-exact) and against the reference's own
``torch.stack(updates).mean(0)`` (Examples/ray_ad.py:188; async_peer.py:170-174) within 1e-6 relative."""

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

# (numel, bits, packed, chunks, exact_self): int8 flat, ragged int8 chunked, chunked int4 (C5's shape at
# a test size), int4 ragged tail
CASES = [(1 << 20, 8, False, 1, True), (1000003, 8, False, 3, True), (1 << 22, 4, True, 4, True),
         (4097, 4, True, 2, True), (1 << 20, 8, False, 1, False), (1 << 22, 4, True, 4, False)]


def _update(rank, numel):
    rng = np.random.default_rng(7000 + rank)
    return rng.standard_normal(numel, dtype=np.float32) * np.float32(10.0 ** (-2 - rank))


def _worker(rank, world, port, errors):
    try:
        sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import torch.distributed as dist
        import slq_oracle as oracle
        from adfl_amd.exchange import PeerExchange

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        for numel, bits, packed, chunks, exact_self in CASES:
            ex = PeerExchange(numel, bits=bits, packed=packed, chunks=chunks, device=dev, exact_self=exact_self)
            assert ex.host_staged
            xs = [_update(r, numel) for r in range(world)]
            for rep in range(2):  # twice: the staging buffers are reused across calls
                got = ex.exchange_mean(torch.from_numpy(xs[rank]).to(dev)).cpu().numpy()
            encs = [oracle.encode(x, bits) for x in xs]
            if packed:
                rows = [oracle.pack_int4(q) for q, _ in encs]
                decoded = [oracle.decode_int4(p, numel, s) for p, (_, s) in zip(rows, encs)]
            else:
                rows = [q for q, _ in encs]
                decoded = [oracle.decode(q, s) for q, s in encs]
            scales = [s for _, s in encs]
            if exact_self:
                want = oracle.dequantize_mean_self(rows, scales, numel, rank, xs[rank], packed)
                stack = [d for r, d in enumerate(decoded) if r != rank] + [xs[rank]]
            else:
                want = (oracle.dequantize_mean_int4(rows, scales, numel) if packed
                        else oracle.dequantize_mean(rows, scales))
                stack = decoded
            case = (rank, numel, bits, packed, chunks, exact_self)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), case
            ref = torch.stack([torch.from_numpy(d) for d in stack]).mean(0).numpy()
            np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-30, err_msg=str(case))
        dist.destroy_process_group()
    except BaseException as e:  # surfaced to the parent
        import traceback
        errors.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


def test_exchange_two_clients_one_gpu():
    pytest.importorskip("adfl_amd")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    errors = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errors)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join(5)
    msgs = []
    while not errors.empty():
        msgs.append(errors.get())
    assert not alive, "exchange ranks did not finish within 100 s"
    assert not msgs, "\n".join(msgs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
