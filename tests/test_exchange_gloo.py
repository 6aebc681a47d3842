"""CPU, world_size 2 (gloo): the peer-exchange protocol of adfl_amd.exchange — message layout, scale
trailer, chunked pipelining, rank-ordered mean — with the oracle codec injected in place of the HIP
codec (the HIP path itself is covered by tests/test_gpu_exchange.py on the GPU)."""

import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import slq_oracle as oracle


class OracleCodec:
    """Test double for exchange.HipCodec built on the oracle (CPU tensors)."""

    def absmax(self, x):
        xa = np.ascontiguousarray(x.numpy())
        self.absmax_val = oracle.lib().oracle_slq_absmax(xa.ctypes.data, xa.size)

    def quantize(self, x, bits, packed, row, payload_bytes):
        scale = np.float32(oracle.lib().oracle_slq_scale(self.absmax_val, bits))
        xa = np.ascontiguousarray(x.numpy())
        q = np.empty(xa.size, np.int8)
        oracle.lib().oracle_slq_quantize(xa.ctypes.data, xa.size, ctypes.c_float(scale), q.ctypes.data)
        payload = oracle.pack_int4(q) if packed else q.view(np.uint8)
        r = row.numpy()
        r[:payload_bytes] = payload
        off = (payload_bytes + 15) // 16 * 16
        r[off:off + 4] = np.array([scale], np.float32).view(np.uint8)

    def mean(self, rows, n, packed, payload_bytes, out, self_row=-1, self_x=None):
        r = rows.numpy()
        off = (payload_bytes + 15) // 16 * 16
        scales = np.ascontiguousarray(r[:, off:off + 4]).view(np.float32).reshape(-1)
        if self_row >= 0:
            res = oracle.dequantize_mean_self([r[k, :payload_bytes] for k in range(r.shape[0])], scales, n,
                                              self_row, self_x.numpy(), packed)
        elif packed:
            res = oracle.dequantize_mean_int4([r[k, :payload_bytes] for k in range(r.shape[0])], scales, n)
        else:
            res = oracle.dequantize_mean([r[k, :payload_bytes].view(np.int8) for k in range(r.shape[0])], scales)
        out.copy_(torch.from_numpy(res))


def _update(rank, numel):
    rng = np.random.default_rng(1000 + rank)
    x = rng.standard_normal(numel, dtype=np.float32) * np.float32(10.0 ** (-rank))
    return x


def _expected(world, numel, bits, packed):
    decoded = []
    for r in range(world):
        q, s = oracle.encode(_update(r, numel), bits)
        decoded.append(oracle.decode_int4(oracle.pack_int4(q), numel, s) if packed else oracle.decode(q, s))
    return decoded


def _mean_self_numpy(rows):
    """fp32 sum in list order, then / K — torch.stack(updates).mean(0)'s value up to its summation order."""
    acc = rows[0].copy()
    for d in rows[1:]:
        acc = (acc + d).astype(np.float32)
    return (acc.astype(np.float64) / len(rows)).astype(np.float32)


def _worker(rank, world, port, cases, errors):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "ad-federatedlearning_amd"))
        from adfl_amd.exchange import PeerExchange
        for numel, bits, packed, chunks, exact_self in cases:
            ex = PeerExchange(numel, bits=bits, packed=packed, chunks=chunks, device=torch.device("cpu"),
                              codec=OracleCodec(), exact_self=exact_self)
            x = torch.from_numpy(_update(rank, numel))
            got = ex.exchange_mean(x).numpy()
            decoded = _expected(world, numel, bits, packed)
            if exact_self:
                # the reference's mean: received updates, then the local fp32 update appended last
                decoded = [d for r, d in enumerate(decoded) if r != rank] + [_update(rank, numel)]
                want = _mean_self_numpy(decoded)
            elif packed:
                want = oracle.dequantize_mean_int4(
                    [oracle.pack_int4(oracle.encode(_update(r, numel), bits)[0]) for r in range(world)],
                    [oracle.encode(_update(r, numel), bits)[1] for r in range(world)], numel)
            else:
                qs = [oracle.encode(_update(r, numel), bits) for r in range(world)]
                want = oracle.dequantize_mean([q for q, _ in qs], [s for _, s in qs])
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (rank, numel, bits, packed, chunks)
            ref = torch.stack([torch.from_numpy(d) for d in decoded]).mean(0).numpy()
            np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-30)
            assert ex.bytes_per_rank == sum(ex.row_bytes)
        dist.destroy_process_group()
    except Exception as e:  # surfaced to the parent
        import traceback
        errors.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_peer_exchange_gloo(world):
    cases = [(1000, 8, False, 1, False), (4097, 8, False, 3, False), (12345, 4, True, 4, False),
             (33, 4, True, 1, False), (64, 2, False, 2, False),
             (1000, 8, False, 1, True), (4097, 8, False, 3, True), (12345, 4, True, 4, True), (33, 4, True, 1, True)]
    ctx = mp.get_context("spawn")
    errors = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, errors)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    msgs = []
    while not errors.empty():
        msgs.append(errors.get())
    assert not msgs, "\n".join(msgs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
