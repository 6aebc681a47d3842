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

    def encode_bucket(self, x, layout, bits, row, packed=False):
        q, scales = oracle.encode_batched(np.ascontiguousarray(x.numpy()), layout.offsets, layout.sizes, bits)
        payload = oracle.pack_int4(q[:layout.total]) if packed else q.view(np.uint8)[:layout.total]
        r = row.numpy()
        r[:payload.size] = payload
        off = (payload.size + 15) // 16 * 16
        r[off:off + 4 * layout.ntensors] = scales.view(np.uint8)

    def mean_bucket(self, rows, layout, out, self_row=-1, self_x=None, packed=False):
        r = rows.numpy()
        pb = (layout.total + 1) // 2 if packed else layout.total
        off = (pb + 15) // 16 * 16
        scales = [np.ascontiguousarray(r[k, off:off + 4 * layout.ntensors]).view(np.float32) for k in range(r.shape[0])]
        res = oracle.dequantize_mean_batched([r[k, :pb] for k in range(r.shape[0])], scales, layout.offsets,
                                             layout.sizes, layout.total, self_row,
                                             self_x.numpy() if self_x is not None else None, packed=packed)
        out.copy_(torch.from_numpy(res))

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
        try:   # host tensors cannot be captured into a HIP graph: refused, not half-captured
            ex.graph(torch.zeros(ex.numel), torch.zeros(ex.numel))
            raise AssertionError("PeerExchange.graph accepted host tensors")
        except ValueError:
            pass
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


def _bucket_update(rank, layout):
    rng = np.random.default_rng(2000 + rank)
    flat = np.zeros(layout.total, np.float32)
    for t, (o, n) in enumerate(zip(layout.offsets, layout.sizes)):
        flat[o:o + n] = rng.standard_normal(int(n), dtype=np.float32) * np.float32(10.0 ** -(t % 3 + rank))
    return flat


def _bucket_worker(rank, world, port, cases, errors):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, os.path.join(os.path.dirname(here), "ad-federatedlearning_amd"))
        from adfl_amd.exchange import PeerExchange
        from adfl_amd.ops import BucketLayout
        for sizes, align, exact_self, packed in cases:
            lay = BucketLayout(sizes, align=align)
            bits = 4 if packed else 8
            ex = PeerExchange(lay.total, bits=bits, packed=packed, device=torch.device("cpu"), codec=OracleCodec(),
                              exact_self=exact_self, layout=lay)
            pb = (lay.total + 1) // 2 if packed else lay.total
            assert ex.row_bytes == [(pb + 15) // 16 * 16 + (4 * lay.ntensors + 15) // 16 * 16]
            got = ex.exchange_mean(torch.from_numpy(_bucket_update(rank, lay))).numpy()
            # per tensor, the reference's mean: every rank's update SLQ-encoded with its own per-tensor
            # scales (quant.py:74-94) and decoded; with exact_self this rank's own update enters exact, last
            for t, (o, n) in enumerate(zip(lay.offsets.tolist(), lay.sizes.tolist())):
                dec = []
                for r in range(world):
                    x = _bucket_update(r, lay)[o:o + n]
                    if exact_self and r == rank:
                        continue
                    q, sc = oracle.encode(x, bits)
                    dec.append(oracle.decode_int4(oracle.pack_int4(q), n, sc) if packed else oracle.decode(q, sc))
                if exact_self:
                    dec.append(_bucket_update(rank, lay)[o:o + n])
                ref = torch.stack([torch.from_numpy(d) for d in dec]).mean(0).numpy()
                np.testing.assert_allclose(got[o:o + n], ref, rtol=1e-6, atol=1e-30, err_msg=str((sizes, t)))
            gaps = np.ones(lay.total, bool)
            for o, n in zip(lay.offsets.tolist(), lay.sizes.tolist()):
                gaps[o:o + n] = False
            assert (got[gaps] == 0).all()
        dist.destroy_process_group()
    except Exception as e:  # surfaced to the parent
        import traceback
        errors.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


def test_peer_exchange_bucket_gloo():
    """A whole state dict per rank (BucketLayout: SLQChannel's per-tensor scales) through the exchange
    protocol: the row carries the bucket payload (int8, or int4-packed) and one scale per tensor, the mean
    is per tensor."""
    cases = [([1000, 7, 4097, 33], 1, True, False), ([1000, 7, 4097, 33], 64, False, False),
             ([8193, 5, 64], 64, True, False), ([1000, 7, 4097, 33], 2, True, True),
             ([8193, 5, 65], 64, False, True)]
    ctx = mp.get_context("spawn")
    errors = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, cases, errors)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    msgs = []
    while not errors.empty():
        msgs.append(errors.get())
    assert not msgs, "\n".join(msgs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
