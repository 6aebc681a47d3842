"""GPU, BASELINE configs C5 and C4 at their stated sizes, through the real HIP exchange path
(adfl_amd.exchange.PeerExchange: HipCodec encode -> all-gather -> fused decode-mean), every simulated client
a process sharing cuda:0 (the reference packs two clients per GPU, Examples/ray_ad.py:29; RCCL needs one
device per rank, so the rows travel over gloo through pinned host memory as in test_gpu_exchange_k2.py):

* C5: K = 2 clients x 2^30 fp32 (4 GiB) each, SLQ bits 4, int4-packed, chunks = 8 (quantize of chunk c
      overlapped with the all-gather of chunk c-1);
* C5 at its stated client count: K = 8 x 2^30 int4-packed, chunks = 8 (the mean checked at sampled positions);
* C4: K = 8 clients x 2^28 fp32 (1 GiB) each, SLQ bits 8.

Client r's update is randn(n) * 1e-3 from a device generator seeded r. Checks, on every rank:
  1. the rank's own message rows (payload + scale trailer) equal the oracle's encode of its update;
  2. every received row's SHA-256 equals the SHA-256 of its sender's oracle payload (all-gathered), so the
     gathered rows ARE the oracle payloads;
  3. the SHA-256 of the rank's mean equals the SHA-256 of oracle.dequantize_mean_self over those rows with
     the rank's own fp32 update exact (Src/ADFL/Client/async_peer.py:170-174, Examples/ray_ad.py:183-188).
"""

import hashlib
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _sha(a) -> str:
    return hashlib.sha256(memoryview(np.ascontiguousarray(a)).cast("B")).hexdigest()


def _sampled_mean_check(out, rows, scales, xh, rank, packed, m=1 << 16):
    """The mean at m random positions (the same for every rank) against the oracle over just those columns.
    numel and m are multiples of 32, so every column sums in the same (SEQ) order whatever its index
    (csrc/torch_sum_order.h), and the oracle over the sampled columns is the oracle at those positions."""
    import slq_oracle as oracle
    numel = xh.size
    assert numel % 32 == 0 and m % 32 == 0
    idx = np.sort(np.random.default_rng(12345).choice(numel, size=m, replace=False))
    qs = []
    for r in range(len(rows)):
        if packed:
            b = rows[r][idx // 2].astype(np.int16)
            qv = np.where(idx % 2 == 0, (b >> 4) & 0xF, b & 0xF) - 8
            qs.append(qv.astype(np.int8))
        else:
            qs.append(rows[r][idx].view(np.int8))
    want = oracle.dequantize_mean_self(qs, scales, m, rank, np.ascontiguousarray(xh[idx]), False)
    got = out[idx]
    return bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))


def _worker(rank, world, port, numel, bits, packed, chunks, q, sampled=False):
    try:
        sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import torch.distributed as dist
        import slq_oracle as oracle
        from adfl_amd.exchange import PeerExchange

        t0 = time.perf_counter()
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        g = torch.Generator(device=dev).manual_seed(rank)
        x = torch.randn(numel, device=dev, generator=g) * 1e-3
        ex = PeerExchange(numel, bits=bits, packed=packed, chunks=chunks, device=dev)
        assert ex.host_staged and len(ex.bounds) == chunks
        t1 = time.perf_counter()
        out = ex.exchange_mean(x)
        torch.cuda.synchronize()
        t_exchange = time.perf_counter() - t1

        # 1. own rows = the oracle's encode of this rank's update (payload bytes and scale trailer)
        xh = x.cpu().numpy()
        del x
        qo, so = oracle.encode(xh, bits)
        payload = oracle.pack_int4(qo) if packed else qo.view(np.uint8)
        del qo
        own_ok = True
        pos = 0
        for (c0, c1), loc, pb in zip(ex.bounds, ex.local, ex.payload):
            row = loc.cpu().numpy()
            off = (pb + 15) // 16 * 16
            own_ok &= bool(np.array_equal(row[:pb], payload[pos:pos + pb]))
            own_ok &= bool(row[off:off + 4].view(np.float32)[0].view(np.uint32) == np.float32(so).view(np.uint32))
            pos += pb
        own_ok &= pos == payload.size

        # 2. every received row is its sender's oracle payload
        sent = [None] * world
        dist.all_gather_object(sent, [_sha(payload[sum(ex.payload[:c]):sum(ex.payload[:c + 1])])
                                      for c in range(len(ex.payload))])
        rows = [np.empty(payload.size, np.uint8) for _ in range(world)]
        scales = np.empty(world, np.float32)
        rows_ok = True
        pos = 0
        for c, (g_rows, pb) in enumerate(zip(ex.gathered, ex.payload)):
            gh = g_rows.cpu().numpy()
            off = (pb + 15) // 16 * 16
            for r in range(world):
                rows_ok &= _sha(gh[r, :pb]) == sent[r][c]
                rows[r][pos:pos + pb] = gh[r, :pb]
                if c == 0:
                    scales[r] = gh[r, off:off + 4].view(np.float32)[0]
            pos += pb
        del payload

        # 3. the mean = oracle.dequantize_mean_self over the (verified) oracle rows, own update exact
        if sampled:   # K = 8 x 2^30: the oracle at 2^16 sampled positions (same order as the full vector)
            ok = _sampled_mean_check(out.cpu().numpy(), rows, scales, xh, rank, packed)
            got_sha, want_sha = ("sampled" if ok else "sampled-mismatch"), "sampled"
        else:
            want = oracle.dequantize_mean_self(rows, scales, numel, rank, xh, packed)
            got_sha, want_sha = _sha(out.cpu().numpy()), _sha(want)
        q.put((rank, {"own_rows_equal_oracle": own_ok, "received_rows_equal_oracle": rows_ok,
                      "mean_sha256": got_sha, "oracle_mean_sha256": want_sha,
                      "exchange_s": round(t_exchange, 3), "total_s": round(time.perf_counter() - t0, 1)}))
        dist.destroy_process_group()
    except BaseException as e:  # surfaced to the parent
        import traceback
        q.put((rank, f"error {e!r}\n{traceback.format_exc()}"))


def _run(world, numel, bits, packed, chunks, limit_s, sampled=False):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, numel, bits, packed, chunks, q, sampled))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.time() + limit_s
    try:
        while len(res) < world and time.time() < deadline:
            try:
                r, v = q.get(timeout=5)
                res[r] = v
                if isinstance(v, str):
                    break
            except Exception:  # queue.Empty: keep waiting while ranks are alive
                if not any(p.is_alive() for p in procs) and q.empty():
                    break
    finally:
        for p in procs:
            p.join(timeout=30 if len(res) == world else 1)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(5)
    errors = [v for v in res.values() if isinstance(v, str)]
    assert not errors, "\n".join(errors)
    assert len(res) == world, f"only ranks {sorted(res)} reported within {limit_s} s"
    for r, v in sorted(res.items()):
        print(f"rank {r}: {v}")
        assert v["own_rows_equal_oracle"], (r, v)
        assert v["received_rows_equal_oracle"], (r, v)
        assert v["mean_sha256"] == v["oracle_mean_sha256"], (r, v)
    return res


@pytest.mark.timeout(300)
def test_c5_two_clients_4gib_int4_packed_chunks8():
    _run(world=2, numel=1 << 30, bits=4, packed=True, chunks=8, limit_s=280)


@pytest.mark.timeout(560)
def test_c5_eight_clients_4gib_int4_packed_chunks8():
    """BASELINE configs[4] at its stated client count (Examples/ray_ad.py:183-188): 8 clients x 2^30 fp32,
    int4-packed in 8 chunks. Rows checked in full (own = oracle encode, received = senders' SHA-256); the
    8-row mean against the oracle at 2^16 sampled positions on every rank."""
    _run(world=8, numel=1 << 30, bits=4, packed=True, chunks=8, limit_s=540, sampled=True)


@pytest.mark.timeout(300)
def test_c4_eight_clients_1gib_int8():
    _run(world=8, numel=1 << 28, bits=8, packed=False, chunks=1, limit_s=280)
