"""GPU: the decentralized exchange of a whole state dict under SLQChannel's per-tensor codec — every
client's bucket encoded with one scale per tensor (Src/ADFL/Channel/quant.py:74-94), all-gathered, and
averaged per tensor (Examples/ray_ad.py:164-190; own update exact, Src/ADFL/Client/async_peer.py:170-174).

* adfl_slq_dequantize_mean_batched[_int4] (ops.dequantize_mean_batched) against oracle.dequantize_mean_batched
  bit for bit: K rows, int8 and int4-packed (PackedSLQChannel per tensor), compact and aligned layouts
  (head / tile / tail paths), multi-chunk tensors, with and without the receiver's own row exact;
* PeerExchange(layout=...) with K = 2 clients sharing cuda:0 (host-staged over gloo) on the C3 layouts
  (ResNet-18's 11,689,512 parameters in 256 tensors, equal and log-uniform sizes), bit-exact against the
  oracle on independently encoded buckets and within 1e-6 of torch.stack(...).mean(0) per tensor."""

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import slq_oracle as oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DEV = torch.device("cuda", 0)


def _bucket(lay, seed, scale=1e-3):
    rng = np.random.default_rng(seed)
    flat = np.zeros(lay.total, np.float32)
    for t, (o, n) in enumerate(zip(lay.offsets.tolist(), lay.sizes.tolist())):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(scale * 10.0 ** -(t % 4))
    return flat


@pytest.mark.parametrize("align", [1, 64])
@pytest.mark.parametrize("k,self_row", [(1, -1), (3, -1), (3, 1), (5, 4)])
def test_dequantize_mean_batched_matches_oracle(k, self_row, align):
    from adfl_amd import ops
    sizes = [1, 15, 17, 1024, 1040, 8192, 8193, 30001, 3]
    lay = ops.BucketLayout(sizes, align=align)
    row = (lay.total + 15) // 16 * 16
    rows = np.zeros((k, row), np.int8)
    scales = np.zeros((k, lay.ntensors), np.float32)
    flats = [_bucket(lay, 10 * k + r) for r in range(k)]
    for r, f in enumerate(flats):
        q, s = oracle.encode_batched(f, lay.offsets, lay.sizes, 8)
        rows[r, :lay.total] = q
        scales[r] = s
    self_x = torch.from_numpy(flats[self_row]).to(DEV) if self_row >= 0 else None
    got = ops.dequantize_mean_batched(torch.from_numpy(rows).to(DEV), torch.from_numpy(scales).to(DEV), lay,
                                      self_row=self_row, self_x=self_x).cpu().numpy()
    want = oracle.dequantize_mean_batched(list(rows), list(scales), lay.offsets, lay.sizes, lay.total, self_row,
                                          flats[self_row] if self_row >= 0 else None)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("align", [2, 64])
@pytest.mark.parametrize("k,self_row", [(1, -1), (3, -1), (3, 1), (5, 4)])
def test_dequantize_mean_batched_int4_matches_oracle(k, self_row, align):
    from adfl_amd import ops
    sizes = [1, 15, 17, 1024, 2047, 2080, 8192, 8193, 30001, 3]
    lay = ops.BucketLayout(sizes, align=align)
    pb = (lay.total + 1) // 2
    rows = np.zeros((k, (pb + 15) // 16 * 16), np.uint8)
    scales = np.zeros((k, lay.ntensors), np.float32)
    flats = [_bucket(lay, 20 * k + r) for r in range(k)]
    for r, f in enumerate(flats):
        q, s = oracle.encode_batched(f, lay.offsets, lay.sizes, 4)
        rows[r, :pb] = oracle.pack_int4(q)
        scales[r] = s
    # the device int4 encode makes the same rows
    p_dev, s_dev = ops.encode_batched_int4(torch.from_numpy(flats[0]).to(DEV), lay, 4)
    got_p = p_dev.cpu().numpy()
    for o, n in zip(lay.offsets.tolist(), lay.sizes.tolist()):
        assert np.array_equal(got_p[o // 2:(o + n) // 2], rows[0, o // 2:(o + n) // 2])
    assert np.array_equal(s_dev.cpu().numpy().view(np.uint32), scales[0].view(np.uint32))
    self_x = torch.from_numpy(flats[self_row]).to(DEV) if self_row >= 0 else None
    got = ops.dequantize_mean_batched(torch.from_numpy(rows).to(DEV), torch.from_numpy(scales).to(DEV), lay,
                                      self_row=self_row, self_x=self_x, packed=True).cpu().numpy()
    want = oracle.dequantize_mean_batched(list(rows), list(scales), lay.offsets, lay.sizes, lay.total, self_row,
                                          flats[self_row] if self_row >= 0 else None, packed=True)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_dequantize_mean_batched_int4_rejects_odd_offsets():
    from adfl_amd import ops
    lay = ops.BucketLayout([3, 5], align=1)
    rows = torch.zeros(2, 16, dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError):
        ops.dequantize_mean_batched(rows, torch.ones(2, 2, device=DEV), lay, packed=True)


def _worker(rank, world, port, errors):
    try:
        sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
        import torch.distributed as dist
        import recipes
        import slq_oracle as oracle
        from adfl_amd import ops
        from adfl_amd.exchange import PeerExchange

        torch.cuda.set_device(DEV)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        for name, align, exact_self, packed in [("equal", 64, True, False), ("loguniform", 1, True, False),
                                                ("equal", 1, False, False), ("loguniform", 2, True, True)]:
            sizes = recipes.bucket_sizes(name) if name == "equal" else recipes.bucket_sizes(name, 0)
            lay = ops.BucketLayout(sizes, align=align)
            bits = 4 if packed else 8
            ex = PeerExchange(lay.total, bits=bits, packed=packed, device=DEV, exact_self=exact_self, layout=lay)
            assert ex.host_staged
            flats = [_bucket(lay, 500 + r) for r in range(world)]
            for _ in range(2):   # staging and row buffers reused
                got = ex.exchange_mean(torch.from_numpy(flats[rank]).to(DEV)).cpu().numpy()
            encs = [oracle.encode_batched(f, lay.offsets, lay.sizes, bits) for f in flats]
            self_row = rank if exact_self else -1
            payloads = [oracle.pack_int4(q) if packed else q for q, _ in encs]
            want = oracle.dequantize_mean_batched(payloads, [s for _, s in encs], lay.offsets, lay.sizes,
                                                  lay.total, self_row, flats[rank] if exact_self else None,
                                                  packed=packed)
            case = (rank, name, align, exact_self, packed)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), case
            for t, (o, n) in enumerate(zip(lay.offsets.tolist(), lay.sizes.tolist())):
                dec = [oracle.decode(q[o:o + n], s[t]) for r, (q, s) in enumerate(encs)
                       if not (exact_self and r == rank)]
                if exact_self:
                    dec.append(flats[rank][o:o + n])
                ref = torch.stack([torch.from_numpy(d) for d in dec]).mean(0).numpy()
                np.testing.assert_allclose(got[o:o + n], ref, rtol=1e-6, atol=1e-30, err_msg=str(case + (t,)))
        dist.destroy_process_group()
    except BaseException as e:  # surfaced to the parent
        import traceback
        errors.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


def test_bucket_exchange_two_clients_c3_layouts():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    errors = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, errors)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=110)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join(5)
    msgs = []
    while not errors.empty():
        msgs.append(errors.get())
    assert not alive, "exchange ranks did not finish within 110 s"
    assert not msgs, "\n".join(msgs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
