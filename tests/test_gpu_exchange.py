"""GPU: the peer exchange's HIP path (HipCodec + RCCL all-gather + fused decode-mean) on one rank.

Multi-rank behaviour of the protocol is covered by tests/test_exchange_gloo.py (world_size 2, gloo,
oracle codec); here the real device codec and the RCCL collective run end to end (world_size 1 on the
single-GPU test box), and the rows a K-rank gather would deliver are fed to the mean kernel directly."""

import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import slq_oracle as oracle

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def rccl_world1():
    pytest.importorskip("adfl_amd")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=DEV)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("numel,bits,packed,chunks", [(1 << 20, 8, False, 1), (1000003, 8, False, 3),
                                                      (1 << 22, 4, True, 4), (4097, 4, True, 2),
                                                      (70000, 2, False, 1)])
def test_exchange_world1_matches_oracle(rccl_world1, numel, bits, packed, chunks):
    from adfl_amd.exchange import PeerExchange
    rng = np.random.default_rng(numel)
    x = rng.standard_normal(numel, dtype=np.float32) * np.float32(1e-3)
    ex = PeerExchange(numel, bits=bits, packed=packed, chunks=chunks, device=DEV, exact_self=False)
    got = ex.exchange_mean(torch.from_numpy(x).to(DEV)).cpu().numpy()
    q, s = oracle.encode(x, bits)
    want = oracle.decode_int4(oracle.pack_int4(q), numel, s) if packed else oracle.decode(q, s)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    # the gathered message rows carry payload + scale exactly as the protocol lays them out
    for (c0, c1), rows, pb in zip(ex.bounds, ex.gathered, ex.payload):
        r = rows.cpu().numpy()[0]
        scale = r[(pb + 15) // 16 * 16:(pb + 15) // 16 * 16 + 4].view(np.float32)[0]
        assert np.float32(scale).view(np.uint32) == np.float32(s).view(np.uint32)


def test_exchange_world1_exact_self_is_identity(rccl_world1):
    """With the reference's mean (own update exact, async_peer.py:170-174), one rank's mean is its update."""
    from adfl_amd.exchange import PeerExchange
    x = torch.randn(1000003, device=DEV) * 1e-3
    for packed, bits in ((False, 8), (True, 4)):
        ex = PeerExchange(x.numel(), bits=bits, packed=packed, chunks=3, device=DEV)
        assert torch.equal(ex.exchange_mean(x), x)


def test_exchange_k8_rows_mean_self(rccl_world1):
    """Rank 3 of an 8-way gather with its own update exact: rows 0-2, 4-7 decoded, then x added last."""
    from adfl_amd import ops
    k, n, me = 8, 300007, 3
    rng = np.random.default_rng(9)
    xs = [rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -r) for r in range(k)]
    enc = [oracle.encode(x, 8) for x in xs]
    row = (n + 15) // 16 * 16 + 16
    rows = np.zeros((k, row), np.uint8)
    for r, (q, s) in enumerate(enc):
        rows[r, :n] = q.view(np.uint8)
        rows[r, row - 16:row - 12] = np.array([s], np.float32).view(np.uint8)
    rows_d = torch.from_numpy(rows).to(DEV)
    scales = rows_d[:, row - 16:].view(torch.float32)[:, :1].contiguous()
    got = ops.dequantize_mean(rows_d.view(torch.int8), scales, n, self_row=me,
                              self_x=torch.from_numpy(xs[me]).to(DEV)).cpu().numpy()
    want = oracle.dequantize_mean_self([q for q, _ in enc], [s for _, s in enc], n, me, xs[me])
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    stack = [oracle.decode(q, s) for r, (q, s) in enumerate(enc) if r != me] + [xs[me]]
    ref = torch.stack([torch.from_numpy(d) for d in stack]).mean(0).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-30)


def test_exchange_k8_rows_mean(rccl_world1):
    """What rank r computes after an 8-way gather: decode-mean over 8 rows of a real exchange layout."""
    from adfl_amd import ops
    k, n = 8, 300007
    rng = np.random.default_rng(8)
    xs = [rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -r) for r in range(k)]
    enc = [oracle.encode(x, 8) for x in xs]
    row = (n + 15) // 16 * 16 + 16
    rows = np.zeros((k, row), np.uint8)
    for r, (q, s) in enumerate(enc):
        rows[r, :n] = q.view(np.uint8)
        rows[r, row - 16:row - 12] = np.array([s], np.float32).view(np.uint8)
    rows_d = torch.from_numpy(rows).to(DEV)
    scales = rows_d[:, row - 16:].view(torch.float32)[:, :1]
    got = ops.dequantize_mean(rows_d.view(torch.int8), scales.contiguous(), n).cpu().numpy()
    want = oracle.dequantize_mean([q for q, _ in enc], [s for _, s in enc])
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("align", [1, 64])
def test_bucket_exchange_world1_over_rccl(rccl_world1, align):
    """PeerExchange(layout=...) through RCCL at world 1: one client's state dict with per-tensor scales
    (quant.py:74-94) comes back as its own SLQ round trip per tensor (exact_self=False), the row carries
    the bucket payload and the T scales, and the gaps between tensors stay zero."""
    from adfl_amd import ops
    from adfl_amd.exchange import PeerExchange
    sizes = [3, 8193, 45662, 17, 70001]
    lay = ops.BucketLayout(sizes, align=align)
    rng = np.random.default_rng(align)
    flat = np.zeros(lay.total, np.float32)
    for t, (o, n) in enumerate(zip(lay.offsets.tolist(), sizes)):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -t)
    ex = PeerExchange(lay.total, device=DEV, exact_self=False, layout=lay)
    assert not ex.host_staged
    got = ex.exchange_mean(torch.from_numpy(flat).to(DEV)).cpu().numpy()
    q, s = oracle.encode_batched(flat, lay.offsets, lay.sizes, 8)
    want = np.zeros(lay.total, np.float32)
    for t, (o, n) in enumerate(zip(lay.offsets.tolist(), sizes)):
        want[o:o + n] = oracle.decode(q[o:o + n], s[t])
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    row = ex.gathered[0].cpu().numpy()[0]
    off = (lay.total + 15) // 16 * 16
    assert np.array_equal(row[off:off + 4 * len(sizes)].view(np.float32).view(np.uint32), s.view(np.uint32))
    # exact_self: one rank's mean is its own update
    ex2 = PeerExchange(lay.total, device=DEV, layout=lay)
    x = torch.from_numpy(flat).to(DEV)
    assert torch.equal(ex2.exchange_mean(x), x)


@pytest.mark.parametrize("case", ["flat_in_order", "flat_side_stream", "int4_chunks", "bucket", "bucket_int4"])
def test_exchange_graph_replays_equal_eager(rccl_world1, case):
    """PeerExchange.graph: the whole exchange (encode, RCCL all-gather, fused mean; the side-stream chunk
    pipeline included) captured once as a HIP graph; every replay on new contents of x equals the eager
    exchange and the oracle's decode (exact_self=False at world 1: the mean is the rank's own round trip)."""
    from adfl_amd import ops
    from adfl_amd.exchange import PeerExchange
    lay = None
    numel, bits, packed, chunks = {"flat_in_order": (1 << 20, 8, False, 1), "flat_side_stream": (1000003, 8, False, 3),
                                   "int4_chunks": (1 << 21, 4, True, 4), "bucket": (None, 8, False, 1),
                                   "bucket_int4": (None, 4, True, 1)}[case]
    if numel is None:
        lay = ops.BucketLayout([3, 8193, 45662, 17, 70001])
        numel = lay.total
    ex = PeerExchange(numel, bits=bits, packed=packed, chunks=chunks, device=DEV, exact_self=False, layout=lay)
    x = torch.zeros(numel, device=DEV)
    out = torch.empty(numel, device=DEV)
    g = ex.graph(x, out)
    for seed in (1, 2, 3):
        xn = np.random.default_rng(seed).standard_normal(numel, dtype=np.float32) * np.float32(10.0 ** -seed)
        if lay is not None:   # gaps stay zero, as the bucket's producer leaves them
            mask = np.zeros(numel, bool)
            for o, n in zip(lay.offsets.tolist(), lay.sizes.tolist()):
                mask[o:o + n] = True
            xn[~mask] = 0.0
        x.copy_(torch.from_numpy(xn))
        got = g.replay().cpu().numpy()
        eager = ex.exchange_mean(torch.from_numpy(xn).to(DEV)).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), eager.view(np.uint32)), seed
        if lay is None:
            q, s = oracle.encode(xn, bits)
            want = oracle.decode_int4(oracle.pack_int4(q), numel, s) if packed else oracle.decode(q, s)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), seed


def test_exchange_graph_rejects_host_staging(rccl_world1):
    """Rows staged through host memory over gloo cannot be captured: graph() refuses instead of capturing
    a partial step."""
    from adfl_amd.exchange import PeerExchange
    gl = dist.new_group(backend="gloo")
    ex = PeerExchange(4096, device=DEV, group=gl)
    assert ex.host_staged
    with pytest.raises(ValueError, match="RCCL"):
        ex.graph(torch.zeros(4096, device=DEV), torch.empty(4096, device=DEV))
    dist.destroy_process_group(gl)
