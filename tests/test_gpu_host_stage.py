"""GPU: the native staging-range calls of the host-resident channel path (include/adfl_host.h,
adfl_stage_encode_range / adfl_stage_decode_range, csrc/host_stage.hip).

A compact ragged bucket is pushed through the calls range by range exactly as the pipelined SLQChannel paths
drive them (tensors reduced and quantized on the device once their last byte is staged; chunks decoded once
staged; ranges that complete nothing enqueue the H2D alone), and the payload, scales and floats that come back
through pinned memory must equal the one-launch device encode / decode bit for bit (ops.encode_batched /
decode_batched, themselves pinned to the reference by the channel and golden suites).
"""

import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from adfl_amd import _lib, ops  # noqa: E402
from adfl_amd.Channel import quant  # noqa: E402

DEV = torch.device("cuda", 0)
E_ARG = -1


def _layout(sizes):
    return ops.BucketLayout(sizes, align=1)


def _cuts(total, nranges):
    c = np.linspace(0, total, nranges + 1).astype(np.int64)
    return list(zip(c[:-1].tolist(), c[1:].tolist()))


@pytest.mark.parametrize("sizes,nranges", [
    ([1], 1),
    ([3, 8192, 8193, 5, 70000, 1, 16385], 4),
    ([100_000] * 3 + [17] * 9 + [250_000], 8),
    ([8192 * 7 + 3, 2, 40_000, 123_457], 16),   # more ranges than some tensors: ranges that complete nothing
])
def test_encode_ranges_match_one_launch(sizes, nranges):
    lib = _lib.load()
    lay = _layout(sizes)
    g = torch.Generator().manual_seed(len(sizes) * 7 + nranges)
    x = (torch.randn(lay.total, generator=g) * 1e-3)
    x[::997] *= 40.0
    x_host = x.pin_memory()
    x_dev = torch.empty(lay.total, device=DEV)
    q_dev = torch.empty(lay.total, dtype=torch.int8, device=DEV)
    q_host = torch.full((lay.total,), 77, dtype=torch.int8).pin_memory()
    s_dev = torch.full((lay.ntensors,), -1.0, device=DEV)
    part_dev = torch.full((lay.nchunks,), -1, dtype=torch.int32, device=DEV)
    chunks = lay.device_chunks(DEV)
    cm = quant._chunk_meta(lay)
    ends = lay.offsets + lay.sizes
    evs = (ctypes.c_void_p * (2 * nranges))()
    assert lib.adfl_stage_events_create(2 * nranges, evs) == 0
    side = torch.cuda.Stream(DEV)
    sh = torch.cuda.current_stream(DEV).cuda_stream
    made = 0
    try:
        for r, (lo, hi) in enumerate(_cuts(lay.total, nranges)):
            done = int(np.searchsorted(ends, hi, side="right"))
            c0 = c1 = e0 = e1 = 0
            if done > made:
                c0, c1 = int(cm.first[made]), int(cm.cend[done - 1])
                e0, e1 = int(lay.offsets[made]), int(ends[done - 1])
            rc = lib.adfl_stage_encode_range(x_host.data_ptr(), x_dev.data_ptr(), lo, hi, part_dev.data_ptr(),
                                             chunks.data_ptr(), c0, c1 - c0, 8,
                                             q_dev.data_ptr(), s_dev.data_ptr(), q_host.data_ptr(), e0, e1, sh,
                                             side.cuda_stream, evs[2 * r], evs[2 * r + 1])
            assert rc == 0
            made = done
        assert made == lay.ntensors
        torch.cuda.synchronize()
        q_ref, s_ref = ops.encode_batched(x.to(DEV), lay, 8)
        assert torch.equal(x_dev.cpu(), x)
        assert torch.equal(q_host, q_ref.cpu())
        assert torch.equal(s_dev.cpu().view(torch.int32), s_ref.cpu().view(torch.int32))
        # the device reduced every chunk itself: its partials are each chunk's max|x| bits
        bits = x.numpy().view(np.uint32) & np.uint32(0x7FFFFFFF)
        want = np.array([bits[a:b].max() for a, b in zip(cm.start, cm.end)], dtype=np.uint32)
        assert np.array_equal(part_dev.cpu().numpy().view(np.uint32), want)
    finally:
        torch.cuda.synchronize()
        lib.adfl_stage_events_destroy(evs, 2 * nranges)


@pytest.mark.parametrize("sizes,nranges", [
    ([1], 1),
    ([3, 8192, 8193, 5, 70000, 1, 16385], 4),
    ([100_000] * 3 + [17] * 9 + [250_000], 8),
    ([8192 * 7 + 3, 2, 40_000, 123_457], 32),
])
def test_decode_ranges_match_one_launch(sizes, nranges):
    lib = _lib.load()
    lay = _layout(sizes)
    g = torch.Generator().manual_seed(len(sizes) * 11 + nranges)
    q = torch.randint(-128, 128, (lay.total,), generator=g, dtype=torch.int8)
    scales = torch.rand(lay.ntensors, generator=g) * 1e-4
    q_host = q.pin_memory()
    q_dev = torch.empty(lay.total, dtype=torch.int8, device=DEV)
    out_dev = torch.empty(lay.total, device=DEV)
    out_host = torch.full((lay.total,), float("nan")).pin_memory()
    s_dev = scales.to(DEV)
    chunks = lay.device_chunks(DEV)
    cm = quant._chunk_meta(lay)
    evs = (ctypes.c_void_p * (2 * nranges))()
    assert lib.adfl_stage_events_create(2 * nranges, evs) == 0
    side = torch.cuda.Stream(DEV)
    sh = torch.cuda.current_stream(DEV).cuda_stream
    c_made = 0
    try:
        for r, (lo, hi) in enumerate(_cuts(lay.total, nranges)):
            c_end = int(np.searchsorted(cm.end, hi, side="right"))
            if c_end <= c_made:
                rc = lib.adfl_stage_decode_range(q_host.data_ptr(), q_dev.data_ptr(), lo, hi, chunks.data_ptr(), 0, 0,
                                                 s_dev.data_ptr(), out_dev.data_ptr(), out_host.data_ptr(), 0, 0, sh,
                                                 side.cuda_stream, evs[2 * r], evs[2 * r + 1])
            else:
                e0, e1 = int(cm.start[c_made]), int(cm.end[c_end - 1])
                rc = lib.adfl_stage_decode_range(q_host.data_ptr(), q_dev.data_ptr(), lo, hi, chunks.data_ptr(),
                                                 c_made, c_end - c_made, s_dev.data_ptr(), out_dev.data_ptr(),
                                                 out_host.data_ptr(), e0, e1, sh, side.cuda_stream, evs[2 * r],
                                                 evs[2 * r + 1])
                c_made = c_end
            assert rc == 0
        assert c_made == lay.nchunks
        torch.cuda.synchronize()
        ref = ops.decode_batched(q.to(DEV), s_dev, lay).cpu()
        assert torch.equal(out_host.view(torch.int32), ref.view(torch.int32))
    finally:
        torch.cuda.synchronize()
        lib.adfl_stage_events_destroy(evs, 2 * nranges)


def test_stage_argument_errors():
    lib = _lib.load()
    buf = torch.empty(64, device=DEV)
    hb = torch.empty(64).pin_memory()
    p = buf.data_ptr()
    h = hb.data_ptr()
    # a negative count, a reversed range, a kernel range with no events: refused, nothing enqueued
    assert lib.adfl_stage_encode_range(h, p, 0, 64, p, p, 0, -1, 8, p, p, h, 0, 64, None, None, None, None) == E_ARG
    assert lib.adfl_stage_encode_range(h, p, 10, 5, p, p, 0, 0, 8, p, p, h, 0, 0, None, None, None, None) == E_ARG
    assert lib.adfl_stage_encode_range(h, p, 0, 64, p, p, 0, 1, 8, p, p, h, 0, 64, None, None, None, None) == E_ARG
    assert lib.adfl_slq_absmax_batched_range(p, p, 0, 0, p, None) == E_ARG
    assert lib.adfl_stage_decode_range(h, p, 0, 64, p, 0, 1, p, p, h, 0, 64, None, None, None, None) == E_ARG
    assert lib.adfl_stage_decode_range(None, p, 0, 64, p, 0, 0, p, p, h, 0, 0, None, None, None, None) == E_ARG
    assert lib.adfl_stage_events_create(-1, None) == E_ARG
    torch.cuda.synchronize()


def test_channel_payload_and_scales_are_the_devices(monkeypatch):
    """The host's max|x| (reduced during the gather) only lets the channel build the qint8 outputs early: the
    payload and the scale of every entry are the device's. With the host's scales deliberately off by one ulp
    the channel must still return exactly what it returns normally."""
    from adfl_amd.Channel import SLQChannel
    g = torch.Generator().manual_seed(3)
    params = {f"l{i}.weight": torch.randn(17, 300 + 97 * i, generator=g) * 1e-3 for i in range(12)}
    params.update({f"l{i}.bias": torch.randn(17, generator=g) for i in range(12)})
    ch = SLQChannel(8)
    want, _ = ch.on_client_send(params)
    real = quant._host_scales
    monkeypatch.setattr(quant, "_host_scales", lambda a, b: np.nextafter(real(a, b), np.float32(np.inf)))
    got, _ = ch.on_client_send(params)
    for n, p in want.params.items():
        q = got.params[n]
        assert q.scale == p.scale
        if p.data.is_quantized:
            assert q.data.q_scale() == p.data.q_scale()
            assert torch.equal(q.data.int_repr(), p.data.int_repr())


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
@pytest.mark.parametrize("sizes,nranges", [([3, 8192, 8193, 5, 70000, 1, 16385], 4),
                                           ([8192 * 7 + 3, 2, 40_000, 123_457], 32)])
def test_stoch_decode_ranges_match_one_launch(codec, sizes, nranges):
    """adfl_stage_stoch_decode_range: both byte planes staged range by range, each completed chunk range decoded
    by the codec's kernel, floats back through pinned memory — equal to the one-launch decode bit for bit."""
    from adfl_amd import stoch as sops
    lib = _lib.load()
    lay = _layout(sizes)
    g = torch.Generator().manual_seed(nranges + len(codec))
    bits = 4
    if codec == "cnat":
        lv = torch.randint(-20, 3, (lay.total,), generator=g, dtype=torch.int8).view(torch.uint8)
    else:
        lv = torch.randint(0, 16, (lay.total,), generator=g, dtype=torch.uint8)
    sg = (torch.randint(0, 2, (lay.total,), generator=g, dtype=torch.int8) * 2 - 1)
    norms = torch.rand(lay.ntensors, generator=g) * 3
    norms[1] = 0.0                                   # the norm == 0 branch
    mins = torch.rand(lay.ntensors, generator=g) * 1e-3
    lv_h, sg_h = lv.pin_memory(), sg.pin_memory()
    lv_d = torch.empty(lay.total, dtype=torch.uint8, device=DEV)
    sg_d = torch.empty(lay.total, dtype=torch.int8, device=DEV)
    out_d = torch.empty(lay.total, device=DEV)
    out_h = torch.full((lay.total,), float("nan")).pin_memory()
    n_d, m_d = norms.to(DEV), mins.to(DEV)
    chunks = lay.device_chunks(DEV)
    cm = quant._chunk_meta(lay)
    evs = (ctypes.c_void_p * (2 * nranges))()
    assert lib.adfl_stage_events_create(2 * nranges, evs) == 0
    side = torch.cuda.Stream(DEV)
    sh = torch.cuda.current_stream(DEV).cuda_stream
    cid = {"qsgd": 0, "rqsgd": 1, "cnat": 2}[codec]
    mp = m_d.data_ptr() if codec == "rqsgd" else None
    c_made = 0
    try:
        for r, (lo, hi) in enumerate(_cuts(lay.total, nranges)):
            c_end = int(np.searchsorted(cm.end, hi, side="right"))
            cnt, e0, e1 = 0, 0, 0
            if c_end > c_made:
                cnt, e0, e1 = c_end - c_made, int(cm.start[c_made]), int(cm.end[c_end - 1])
            rc = lib.adfl_stage_stoch_decode_range(cid, bits, lv_h.data_ptr(), lv_d.data_ptr(), sg_h.data_ptr(),
                                                   sg_d.data_ptr(), lo, hi, chunks.data_ptr(), c_made if cnt else 0,
                                                   cnt, n_d.data_ptr(), mp, out_d.data_ptr(), out_h.data_ptr(), e0,
                                                   e1, sh, side.cuda_stream, evs[2 * r], evs[2 * r + 1])
            assert rc == 0
            c_made = max(c_made, c_end)
        torch.cuda.synchronize()
        lvd, sgd = lv.to(DEV), sg.to(DEV)
        if codec == "qsgd":
            ref = sops.qsgd_decode_batched(lvd, sgd, n_d, lay, bits)
        elif codec == "rqsgd":
            ref = sops.rqsgd_decode_batched(lvd, sgd, n_d, m_d, lay, bits)
        else:
            ref = sops.cnat_decode_batched(lvd.view(torch.int8), sgd, n_d, lay)
        assert torch.equal(out_h.view(torch.int32), ref.cpu().view(torch.int32))
        # RQSGD without mins, or an unknown codec: refused
        assert lib.adfl_stage_stoch_decode_range(1, bits, lv_h.data_ptr(), lv_d.data_ptr(), sg_h.data_ptr(),
                                                 sg_d.data_ptr(), 0, 0, chunks.data_ptr(), 0, 1, n_d.data_ptr(), None,
                                                 out_d.data_ptr(), out_h.data_ptr(), 0, 1, sh, side.cuda_stream,
                                                 evs[0], evs[1]) == E_ARG
        assert lib.adfl_stage_stoch_decode_range(7, bits, lv_h.data_ptr(), lv_d.data_ptr(), sg_h.data_ptr(),
                                                 sg_d.data_ptr(), 0, 0, chunks.data_ptr(), 0, 0, n_d.data_ptr(), None,
                                                 out_d.data_ptr(), out_h.data_ptr(), 0, 0, sh, side.cuda_stream,
                                                 evs[0], evs[1]) == E_ARG
    finally:
        torch.cuda.synchronize()
        lib.adfl_stage_events_destroy(evs, 2 * nranges)


@pytest.mark.parametrize("cls", ["QSGDChannel", "RQSGDChannel", "CNATChannel"])
def test_stoch_host_encode_ranges_match_whole_bucket(cls, monkeypatch):
    """The range-pipelined stochastic host encode (each range's completed tensors encoded over a sub-layout at
    their bucket offsets) gives the whole-bucket encode's bytes: same seed, same levels / exponents, signs,
    norms and minima, with staging ranges cutting through tensors, a zero tensor and single elements."""
    import importlib
    C = importlib.import_module("adfl_amd.Channel")
    ch = getattr(C, cls)(8)
    g = torch.Generator().manual_seed(5)
    sizes = [3 * 8192 + 5, 17, 100_000, 9, 70_001, 1, 250_000] + [4096] * 20
    params = {f"w{i}": torch.randn(1, n, generator=g) * 1e-2 for i, n in enumerate(sizes)}
    params["w3"].zero_()
    params["b"] = torch.randn(10, generator=g)
    monkeypatch.setattr(quant, "_PIECE_BYTES", 1 << 16)   # many ranges
    got = ch._quantize_params(params, 8, seed=1234)
    monkeypatch.setattr(quant, "_PIPELINE", False)
    want = ch._quantize_params(params, 8, seed=1234)
    for n in params:
        a, b = got.params[n], want.params[n]
        assert float(a.scale) == float(b.scale) and float(a.scale_2) == float(b.scale_2), n
        if params[n].ndim > 1:
            assert a.data.dtype == b.data.dtype and a.data.shape == b.data.shape
            assert torch.equal(a.data.view(torch.uint8), b.data.view(torch.uint8)), n
            assert torch.equal(a.signs, b.signs), n
    assert got.size == want.size
