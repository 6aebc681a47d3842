"""GPU: the torch.ops.adfl.* custom ops (SURVEY.md §8b's surface) called through the op registry, each
against the oracle bit for bit, each through torch.library.opcheck (schema, fake implementation, AOT
dispatch), and a codec pipeline under torch.compile (aot_eager, fullgraph) equal to eager.

Reference loops: Src/ADFL/Channel/quant.py:74-94 (per-tensor encode of a state dict) and :97-112,
Src/ADFL/compression.py:35-66 (pack_4bit / unpack_4bit), Examples/ray_ad.py:188 (peer mean)."""

import numpy as np
import pytest
import torch

import slq_oracle as oracle

pytestmark = pytest.mark.gpu

import adfl_amd  # noqa: E402,F401  registers torch.ops.adfl.*

DEV = torch.device("cuda", 0)
A = torch.ops.adfl


def _bucket(seed, sizes, gap=0, order=None):
    """Flat fp32 buffer with tensors at offsets separated by `gap` elements, in `order` (a permutation)."""
    rng = np.random.default_rng(seed)
    order = list(range(len(sizes))) if order is None else order
    offsets = [0] * len(sizes)
    pos = 0
    for t in order:
        offsets[t] = pos
        pos += sizes[t] + gap
    flat = np.zeros(pos, np.float32)
    for t, n in enumerate(sizes):
        flat[offsets[t]:offsets[t] + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -(t % 4))
    return flat, torch.tensor(offsets, dtype=torch.int64), torch.tensor(sizes, dtype=torch.int64)


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32 if a.dtype == np.float32 else np.uint8)


def test_slq_absmax_matches_torch_max_abs():
    for seed, n in [(0, 1), (1, 1027), (2, 1 << 20)]:
        x = torch.from_numpy(np.random.default_rng(seed).standard_normal(n, dtype=np.float32))
        got = A.slq_absmax(x.to(DEV))
        assert got.shape == () and got.dtype == torch.float32
        assert got.item() == torch.max(torch.abs(x)).item()
    x = torch.ones(4099, device=DEV)
    x[17] = float("nan")
    assert torch.isnan(A.slq_absmax(x)).item()


@pytest.mark.parametrize("bits", [8, 4, 2])
@pytest.mark.parametrize("gap,order", [(0, None), (5, None), (3, [2, 0, 3, 1, 4])])
def test_encode_decode_batched_match_oracle(bits, gap, order):
    sizes = [1, 4097, 8192, 70001, 33]
    flat, off, siz = _bucket(bits + gap, sizes, gap, order)
    q, s = A.slq_encode_batched(torch.from_numpy(flat).to(DEV), off, siz, bits)
    d = A.slq_decode_batched(q, s, off, siz)
    qo, so = oracle.encode_batched(flat, off.numpy(), siz.numpy(), bits)
    assert q.shape == (flat.size,) and s.shape == (len(sizes),)
    assert np.array_equal(q.cpu().numpy(), qo)                   # gaps are zero on both sides
    assert np.array_equal(_bits(s.cpu().numpy()), _bits(so))
    want = np.zeros(flat.size, np.float32)
    for t, (o, n) in enumerate(zip(off.tolist(), sizes)):
        want[o:o + n] = oracle.decode(qo[o:o + n], so[t])
    assert np.array_equal(_bits(d.cpu().numpy()), _bits(want))


@pytest.mark.parametrize("gap", [0, 6])
def test_encode_decode_batched_int4_match_oracle(gap):
    """int4 buckets need even tensor offsets: each slot is the tensor rounded up to even, plus `gap`."""
    sizes = [2, 4097, 8192, 70001, 31]
    offsets, pos = [], 0
    for n in sizes:
        offsets.append(pos)
        pos += n + n % 2 + gap
    rng = np.random.default_rng(40 + gap)
    flat = np.zeros(pos, np.float32)
    for o, n in zip(offsets, sizes):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(1e-2)
    off, siz = torch.tensor(offsets), torch.tensor(sizes)
    p, s = A.slq_encode_batched_int4(torch.from_numpy(flat).to(DEV), off, siz, 4)
    d = A.slq_decode_batched_int4(p, s, off, siz, flat.size)
    ph, sh, dh = p.cpu().numpy(), s.cpu().numpy(), d.cpu().numpy()
    assert ph.size == (flat.size + 1) // 2 and dh.size == flat.size
    for t, (o, n) in enumerate(zip(offsets, sizes)):
        qo, so = oracle.encode(flat[o:o + n], 4)
        packed = oracle.pack_int4(qo)   # an odd tensor's last byte pairs its last element with pack_4bit's pad
        assert _bits(np.float32(so)) == _bits(sh[t:t + 1])[0], t
        assert np.array_equal(ph[o // 2:o // 2 + packed.size], packed), t
        assert np.array_equal(_bits(dh[o:o + n]), _bits(oracle.decode_int4(packed, n, so))), t


def test_pack_unpack_int4_match_oracle():
    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 4096, 100003):
        q = rng.integers(-8, 8, n, dtype=np.int8)
        p = A.pack_int4(torch.from_numpy(q).to(DEV))
        assert np.array_equal(p.cpu().numpy(), oracle.pack_int4(q)), n
        u = A.unpack_int4(p, [n])
        assert np.array_equal(u.cpu().numpy(), oracle.unpack_int4(oracle.pack_int4(q), n)), n
    u = A.unpack_int4(A.pack_int4(torch.from_numpy(q[:12]).to(DEV)), [3, 4])
    assert u.shape == (3, 4)


@pytest.mark.parametrize("self_row", [-1, 0, 2])
def test_dequantize_mean_matches_oracle(self_row):
    k, n = 4, 10007
    rng = np.random.default_rng(11 + self_row)
    xs = [rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -r) for r in range(k)]
    encs = [oracle.encode(x, 8) for x in xs]
    row = (n + 15) // 16 * 16
    rows = np.zeros((k, row), np.int8)
    for r, (q, _) in enumerate(encs):
        rows[r, :n] = q
    scales = np.array([s for _, s in encs], np.float32)
    self_x = torch.from_numpy(xs[self_row]).to(DEV) if self_row >= 0 else None
    got = A.slq_dequantize_mean(torch.from_numpy(rows).to(DEV), torch.from_numpy(scales).to(DEV), n, self_row,
                                self_x).cpu().numpy()
    want = (oracle.dequantize_mean_self([r for r in rows[:, :n]], scales, n, self_row, xs[self_row])
            if self_row >= 0 else oracle.dequantize_mean([r for r in rows[:, :n]], scales))
    assert np.array_equal(_bits(got), _bits(want))


def test_dequantize_mean_batched_op_matches_oracle():
    """torch.ops.adfl.slq_dequantize_mean_batched: K bucketed payloads with per-tensor scales averaged per
    tensor (ray_ad.py:164-190 under quant.py:74-94), caller-placed tensors, own row exact."""
    sizes, offsets = [5000, 3, 9000], [9100, 0, 16]
    n = 14208   # a 16-byte multiple row
    k = 3
    rng = np.random.default_rng(77)
    rows = np.zeros((k, n), np.int8)
    scales = np.zeros((k, 3), np.float32)
    flats = []
    for r in range(k):
        f = np.zeros(n, np.float32)
        for o, m in zip(offsets, sizes):
            f[o:o + m] = rng.standard_normal(m, dtype=np.float32) * np.float32(1e-3)
        q, s = oracle.encode_batched(f, offsets, sizes, 8)
        rows[r], scales[r] = q, s
        flats.append(f)
    got = A.slq_dequantize_mean_batched(torch.from_numpy(rows).to(DEV), torch.from_numpy(scales).to(DEV),
                                        torch.tensor(offsets), torch.tensor(sizes), n, 1,
                                        torch.from_numpy(flats[1]).to(DEV)).cpu().numpy()
    want = oracle.dequantize_mean_batched(list(rows), list(scales), offsets, sizes, n, 1, flats[1])
    assert np.array_equal(_bits(got), _bits(want))
    # the int4 exchange rows (PackedSLQChannel per tensor): even offsets, packed payload
    offs4 = [9100, 0, 18]
    prow = np.zeros((k, n // 2), np.uint8)
    for r in range(k):
        q4, s4 = oracle.encode_batched(np.roll(flats[r], 2), offs4, sizes, 4)
        prow[r], scales[r] = oracle.pack_int4(q4), s4
    got4 = A.slq_dequantize_mean_batched_int4(torch.from_numpy(prow).to(DEV), torch.from_numpy(scales).to(DEV),
                                              torch.tensor(offs4), torch.tensor(sizes), n).cpu().numpy()
    want4 = oracle.dequantize_mean_batched(list(prow), list(scales), offs4, sizes, n, -1, None, packed=True)
    assert np.array_equal(_bits(got4), _bits(want4))


def _opcheck_cases():
    flat, off, siz = _bucket(5, [3, 4097, 900], 2)
    x = torch.from_numpy(flat).to(DEV)
    q, s = A.slq_encode_batched(x, off, siz, 8)
    p4, s4 = A.slq_encode_batched_int4(torch.zeros(6000, device=DEV).normal_(), torch.tensor([0, 4000]),
                                       torch.tensor([3999, 1000]), 4)
    rows = torch.randint(-128, 128, (3, 1024), dtype=torch.int8, device=DEV)
    return [
        (A.slq_absmax, (x,)),
        (A.slq_encode, (x.reshape(1, -1), 8)),
        (A.slq_decode, (q.reshape(1, -1), s[:1])),
        (A.slq_encode_int4, (x, 4)),
        (A.slq_decode_int4, (A.pack_int4(q), q.numel(), s[:1])),
        (A.slq_encode_batched, (x, off, siz, 8)),
        (A.slq_decode_batched, (q, s, off, siz)),
        (A.slq_encode_batched_int4, (torch.zeros(6000, device=DEV).normal_(), torch.tensor([0, 4000]),
                                     torch.tensor([3999, 1000]), 4)),
        (A.slq_decode_batched_int4, (p4, s4, torch.tensor([0, 4000]), torch.tensor([3999, 1000]), 6000)),
        (A.pack_int4, (q,)),
        (A.unpack_int4, (A.pack_int4(q), [q.numel()])),
        (A.slq_dequantize_mean, (rows, torch.rand(3, device=DEV), 1000, -1, None)),
        (A.slq_dequantize_mean, (rows, torch.rand(3, device=DEV), 1000, 1, torch.randn(1000, device=DEV))),
        (A.slq_dequantize_mean_batched, (rows, torch.rand(3, 2, device=DEV), torch.tensor([0, 500]),
                                         torch.tensor([300, 500]), 1024, -1, None)),
        (A.slq_dequantize_mean_batched, (rows, torch.rand(3, 2, device=DEV), torch.tensor([0, 500]),
                                         torch.tensor([300, 500]), 1000, 2, torch.randn(1000, device=DEV))),
        (A.slq_dequantize_mean_batched_int4, (rows.view(torch.uint8)[:, :512].contiguous(),
                                              torch.rand(3, 2, device=DEV), torch.tensor([0, 500]),
                                              torch.tensor([300, 500]), 1000, 1, torch.randn(1000, device=DEV))),
    ]


@pytest.mark.parametrize("case", range(16))
def test_opcheck(case):
    op, args = _opcheck_cases()[case]
    torch.library.opcheck(op, args)


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
@pytest.mark.parametrize("gap", [0, 3])
def test_stoch_ops_match_the_bucket_api(codec, gap):
    """torch.ops.adfl.stoch_encode_batched / stoch_decode_batched over caller-placed tensors equal the
    adfl_amd.stoch bucket calls on the same layout and Philox stream byte for byte (those are pinned to the
    reference's fixtures and the oracle in tests/test_gpu_stoch.py); positions no tensor owns are zero."""
    from adfl_amd import ops, stoch
    flat, off, siz = _bucket(21, [3, 4097, 900, 8192], gap)
    x = torch.from_numpy(flat).to(DEV)
    lv, sg, nr, mn = A.stoch_encode_batched(x, off, siz, codec, 8, 1234, 5)
    lay = ops.layout_for(off, siz)
    if codec == "qsgd":
        want = stoch.qsgd_encode_batched(x, lay, 8, seed=1234, counter=5)
        wdec = stoch.qsgd_decode_batched(want[0], want[1], want[2], lay, 8)
    elif codec == "rqsgd":
        want = stoch.rqsgd_encode_batched(x, lay, 8, seed=1234, counter=5)
        wdec = stoch.rqsgd_decode_batched(want[0], want[1], want[2], want[3], lay, 8)
    else:
        want = stoch.cnat_encode_batched(x, lay, 8, seed=1234, counter=5)
        wdec = stoch.cnat_decode_batched(want[0], want[1], want[2], lay)
    d = A.stoch_decode_batched(lv, sg, nr, mn, off, siz, codec, 8)
    owned = torch.zeros(x.numel(), dtype=torch.bool, device=DEV)
    for o, n in zip(off.tolist(), siz.tolist()):
        owned[o:o + n] = True
    w = owned[:lay.total]                      # the bucket calls' planes end at the layout's last element
    assert torch.equal(lv[owned].view(torch.uint8), want[0][w].view(torch.uint8))
    assert torch.equal(sg[owned], want[1][w]) and torch.equal(nr, want[2])
    assert torch.equal(d[owned].view(torch.int32), wdec[w].view(torch.int32))
    if codec == "rqsgd":
        assert torch.equal(mn, want[3])
    if gap:
        assert not lv[~owned].any() and not sg[~owned].any() and not d[~owned].any()


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float64])
def test_stoch_ops_dtype_buckets(codec, dtype):
    """fp16 / bf16 / fp64 buffers through torch.ops.adfl.stoch_encode_batched are encoded in their own dtype's
    arithmetic: planes equal adfl_amd.stoch.encode_batched_dt on the same layout and Philox stream (pinned to
    the reference's fp16 / bf16 / fp64 fixtures in tests/test_gpu_stoch_dt.py); norms / mins come back as the
    fp32 values the decode uses, and the decode op equals the fp32 decode with them."""
    from adfl_amd import ops, stoch
    flat, off, siz = _bucket(33, [3, 4097, 900, 8192], 3)
    x = torch.from_numpy(flat).to(DEV).to(dtype)
    lv, sg, nr, mn = A.stoch_encode_batched(x, off, siz, codec, 8, 4321, 2)
    lay = ops.layout_for(off, siz)
    wl, ws_, wn, wm = stoch.encode_batched_dt(codec, x, lay, 8, seed=4321, counter=2)
    owned = torch.zeros(x.numel(), dtype=torch.bool, device=DEV)
    for o, n in zip(off.tolist(), siz.tolist()):
        owned[o:o + n] = True
    w = owned[:lay.total]
    assert torch.equal(lv[owned].view(torch.uint8), wl[w].view(torch.uint8)) and torch.equal(sg[owned], ws_[w])
    assert nr.dtype == torch.float32 and torch.equal(nr, wn.float())
    assert torch.equal(mn, wm.float()) if codec == "rqsgd" else not mn.any()
    assert not lv[~owned].any() and not sg[~owned].any()
    d = A.stoch_decode_batched(lv, sg, nr, mn, off, siz, codec, 8)
    if codec == "qsgd":
        wdec = stoch.qsgd_decode_batched(wl.view(torch.uint8), ws_, wn.float(), lay, 8)
    elif codec == "rqsgd":
        wdec = stoch.rqsgd_decode_batched(wl.view(torch.uint8), ws_, wn.float(), wm.float(), lay, 8)
    else:
        wdec = stoch.cnat_decode_batched(wl.view(torch.int8), ws_, wn.float(), lay)
    assert torch.equal(d[owned].view(torch.int32), wdec[w].view(torch.int32))
    torch.library.opcheck(A.stoch_encode_batched, (x, off, siz, codec, 8, 99, 0))


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_stoch_ops_opcheck_and_compile(codec):
    flat, off, siz = _bucket(8, [3, 4097, 900], 2)
    x = torch.from_numpy(flat).to(DEV)
    torch.library.opcheck(A.stoch_encode_batched, (x, off, siz, codec, 8, 99, 0))
    lv, sg, nr, mn = A.stoch_encode_batched(x, off, siz, codec, 8, 99, 0)
    torch.library.opcheck(A.stoch_decode_batched, (lv, sg, nr, mn, off, siz, codec, 8))

    def pipeline(x):
        e = torch.ops.adfl.stoch_encode_batched(x, off, siz, codec, 8, 99, 0)
        return torch.ops.adfl.stoch_decode_batched(*e, off, siz, codec, 8)

    eager = pipeline(x)
    compiled = torch.compile(pipeline, backend="aot_eager", fullgraph=True)(x)
    assert torch.equal(eager.view(torch.int32), compiled.view(torch.int32))


def test_codec_pipeline_under_torch_compile():
    """encode -> decode -> mean of a bucketed update traced by torch.compile (fullgraph: every op goes through
    its fake implementation at trace time, the HIP kernels at run time) equals eager bit for bit."""
    flat, off, siz = _bucket(9, [4096, 80, 8192], 0)   # 12,368 elements: a 16-byte multiple row
    x = torch.from_numpy(flat).to(DEV)

    def pipeline(x):
        q, s = torch.ops.adfl.slq_encode_batched(x, off, siz, 8)
        d = torch.ops.adfl.slq_decode_batched(q, s, off, siz)
        p, sc = torch.ops.adfl.slq_encode_int4(x, 4)
        d4 = torch.ops.adfl.slq_decode_int4(p, x.numel(), sc)
        rows = torch.stack([q, q]).contiguous()
        m = torch.ops.adfl.slq_dequantize_mean(rows, torch.cat([s[:1], s[:1]]), x.numel(), -1, None)
        return d, d4, m, torch.ops.adfl.slq_absmax(x)

    eager = pipeline(x)
    compiled = torch.compile(pipeline, backend="aot_eager", fullgraph=True)(x)
    for e, c in zip(eager, compiled):
        assert torch.equal(e.view(torch.int32), c.view(torch.int32))
