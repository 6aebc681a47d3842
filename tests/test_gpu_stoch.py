"""GPU: the HIP stochastic codecs (include/adfl_stoch.h) against the reference and the oracle.

* golden: every case of tests/golden/stoch.npz (the reference executed with recorded uniforms). With the
  same uniforms and the reference's norm injected, levels / exponents, signs and decoded floats are
  bit-identical; the HIP L2 norm is within 1 ulp of the oracle's correctly rounded norm and max/min
  norms are exact; CNAT's encode (which does not need the norm) is bit-identical end to end.
* buckets: many tensors in one compact or aligned bucket (chunk heads at every offset mod 4).
* Philox: the in-kernel uniforms equal the oracle's Philox restatement bit for bit, and an encode that
  draws them equals the oracle run on those uniforms.
* statistics at sizes the oracle cannot replay: unbiasedness of QSGD / RQSGD / CNAT decode, and the
  reference test's CNAT rounding frequency (Src/ADFL/Channel/Tests/test_quant.py:117-123).
* channels: QSGD / RQSGD / CNAT channel round trips bit-identical to the oracle on the channel's own
  uniforms and norms, reference payload types.
"""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from golden_util import same_f32

import stoch_oracle as so

pytestmark = pytest.mark.gpu

from adfl_amd import ops, stoch  # noqa: E402
from adfl_amd.Channel import CNATChannel, QSGDChannel, RQSGDChannel  # noqa: E402

MANIFEST = json.load(open(os.path.join(GOLDEN, "stoch_manifest.json")))
ARR = np.load(os.path.join(GOLDEN, "stoch.npz"))
CASES = MANIFEST["cases"]
DEV = torch.device("cuda", 0)


def _scale(rec) -> np.float32:
    if "int" in rec:
        return np.float32(rec["int"])
    return np.array([rec["bits"]], np.uint32).view(np.float32)[0]


def load_case(c):
    n = c["name"]
    return (ARR[f"{n}__x"], ARR[f"{n}__u"], ARR[f"{n}__q"], ARR[f"{n}__signs"], ARR[f"{n}__deq"],
            _scale(c["scale"]), _scale(c["scale_2"]))


def d(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(DEV)


def h(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy()


def ulp_diff(a: np.float32, b: np.float32) -> int:
    ia = int(np.array([a], np.float32).view(np.int32)[0])
    ib = int(np.array([b], np.float32).view(np.int32)[0])
    return abs(ia - ib)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_golden_case(c):
    x, u, q_ref, s_ref, d_ref, norm, scale2 = load_case(c)
    bits = c["bits"]
    lay = ops.BucketLayout([x.size], align=1)
    xd, ud = d(x), d(u)
    norm_d = torch.tensor([norm], dtype=torch.float32, device=DEV)
    if c["codec"] == "cnat":
        e, s, nrm = stoch.cnat_encode_batched(xd, lay, bits, uniforms=ud)
        np.testing.assert_array_equal(h(e).view(np.uint8), q_ref.reshape(-1))
        np.testing.assert_array_equal(h(s), s_ref.reshape(-1))
        mine = h(nrm)[0]
        assert ulp_diff(mine, so.l2_norm(x)) <= 1 or (np.isnan(mine) and np.isnan(so.l2_norm(x)))
        out = stoch.cnat_decode_batched(d(q_ref.view(np.int8)), d(s_ref), norm_d, lay)
    elif c["codec"] == "qsgd":
        nrm, _ = stoch.norms_batched(xd, lay, stoch.NORM_L2)
        mine = h(nrm)[0]
        assert ulp_diff(mine, so.l2_norm(x)) <= 1 or (np.isnan(mine) and np.isnan(so.l2_norm(x)))
        lv, s = stoch.qsgd_quantize_batched(xd, lay, bits, norm_d, uniforms=ud)
        np.testing.assert_array_equal(h(lv), q_ref.reshape(-1))
        np.testing.assert_array_equal(h(s), s_ref.reshape(-1))
        out = stoch.qsgd_decode_batched(d(q_ref), d(s_ref), norm_d, lay, bits)
    else:
        lv, s, nrm, mn = stoch.rqsgd_encode_batched(xd, lay, bits, uniforms=ud)
        assert same_f32(h(nrm)[:1], np.array([norm], np.float32))
        if "tensor" not in c["scale"]:
            assert same_f32(h(mn)[:1], np.array([scale2], np.float32))
        np.testing.assert_array_equal(h(lv), q_ref.reshape(-1))
        np.testing.assert_array_equal(h(s), s_ref.reshape(-1))
        mins_d = torch.tensor([scale2], dtype=torch.float32, device=DEV)
        out = stoch.rqsgd_decode_batched(d(q_ref), d(s_ref), norm_d, mins_d, lay, bits)
    assert same_f32(h(out), d_ref.reshape(-1))


def _bucket(codec, bits, align):
    cs = [c for c in CASES if c["codec"] == codec and c["bits"] == bits]
    xs = [load_case(c) for c in cs]
    lay = ops.BucketLayout([x[0].size for x in xs], align=align)
    flat = np.zeros(lay.total, np.float32)
    uni = np.zeros(lay.total, np.float32)
    for (x, u, *_), off in zip(xs, lay.offsets):
        flat[off:off + x.size] = x.reshape(-1)
        uni[off:off + x.size] = u.reshape(-1)
    return cs, xs, lay, flat, uni


@pytest.mark.parametrize("align", [1, 64])
@pytest.mark.parametrize("codec,bits", [("qsgd", 8), ("rqsgd", 8), ("cnat", 8), ("qsgd", 4), ("cnat", 4)])
def test_golden_bucket(codec, bits, align):
    """All golden cases of one codec / bit width in one bucket: per-tensor norms, chunk heads."""
    cs, xs, lay, flat, uni = _bucket(codec, bits, align)
    xd, ud = d(flat), d(uni)
    ref_norms = torch.tensor([x[5] for x in xs], dtype=torch.float32, device=DEV)
    if codec == "cnat":
        q, s, nrm = stoch.cnat_encode_batched(xd, lay, bits, uniforms=ud)
        out = stoch.cnat_decode_batched(q, s, ref_norms, lay)
    elif codec == "qsgd":
        nrm, _ = stoch.norms_batched(xd, lay)
        q, s = stoch.qsgd_quantize_batched(xd, lay, bits, ref_norms, uniforms=ud)
        out = stoch.qsgd_decode_batched(q, s, ref_norms, lay, bits)
    else:
        q, s, nrm, mn = stoch.rqsgd_encode_batched(xd, lay, bits, uniforms=ud)
        mins = torch.tensor([x[6] for x in xs], dtype=torch.float32, device=DEV)
        out = stoch.rqsgd_decode_batched(q, s, nrm, mins, lay, bits)
    qh, sh, oh, nh = h(q).view(np.uint8), h(s), h(out), h(nrm)
    for i, (c, (x, u, q_ref, s_ref, d_ref, norm, _)) in enumerate(zip(cs, xs)):
        o, n = int(lay.offsets[i]), x.size
        np.testing.assert_array_equal(qh[o:o + n], q_ref.reshape(-1), err_msg=c["name"])
        np.testing.assert_array_equal(sh[o:o + n], s_ref.reshape(-1), err_msg=c["name"])
        assert same_f32(oh[o:o + n], d_ref.reshape(-1)), c["name"]
        if codec == "rqsgd":
            assert same_f32(nh[i:i + 1], np.array([norm], np.float32))
        else:
            ora = so.l2_norm(x)
            assert ulp_diff(nh[i], ora) <= 1 or (np.isnan(nh[i]) and np.isnan(ora)), c["name"]


def test_philox_uniforms_match_oracle():
    for seed, counter, start, n in [(0, 0, 0, 4096), (123456789123, 77, 5, 100003), (2 ** 64 - 1, 2 ** 40, 3, 999)]:
        u = h(stoch.philox_uniforms(n, seed, counter, start, device=DEV))
        np.testing.assert_array_equal(u, so.philox_uniforms(n, seed, counter, start))


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
@pytest.mark.parametrize("sizes", [[(1 << 20) + 37], [5, 17, 8192, 8193, 70001, 3]])
def test_seeded_encode_matches_oracle_on_philox_uniforms(codec, sizes):
    """The production path (uniforms drawn in-kernel) = the oracle run on the Philox uniforms, per tensor,
    given the kernel's own norms."""
    rng = np.random.default_rng(11)
    lay = ops.BucketLayout(sizes, align=1)
    flat = (rng.standard_normal(lay.total, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
    flat[3] = 0.0
    seed, counter, bits = 987654321, 1000, 8
    xd = d(flat)
    if codec == "qsgd":
        q, s, nrm = stoch.qsgd_encode_batched(xd, lay, bits, seed=seed, counter=counter)
        mins = None
    elif codec == "rqsgd":
        q, s, nrm, mins = stoch.rqsgd_encode_batched(xd, lay, bits, seed=seed, counter=counter)
    else:
        q, s, nrm = stoch.cnat_encode_batched(xd, lay, bits, seed=seed, counter=counter)
        mins = None
    u_all = so.philox_uniforms(lay.total, seed, counter)
    qh, sh, nh = h(q).view(np.uint8), h(s), h(nrm)
    for i, n in enumerate(sizes):
        o = int(lay.offsets[i])
        x, u = flat[o:o + n], u_all[o:o + n]
        if codec == "cnat":
            qo, so_ = so.cnat_quantize(x, bits, nh[i], u)
            assert ulp_diff(nh[i], so.l2_norm(x)) <= 1
        else:
            qo, so_ = so.qsgd_quantize(x, 2 ** bits - 1, nh[i], u)
        np.testing.assert_array_equal(qh[o:o + n], qo.view(np.uint8))
        np.testing.assert_array_equal(sh[o:o + n], so_)
    if mins is not None:
        mh = h(mins)
        for i, n in enumerate(sizes):
            o = int(lay.offsets[i])
            assert mh[i] == so.lminf_norm(flat[o:o + n]) and nh[i] == so.linf_norm(flat[o:o + n])


@pytest.mark.parametrize("mode", ["l2", "linf"])
def test_norm_finalize_many_chunks(mode):
    """A tensor of 16,387 chunks between two small ones: the finalize's large-tensor role sums it in two
    batches of 16 loads per thread, the second one partial (clamped index, masked slots). A duplicated or
    dropped slot moves the L2 norm by ~1/16,387 (thousands of ulps); the fp64 sum's order may move it by 1."""
    n_big = (16 * 1024 + 3) * 8192 + 77   # ADFL_SLQ_CHUNK_ELEMS = 8192
    sizes = [5, n_big, 9000]
    lay = ops.BucketLayout(sizes, align=1)
    g = torch.Generator(device=DEV).manual_seed(5)
    xd = torch.randn(lay.total, device=DEV, generator=g) * 1e-3
    assert lay.nchunks > 16 * 1024 + 3
    nrm, mins = stoch.norms_batched(xd, lay, stoch.NORM_L2 if mode == "l2" else stoch.NORM_LINF)
    flat, nh = h(xd), h(nrm)
    for i, n in enumerate(sizes):
        o = int(lay.offsets[i])
        x = flat[o:o + n]
        if mode == "l2":
            s = np.sum((x * x).astype(np.float64))     # fp32 squares, fp64 sum
            want = np.float32(np.sqrt(np.float64(np.float32(s))))
            assert ulp_diff(nh[i], want) <= 1, (i, nh[i], want)
        else:
            assert nh[i] == np.abs(x).max() and h(mins)[i] == np.abs(x).min()


def test_philox_uniform_statistics():
    n = 1 << 24
    u = stoch.philox_uniforms(n, 42, 0, device=DEV).double()
    assert abs(u.mean().item() - 0.5) < 3e-4
    assert abs(u.var().item() - 1 / 12) < 3e-4
    hist = torch.histc(u.float(), bins=256, min=0.0, max=1.0).cpu().numpy()
    chi2 = float(((hist - n / 256) ** 2 / (n / 256)).sum())
    assert chi2 < 256 + 6 * np.sqrt(2 * 256)  # 255 dof, ~6 sigma


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_unbiased_decode(codec):
    """E[decode(encode(x))] = x for QSGD / RQSGD (norm-scaled levels; RQSGD except its zero-level floor) and
    E[2^e] = |x| + eps-scale for CNAT's exponent rounding: averaged over many seeds on the device."""
    torch.manual_seed(0)
    n, reps = 4096, 4000
    x = torch.randn(n, device=DEV) * 1e-3
    lay = ops.BucketLayout([n], align=1)
    acc = torch.zeros(n, dtype=torch.float64, device=DEV)
    for r in range(reps):
        if codec == "qsgd":
            q, s, nr = stoch.qsgd_encode_batched(x, lay, 4, seed=r, counter=0)
            acc += stoch.qsgd_decode_batched(q, s, nr, lay, 4).double()
        elif codec == "rqsgd":
            q, s, nr, mn = stoch.rqsgd_encode_batched(x, lay, 4, seed=r, counter=0)
            acc += stoch.rqsgd_decode_batched(q, s, nr, mn, lay, 4).double()
        else:
            e, s, _ = stoch.cnat_encode_batched(x, lay, 8, seed=r, counter=0)
            one = torch.ones(1, device=DEV)
            acc += stoch.cnat_decode_batched(e, s, one, lay).double()  # norm 1: sign * 2^e
    mean = (acc / reps).float()
    if codec == "qsgd":
        nrm = torch.linalg.vector_norm(x).item()
        tol = 5 * nrm / 15 / np.sqrt(reps)  # per-element std <= norm / levels / 2
        assert (mean - x).abs().max().item() < tol
    elif codec == "rqsgd":
        nrm = x.abs().max().item()
        big = x.abs() * 15 >= nrm  # level >= 1 with certainty: no min-factor substitution
        tol = 5 * nrm / 15 / np.sqrt(reps)
        assert (mean - x)[big].abs().max().item() < tol
    else:
        # CNAT rounds v = |x| + eps between 2^f and 2^c with P(f) = (2^c - |x|) / 2^f: E = |x| + ... exact
        # for |x| in [2^f, 2^c]; check the relative bias is within sampling error
        rel = ((mean.abs() - x.abs()) / x.abs())[x.abs() > 1e-5]
        assert rel.abs().mean().item() < 0.02


def test_cnat_reference_frequency_check():
    """Src/ADFL/Channel/Tests/test_quant.py:117-123: 0.6 rounds to exponent -1 with probability 0.8 and
    to 0 with probability 0.2 (10000 draws in the reference; 2^22 here)."""
    n = 1 << 22
    lay = ops.BucketLayout([n], align=1)
    x = torch.full((n,), 0.6, device=DEV)
    e, s, _ = stoch.cnat_encode_batched(x, lay, 8, seed=1234, counter=0)
    e = e.cpu()
    zero = (e == 0).double().mean().item()
    assert set(torch.unique(e).tolist()) == {-1, 0}
    assert abs(zero - 0.2) < 0.002


@pytest.mark.parametrize("cls", [QSGDChannel, RQSGDChannel, CNATChannel], ids=lambda c: c.__name__)
def test_channel_round_trip_matches_oracle(cls):
    """Channel encode with injected uniforms: payload types as the reference; bytes = oracle on the same
    uniforms and the channel's norms; decode = oracle decode of that payload."""
    torch.manual_seed(5)
    shapes = [(64, 3, 3, 3), (64,), (128, 64), (10, 512), (10,), (7, 1)]
    params = {f"p{i}": torch.randn(*s) * 1e-2 for i, s in enumerate(shapes)}
    params["zero"] = torch.zeros(4, 4)
    params["num_batches_tracked"] = torch.tensor(12)
    ch = cls(8)
    names = [k for k, v in params.items() if v.ndim > 1]
    total = sum(params[k].numel() for k in names)
    u = torch.rand(total, generator=torch.Generator().manual_seed(9))
    qp = ch._quantize_params(params, 8, uniforms=u.to(DEV))
    off = 0
    for k, v in params.items():
        p = qp.params[k]
        if v.ndim <= 1:
            assert p.data is v and p.scale == 0 and p.signs.dtype == torch.uint8
            continue
        n = v.numel()
        x, uu = v.numpy(), u[off:off + n].numpy().reshape(v.shape)
        off += n
        if k == "zero":
            assert p.data.dtype == torch.uint8 and isinstance(p.scale, torch.Tensor) and p.scale.item() == 0
            assert (p.data == 0).all() and (p.signs == 1).all()
            continue
        if cls is CNATChannel:
            qo, sg = so.cnat_quantize(x, 8, p.scale, uu)
            assert p.data.dtype == torch.int8
        else:
            qo, sg = so.qsgd_quantize(x, 255, p.scale, uu)
            assert p.data.dtype == torch.uint8
        if cls is RQSGDChannel:
            assert p.scale == float(so.linf_norm(x)) and p.scale_2 == float(so.lminf_norm(x))
        else:
            assert ulp_diff(np.float32(p.scale), so.l2_norm(x)) <= 1
        assert isinstance(p.scale, float) and p.shape == v.shape and p.q_dtype == p.data.dtype
        np.testing.assert_array_equal(p.data.numpy(), qo)
        np.testing.assert_array_equal(p.signs.numpy(), sg)
        assert p.data.untyped_storage().nbytes() == n  # owned bytes
    assert qp.size == sum(p.data.nbytes for p in qp.params.values())
    dec, _ = ch.on_server_receive(qp)
    for k, v in params.items():
        p = qp.params[k]
        if v.ndim <= 1:
            assert dec[k].data_ptr() == v.data_ptr()
            continue
        if cls is CNATChannel:
            want = so.cnat_dequantize(p.data.numpy(), p.signs.numpy(), float(p.scale))
        elif cls is QSGDChannel:
            want = so.qsgd_dequantize(p.data.numpy(), p.signs.numpy(), 255, float(p.scale))
        else:
            want = so.rqsgd_dequantize(p.data.numpy(), p.signs.numpy(), 255, float(p.scale), float(p.scale_2))
        assert dec[k].dtype == torch.float32 and dec[k].shape == v.shape
        assert same_f32(dec[k].numpy(), want)


@pytest.mark.parametrize("cls", [QSGDChannel, RQSGDChannel, CNATChannel], ids=lambda c: c.__name__)
def test_channel_seeded_by_torch_generator(cls):
    x = {"w": torch.randn(64, 65)}
    torch.manual_seed(1)
    a, _ = cls(8).on_client_send(x)
    torch.manual_seed(1)
    b, _ = cls(8).on_client_send(x)
    c, _ = cls(8).on_client_send(x)
    assert torch.equal(a.params["w"].data, b.params["w"].data)
    assert not torch.equal(b.params["w"].data, c.params["w"].data)


def test_decode_accepts_reference_built_payloads():
    """Payloads laid out exactly as the reference builds them (from the golden set) decode bit-exactly
    through the channel's _receive."""
    from adfl_amd.model import QuantParameter, QuantParameters
    for codec, cls in [("qsgd", QSGDChannel), ("rqsgd", RQSGDChannel), ("cnat", CNATChannel)]:
        cs = [c for c in CASES if c["codec"] == codec and c["bits"] == 8][:12]
        qp = QuantParameters({}, 0)
        want = {}
        for c in cs:
            x, u, q_ref, s_ref, d_ref, norm, scale2 = load_case(c)
            data = torch.from_numpy(q_ref.copy())
            if c["q_dtype"] == "int8":
                data = data.view(torch.int8)
            scale = torch.tensor(float(norm)) if "tensor" in c["scale"] else float(norm)
            qp.params[c["name"]] = QuantParameter(data=data, bits=8, scale=scale, signs=torch.from_numpy(s_ref.copy()),
                                                  shape=data.shape, dtype=torch.float32, q_dtype=data.dtype,
                                                  scale_2=float(scale2) if "int" not in c["scale_2"] else 0)
            want[c["name"]] = d_ref
        dec, _ = cls(8).on_server_receive(qp)
        for k, v in want.items():
            assert same_f32(dec[k].numpy(), v), k


L2_CASES = [c for c in CASES if c["codec"] != "rqsgd"]


@pytest.mark.parametrize("c", L2_CASES, ids=[c["name"] for c in L2_CASES])
def test_golden_torch_order_norm_end_to_end(c):
    """torch_norm=True: the norm in torch's own reduction order (ADFL_NORM_L2_TORCH) is the reference's
    norm bit for bit, so with the recorded uniforms the WHOLE encode — levels / exponents, signs and the
    scale — equals the reference's output with nothing injected but the uniforms."""
    x, u, q_ref, s_ref, d_ref, norm, _ = load_case(c)
    lay = ops.BucketLayout([x.size], align=1)
    xd, ud = d(x), d(u)
    nrm, _ = stoch.norms_batched(xd, lay, stoch.NORM_L2_TORCH)
    assert same_f32(h(nrm)[:1], np.array([norm], np.float32)), c["name"]
    if c["codec"] == "qsgd":
        lv, s, nrm = stoch.qsgd_encode_batched(xd, lay, c["bits"], uniforms=ud, torch_norm=True)
    else:
        lv, s, nrm = stoch.cnat_encode_batched(xd, lay, c["bits"], uniforms=ud, torch_norm=True)
    np.testing.assert_array_equal(h(lv).view(np.uint8), q_ref.reshape(-1).view(np.uint8))
    np.testing.assert_array_equal(h(s), s_ref.reshape(-1))
    assert same_f32(h(nrm)[:1], np.array([norm], np.float32))


@pytest.mark.parametrize("align", [1, 64])
def test_torch_order_norm_bucket_and_sizes(align):
    """Per-tensor torch-order norms over a bucket: every golden L2 case plus sizes around the 8-lane and
    64-element group edges and a multi-chunk tensor, against the oracle's restatement."""
    xs = [load_case(c)[0].reshape(-1) for c in L2_CASES]
    rng = np.random.default_rng(77)
    for n in (1, 7, 8, 9, 63, 64, 65, 71, 72, 511, 513, 8192 * 3 + 13, 100003):
        xs.append(rng.standard_normal(n, dtype=np.float32) * np.float32(0.37))
    lay = ops.BucketLayout([x.size for x in xs], align=align)
    flat = np.zeros(lay.total, np.float32)
    for x, o in zip(xs, lay.offsets):
        flat[o:o + x.size] = x
    nrm, _ = stoch.norms_batched(d(flat), lay, stoch.NORM_L2_TORCH)
    got = h(nrm)
    for i, x in enumerate(xs):
        assert same_f32(got[i:i + 1], np.array([so.torch_l2_norm(x)], np.float32)), (i, x.size)


@pytest.mark.parametrize("c", L2_CASES, ids=[c["name"] for c in L2_CASES])
def test_default_channel_equals_reference_end_to_end(c):
    """QSGDChannel(bits) / CNATChannel(bits), built with exactly the reference's constructor, on the golden
    tensor with only the reference's uniforms injected: levels / exponents, signs, the scale (the reference's
    own norm, quant.py:226,512, as its Python float — or the 0-dim tensor of the norm == 0 branch) and the
    decoded floats are the reference's, bit for bit."""
    x, u, q_ref, s_ref, d_ref, norm, _ = load_case(c)
    cls = QSGDChannel if c["codec"] == "qsgd" else CNATChannel
    ch = cls(c["bits"])
    assert vars(ch) == {"bits": c["bits"], "levels": 2 ** c["bits"] - 1}  # the reference's attributes only
    qp = ch._quantize_params({"w": torch.from_numpy(x.copy())}, c["bits"], uniforms=d(u))
    p = qp.params["w"]
    np.testing.assert_array_equal(p.data.numpy().reshape(-1).view(np.uint8), q_ref.reshape(-1).view(np.uint8))
    np.testing.assert_array_equal(p.signs.numpy().reshape(-1), s_ref.reshape(-1))
    assert str(p.data.dtype).replace("torch.", "") == c["q_dtype"]
    if "tensor" in c["scale"]:
        assert isinstance(p.scale, torch.Tensor) and float(p.scale) == float(norm)
    else:
        assert isinstance(p.scale, float)
        assert same_f32(np.array([p.scale], np.float32), np.array([norm], np.float32)), (p.scale, norm)
        assert p.scale == float(norm) or (np.isnan(p.scale) and np.isnan(norm))
    dec, _ = ch.on_server_receive(qp)
    assert same_f32(dec["w"].numpy().reshape(-1), d_ref.reshape(-1))


@pytest.mark.parametrize("cls", [QSGDChannel, CNATChannel])
def test_fp64_norm_switch(cls, monkeypatch):
    """ADFL_STOCH_NORM=fp64 selects the correctly rounded norm (fp64 accumulation), which differs from the
    reference's on a long tensor; unset, the scale is torch.linalg.vector_norm's bits."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2048, 1024, generator=g) * 1e-3
    ref = torch.linalg.vector_norm(x).item()
    qp, _ = cls(8).on_client_send({"w": x})
    assert qp.params["w"].scale == ref
    monkeypatch.setenv("ADFL_STOCH_NORM", "fp64")
    qp64, _ = cls(8).on_client_send({"w": x})
    assert qp64.params["w"].scale == float(np.float32(so.l2_norm(x.numpy())))
    monkeypatch.setenv("ADFL_STOCH_NORM", "bogus")
    with pytest.raises(ValueError, match="ADFL_STOCH_NORM"):
        cls(8).on_client_send({"w": x})


@pytest.mark.parametrize("align", [1, 64])
def test_cnat_multilaunch_zero_tensor_fixup(align):
    """An all-zero tensor of several chunks beside non-zero ones, through the multi-launch CNAT encode (a
    tensor above one block's 8 chunks forces it): the reference's norm == 0 branch (quant.py:513-514) gives
    u8 zeros and int8 ones for exactly that tensor's bytes; the neighbours keep their exponents."""
    sizes = [3 * 8192 + 77, 70001, 5]
    lay = ops.BucketLayout(sizes, align=align)
    assert lay.nwork == 0                                  # multi-launch: k_cnat_quantize + finalize + fixup
    rng = np.random.default_rng(9)
    flat = np.zeros(lay.total, np.float32)
    flat[lay.offsets[1]:lay.offsets[1] + sizes[1]] = rng.standard_normal(sizes[1], dtype=np.float32)
    flat[lay.offsets[2]:lay.offsets[2] + sizes[2]] = 1.5
    u = rng.random(lay.total, dtype=np.float32)
    e, s, nrm = stoch.cnat_encode_batched(d(flat), lay, 8, uniforms=d(u))
    eh, sh, nh = h(e).view(np.uint8), h(s), h(nrm)
    o0 = int(lay.offsets[0])
    assert nh[0] == 0.0 and nh[1] > 0 and nh[2] > 0
    assert (eh[o0:o0 + sizes[0]] == 0).all() and (sh[o0:o0 + sizes[0]] == 1).all()
    for t in (1, 2):
        o, n = int(lay.offsets[t]), sizes[t]
        ce, cs = so.cnat_quantize(flat[o:o + n], 8, np.float32(nh[t]), u[o:o + n])
        np.testing.assert_array_equal(eh[o:o + n], ce.view(np.uint8))
        np.testing.assert_array_equal(sh[o:o + n], cs)
