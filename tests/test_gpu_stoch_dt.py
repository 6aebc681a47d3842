"""GPU: the stochastic codecs on fp16 / bf16 / fp64 tensors (csrc/stoch_dtype.hip), computed in the tensor's
own dtype as the reference computes them (Src/ADFL/Channel/quant.py:223-240, :364-382, :509-534).

* every golden case of tests/golden/stoch_dt.npz (the reference executed on fp16 / bf16 / fp64 tensors with
  recorded uniforms): with the reference's norm injected, every level / exponent byte and sign is
  bit-identical, and the decoded floats are;
* the kernels' own norms against the oracle's (fp16 / bf16 exactly; fp64 within a few ulps), and the bytes
  against the oracle run on the kernels' norm, in compact buckets with odd offsets;
* the Philox stream on each dtype's grid equals oracle.philox_uniforms_dt bit for bit;
* the channels end to end (QSGD / RQSGD / CNAT, mixed-dtype state dicts): fp16 / bf16 / fp64 entries are
  encoded in their dtype, payload metadata as the reference's, decoded fp32."""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from golden_util import same_f32

import stoch_dt_oracle as do

pytestmark = pytest.mark.gpu

adfl_amd = pytest.importorskip("adfl_amd")
from adfl_amd import ops, stoch  # noqa: E402
from adfl_amd.Channel import CNATChannel, QSGDChannel, RQSGDChannel  # noqa: E402
from adfl_amd.Channel import stoch as stoch_channel  # noqa: E402

DEV = torch.device("cuda", 0)
MANIFEST = json.load(open(os.path.join(GOLDEN, "stoch_dt_manifest.json")))
ARR = np.load(os.path.join(GOLDEN, "stoch_dt.npz"))
CASES = MANIFEST["cases"]
DT = {"float16": do.DT_F16, "bfloat16": do.DT_BF16, "float64": do.DT_F64}
TDT = {"float16": torch.float16, "bfloat16": torch.bfloat16, "float64": torch.float64}
CHANNELS = {"qsgd": QSGDChannel, "rqsgd": RQSGDChannel, "cnat": CNATChannel}


def scale_value(rec) -> float:
    if "int" in rec:
        return float(rec["int"])
    if rec.get("tensor"):
        return float(rec["value"])
    return float(np.array([rec["f64_bits"]], np.uint64).view(np.float64)[0])


def to_torch(raw: np.ndarray, dtname: str) -> torch.Tensor:
    if dtname == "float64":
        return torch.from_numpy(np.ascontiguousarray(raw).reshape(-1).copy())
    return torch.from_numpy(np.ascontiguousarray(raw).reshape(-1).view(np.int16).copy()).view(TDT[dtname])


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_kernels_match_reference_given_its_norm(c):
    n = c["name"]
    x, u = ARR[f"{n}__x"], ARR[f"{n}__u"]
    q_ref, s_ref, d_ref = ARR[f"{n}__q"], ARR[f"{n}__signs"], ARR[f"{n}__deq"]
    norm, scale2 = scale_value(c["scale"]), scale_value(c["scale_2"])
    lay = ops.BucketLayout([x.size], align=1)
    xt = to_torch(x, c["dtype"]).to(DEV)
    ut = to_torch(u, c["dtype"]).to(DEV)
    q, s = stoch.quantize_batched_dt(c["codec"], xt, lay, c["bits"], torch.tensor([norm], dtype=torch.float64,
                                                                                 device=DEV), uniforms=ut)
    np.testing.assert_array_equal(q.cpu().numpy().view(np.uint8), q_ref.reshape(-1))
    np.testing.assert_array_equal(s.cpu().numpy(), s_ref.reshape(-1))
    # the fp32 decoders with scale = fp32(norm) give the reference's decoded floats
    nr = torch.tensor([norm], dtype=torch.float64).float().to(DEV)
    ql, sl = torch.from_numpy(q_ref.reshape(-1).copy()).to(DEV), torch.from_numpy(s_ref.reshape(-1).copy()).to(DEV)
    if c["codec"] == "qsgd":
        d = stoch.qsgd_decode_batched(ql, sl, nr, lay, c["bits"])
    elif c["codec"] == "rqsgd":
        d = stoch.rqsgd_decode_batched(ql, sl, nr, torch.tensor([scale2], dtype=torch.float64).float().to(DEV),
                                       lay, c["bits"])
    else:
        d = stoch.cnat_decode_batched(ql.view(torch.int8), sl, nr, lay)
    assert same_f32(d.cpu().numpy(), d_ref.reshape(-1))


L2_CASES = [c for c in CASES if c["codec"] != "rqsgd"]


@pytest.mark.parametrize("c", L2_CASES, ids=[c["name"] for c in L2_CASES])
def test_default_channel_equals_reference_end_to_end(c):
    """QSGDChannel(bits) / CNATChannel(bits) with the reference's constructor on the golden fp16 / bf16 / fp64
    tensor, only the uniforms injected: the norm is the reference's own in the dtype (torch's CPU order,
    csrc/torch_norm.hip), so the bytes, signs, scale and decoded floats are the reference's bit for bit."""
    n = c["name"]
    x, u = ARR[f"{n}__x"], ARR[f"{n}__u"]
    q_ref, s_ref, d_ref = ARR[f"{n}__q"], ARR[f"{n}__signs"], ARR[f"{n}__deq"]
    norm = scale_value(c["scale"])
    xt = to_torch(x, c["dtype"]).view(tuple(c["shape"]))
    ch = CHANNELS[c["codec"]](c["bits"])
    qp = ch._quantize_params({"w": xt}, c["bits"], uniforms=to_torch(u, c["dtype"]).to(DEV))
    p = qp.params["w"]
    np.testing.assert_array_equal(p.data.numpy().reshape(-1).view(np.uint8), q_ref.reshape(-1).view(np.uint8))
    np.testing.assert_array_equal(p.signs.numpy().reshape(-1), s_ref.reshape(-1))
    if c["scale"].get("tensor"):
        assert isinstance(p.scale, torch.Tensor) and float(p.scale) == norm
    else:
        assert isinstance(p.scale, float) and (p.scale == norm or (np.isnan(p.scale) and np.isnan(norm))), \
            (p.scale, norm)
    dec, _ = ch.on_server_receive(qp)
    assert same_f32(dec["w"].numpy().reshape(-1), d_ref.reshape(-1))


def _bucket(dtname, sizes, seed, scale):
    rng = np.random.default_rng(seed)
    lay = ops.BucketLayout(sizes, align=1)   # compact: odd offsets
    flat = np.zeros(lay.total, np.float64)
    for t, (o, m) in enumerate(zip(lay.offsets.tolist(), sizes)):
        flat[o:o + m] = rng.standard_normal(m) * scale * 10.0 ** -(t % 3)
    if sizes[1] >= 4:   # one all-zero tensor (the norm == 0 branch)
        o = int(lay.offsets[1])
        flat[o:o + sizes[1]] = 0
    xt = torch.from_numpy(flat).to(TDT[dtname])
    raw = xt.numpy() if dtname == "float64" else xt.view(torch.int16).numpy().view(np.uint16)
    return lay, xt, raw


@pytest.mark.parametrize("dtname", list(DT))
@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
@pytest.mark.parametrize("bits", [8, 4])
def test_bucket_encode_matches_oracle(dtname, codec, bits):
    """A compact bucket (odd offsets, an all-zero tensor) through adfl_stoch_encode_batched_dt, uniforms
    from the Philox stream: every byte equals the oracle run on the kernel's norms with the same stream;
    the norms equal the oracle's (fp64 within a few ulps)."""
    dt = DT[dtname]
    sizes = [7, 64, 8193, 333, 1, 20000]
    lay, xt, raw = _bucket(dtname, sizes, 11 + bits, 1e-2)
    seed, counter = 987654321, 3
    q, s, norms, mins = stoch.encode_batched_dt(codec, xt.to(DEV), lay, bits, seed=seed, counter=counter)
    q, s, norms = q.cpu().numpy().view(np.uint8), s.cpu().numpy(), norms.cpu().numpy()
    u_all = do.philox_uniforms_dt(dt, lay.total, seed, counter)
    for t, (o, m) in enumerate(zip(lay.offsets.tolist(), sizes)):
        xr = raw[o:o + m]
        if codec == "rqsgd":
            want_n, want_m = do.linf_norm(xr, dt), do.lminf_norm(xr, dt)
            assert norms[t] == want_n and mins.cpu().numpy()[t] == want_m
        else:
            want_n = do.l2_norm(xr, dt)
            if dt == do.DT_F64:
                assert abs(norms[t] - want_n) <= 8 * 2.0 ** -52 * want_n, t
            else:
                assert norms[t] == want_n, t
        qo, so_ = do.quantize(codec, xr, dt, bits, float(norms[t]), u_all[o:o + m])
        np.testing.assert_array_equal(q[o:o + m], qo.view(np.uint8), err_msg=f"tensor {t}")
        np.testing.assert_array_equal(s[o:o + m], so_, err_msg=f"tensor {t}")


@pytest.mark.parametrize("dtname", list(DT))
def test_philox_stream_matches_oracle(dtname):
    dt = DT[dtname]
    got = stoch.philox_uniforms_dt(TDT[dtname], 5000, 1234567, 9, start=13, device=DEV).cpu()
    got = got.numpy() if dtname == "float64" else got.view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(got, do.philox_uniforms_dt(dt, 5000, 1234567, 9, start=13))


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_channel_mixed_dtype_dict(codec):
    """A state dict with fp32, fp16, bf16 and fp64 weights and a bias: every weight is encoded in its own
    dtype (payload scale = the dtype's norm as a Python float, dtype field = the input's), biases pass
    through, decode gives fp32; each non-fp32 entry's bytes equal the oracle on the channel's own norm with
    the channel's Philox stream (seed fixed)."""
    torch.manual_seed(5)
    params = {"w32": torch.randn(30, 17) * 1e-2, "w16": (torch.randn(33, 31) * 1e-2).half(),
              "wbf": (torch.randn(12, 40) * 1e-2).bfloat16(), "w64": torch.randn(5, 77, dtype=torch.float64) * 1e-2,
              "z16": torch.zeros(3, 3, dtype=torch.float16), "b": torch.randn(10)}
    ch = CHANNELS[codec](8)
    seed = 4242
    qp = ch._quantize_params(params, 8, seed=seed)
    dec, _ = ch.on_server_receive(qp)
    for name, x in params.items():
        p = qp.params[name]
        if x.ndim <= 1:
            assert p.data is x
            continue
        assert p.dtype == x.dtype and p.shape == x.shape and dec[name].dtype == torch.float32
        assert p.data.dtype == (torch.int8 if codec == "cnat" and name != "z16" else torch.uint8)
        if name == "z16":   # norm == 0: the reference's branch, scale the 0-dim tensor of the dtype
            assert isinstance(p.scale, torch.Tensor) and p.scale.dtype == torch.float16 and p.scale.item() == 0
            assert (p.data == 0).all() and (p.signs == 1).all() and (dec[name] == 0).all()
            continue
        assert isinstance(p.scale, float)
        if codec != "rqsgd":   # the reference's own norm (quant.py:226,512), in the tensor's dtype
            assert p.scale == torch.linalg.vector_norm(x).item(), name
        if x.dtype == torch.float32:
            continue
        dt = {torch.float16: do.DT_F16, torch.bfloat16: do.DT_BF16, torch.float64: do.DT_F64}[x.dtype]
        raw = x.numpy() if dt == do.DT_F64 else x.view(torch.int16).numpy().view(np.uint16)
        # the dtype bucket holds this dtype's tensors back to back (z16 after w16 for fp16), drawing from its own
        # part of the stream (Channel.stoch.COUNTER_BASE: disjoint from the fp32 bucket's and the others')
        group = [n for n in params if params[n].ndim > 1 and params[n].dtype == x.dtype]
        off = sum(params[n].numel() for n in group[:group.index(name)])
        u = do.philox_uniforms_dt(dt, x.numel(), seed, stoch_channel.COUNTER_BASE[x.dtype], start=off)
        norm = p.scale
        qo, so_ = do.quantize(codec, raw.reshape(-1), dt, 8, norm, u)
        np.testing.assert_array_equal(p.data.numpy().reshape(-1).view(np.uint8), qo.view(np.uint8), err_msg=name)
        np.testing.assert_array_equal(p.signs.numpy().reshape(-1), so_, err_msg=name)
        want = do.decode(codec, qo, so_, 8, norm, p.scale_2 if codec == "rqsgd" else 0.0)
        assert same_f32(dec[name].numpy().reshape(-1), want.reshape(-1)), name


@pytest.mark.parametrize("dtname,n", [("float16", (1 << 24) + 3 * 8192 + 11), ("bfloat16", (1 << 23) + 5),
                                       ("float64", (1 << 22) + 3)])
def test_large_tensor_multichunk_norm_and_bytes(dtname, n):
    """One large tensor (thousands of chunks: the per-tensor norm is reduced by a block over its chunk
    partials; fp16's 2,052 chunks take the finalize's per-thread loop twice, the second batch partial): the
    norm equals the oracle's (fp64 within a few ulps), RQSGD's max / min exactly, and every byte equals the
    oracle on the kernel's norm with the same Philox stream."""
    dt = DT[dtname]
    g = torch.Generator().manual_seed(n)
    xt = (torch.randn(n, generator=g, dtype=torch.float64) * 1e-2).to(TDT[dtname])
    raw = xt.numpy() if dtname == "float64" else xt.view(torch.int16).numpy().view(np.uint16)
    lay = ops.BucketLayout([n], align=1)
    for codec in ("qsgd", "rqsgd", "cnat"):
        q, s, norms, mins = stoch.encode_batched_dt(codec, xt.to(DEV), lay, 8, seed=77, counter=0)
        norm = float(norms.cpu()[0])
        want = do.linf_norm(raw, dt) if codec == "rqsgd" else do.l2_norm(raw, dt)
        if codec == "rqsgd":
            assert norm == want and float(mins.cpu()[0]) == do.lminf_norm(raw, dt)
        elif dt == do.DT_F64:
            assert abs(norm - want) <= 64 * 2.0 ** -52 * want
        else:
            assert norm == want
        qo, so_ = do.quantize(codec, raw, dt, 8, norm, do.philox_uniforms_dt(dt, n, 77, 0))
        assert np.array_equal(q.cpu().numpy().view(np.uint8), qo.view(np.uint8)), codec
        assert np.array_equal(s.cpu().numpy(), so_), codec


@pytest.mark.parametrize("codec", ["qsgd", "cnat"])
def test_dtype_buckets_draw_disjoint_uniforms_and_injection_covers_one_dtype(codec):
    """One seed for a mixed dict: the fp32 bucket draws from counter 0 and each other dtype from its own base
    (identical (seed, counter) made rounding decisions correlated across dtypes); injected uniforms
    for a dict with more than their own dtype are refused instead of silently replaced."""
    params = {"w32": torch.randn(64, 64) * 1e-2, "w16": (torch.randn(64, 64) * 1e-2).half()}
    ch = CHANNELS[codec](8)
    bases = set(stoch_channel.COUNTER_BASE.values())
    assert len(bases) == 4 and stoch_channel.COUNTER_BASE[torch.float32] == 0
    u32 = stoch.philox_uniforms(4096, 77, 0, device=DEV)
    u16 = stoch.philox_uniforms_dt(torch.float16, 4096, 77, stoch_channel.COUNTER_BASE[torch.float16], device=DEV)
    assert not torch.equal(u32.double(), u16.double())
    with pytest.raises(ValueError, match="cover one dtype"):
        ch._quantize_params(params, 8, uniforms=torch.rand(4096, device=DEV))
