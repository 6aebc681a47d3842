"""The one-launch register-resident stochastic encodes (k_stoch_encode_resident, adfl_*_encode_batched_work)
against the multi-launch path and the oracle.

The resident path runs whenever every tensor of a bucket has at most ADFL_SLQ_RESIDENT_CHUNKS chunks
(65,536 elements; C3's ResNet-18 layout). It must produce the multi-launch path's bytes exactly: levels /
exponents, signs, norms (its L2 partials are formed in the same order) and RQSGD's mins, for seeded Philox
and injected uniforms, across chunk heads, one-block limits, norm == 0 (zeros and fp32-square underflow),
NaN and inf tensors. Reference: Src/ADFL/Channel/quant.py:223-252 (QSGD), :364-398 (RQSGD), :509-545 (CNAT).
"""

import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import stoch_oracle as so  # noqa: E402  (checker only)

from adfl_amd import ops, stoch  # noqa: E402

DEV = torch.device("cuda", 0)
MAXR = 8 * 8192  # ADFL_SLQ_RESIDENT_CHUNKS * ADFL_SLQ_CHUNK_ELEMS


def _sizes(seed):
    rng = np.random.default_rng(seed)
    fixed = [1, 2, 3, 4, 5, 7, 8191, 8192, 8193, 16385, MAXR - 1, MAXR, 45662, 45663]
    return fixed + [int(v) for v in rng.integers(1, MAXR + 1, 20)]


def _flat(lay, seed, specials=True):
    rng = np.random.default_rng(seed)
    flat = (rng.standard_normal(lay.total, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
    if specials:
        o, n = lay.offsets, lay.sizes
        flat[o[5]:o[5] + n[5]] = 0.0                         # all zero: norm 0
        flat[o[6]:o[6] + n[6]] *= np.float32(1e-32)          # squares underflow: L2 norm 0, max|x| > 0
        flat[o[7] + 100] = np.nan                            # NaN tensor
        flat[o[8] + 5] = np.inf                              # inf tensor
        flat[o[9]:o[9] + n[9]] *= np.float32(1e25)           # squares overflow: L2 norm inf
        flat[o[10]:o[10] + 50] = 0.0
    return flat


def _enc(codec, xd, lay, bits, resident, **kw):
    if codec == "qsgd":
        q, s, n = stoch.qsgd_encode_batched(xd, lay, bits, resident=resident, **kw)
        return q.view(torch.uint8), s, n, None
    if codec == "rqsgd":
        q, s, n, m = stoch.rqsgd_encode_batched(xd, lay, bits, resident=resident, **kw)
        return q, s, n, m
    q, s, n = stoch.cnat_encode_batched(xd, lay, bits, resident=resident, **kw)
    return q.view(torch.uint8), s, n, None


def _same(a, b, lay=None):
    """Bit equality; for element planes (lay given) only over the tensors' elements, not the pads."""
    if a is None:
        return b is None
    if lay is not None:
        idx = torch.from_numpy(np.concatenate([np.arange(o, o + n) for o, n in zip(lay.offsets, lay.sizes)]))
        a, b = a[idx.to(a.device)], b[idx.to(b.device)]
    return torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a,
                       b.view(torch.int32) if b.dtype == torch.float32 else b)


@pytest.mark.parametrize("align", [1, 64])
@pytest.mark.parametrize("bits", [8, 4, 2])
@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_resident_equals_multi_launch(codec, bits, align):
    lay = ops.BucketLayout(_sizes(bits + align), align=align)
    assert lay.nwork == lay.ntensors  # every tensor fits a block: the resident path runs
    xd = torch.from_numpy(_flat(lay, 3 * bits + align)).to(DEV)
    for kw in ({"seed": 12345 + bits, "counter": 77}, {"uniforms": torch.rand(lay.total, device=DEV)}):
        a = _enc(codec, xd, lay, bits, None, **kw)
        b = _enc(codec, xd, lay, bits, False, **kw)
        torch.cuda.synchronize()
        for name, p, r in zip(("planes", "signs", "norms", "mins"), a, b):
            assert _same(p, r, lay if name in ("planes", "signs") else None), (codec, bits, align, name, list(kw))


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_resident_matches_oracle_on_philox_uniforms(codec):
    """Seeded resident encode = the oracle run on the kernel's Philox uniforms, per tensor, with the norm the
    oracle restates (L2 within 1 ulp of the correctly rounded norm; max / min exact)."""
    sizes = [5, 17, 8192, 8193, 65536, 3, 40000]
    lay = ops.BucketLayout(sizes, align=1)
    assert lay.nwork == len(sizes)
    rng = np.random.default_rng(5)
    flat = (rng.standard_normal(lay.total, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
    flat[3] = 0.0
    seed, counter, bits = 424242, 9, 8
    q, s, nrm, mins = _enc(codec, torch.from_numpy(flat).to(DEV), lay, bits, None, seed=seed, counter=counter)
    u_all = so.philox_uniforms(lay.total, seed, counter)
    qh, sh, nh = q.cpu().numpy(), s.cpu().numpy(), nrm.cpu().numpy()
    for i, n in enumerate(sizes):
        o = int(lay.offsets[i])
        x, u = flat[o:o + n], u_all[o:o + n]
        if codec == "cnat":
            qo, so_ = so.cnat_quantize(x, bits, nh[i], u)
        else:
            qo, so_ = so.qsgd_quantize(x, 2 ** bits - 1, nh[i], u)
        if codec == "rqsgd":
            assert nh[i] == so.linf_norm(x) and mins.cpu().numpy()[i] == so.lminf_norm(x)
        else:
            ref = np.float32(so.l2_norm(x))
            assert abs(int(nh[i:i + 1].view(np.int32)[0]) - int(np.array([ref]).view(np.int32)[0])) <= 1
        np.testing.assert_array_equal(qh[o:o + n], qo.view(np.uint8))
        np.testing.assert_array_equal(sh[o:o + n], so_)


def test_layout_with_a_large_tensor_runs_multi_launch():
    lay = ops.BucketLayout([100, MAXR + 1, 7], align=1)
    assert lay.nwork == 0
    xd = torch.randn(lay.total, device=DEV)
    a = _enc("qsgd", xd, lay, 8, None, seed=1, counter=0)
    b = _enc("qsgd", xd, lay, 8, False, seed=1, counter=0)
    torch.cuda.synchronize()
    assert all(_same(p, r) for p, r in zip(a, b))


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_full_size_sign_symmetry(codec):
    """Size-independent property at the bench size (2^28 elements, C2, multi-launch path): with the same
    Philox stream, encode(-x) has the same levels / exponents and norms as encode(x) and negated signs
    (quant.py:230-236 uses |x|; torch.sign flips)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(1 << 28, device=DEV, generator=g) * 1e-3
    lay = ops.BucketLayout([x.numel()], align=1)
    a = _enc(codec, x, lay, 8, None, seed=5, counter=0)
    b = _enc(codec, -x, lay, 8, None, seed=5, counter=0)
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2])
    assert torch.equal(a[1], -b[1])
    if codec == "rqsgd":
        assert torch.equal(a[3], b[3])
    del x, a, b
    torch.cuda.empty_cache()
