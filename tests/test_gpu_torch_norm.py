"""GPU: the fp32 reference-order L2 norm (stoch.torch_norms -> adfl_torch_norms: csrc/torch_norm.hip for long
tensors, the in-order walker csrc/torch_norm_walk.h for short ones), torch's fp32 vector_norm order.

The norm must equal the reference's — torch 2.10's CPU vector_norm, restated in the oracle
(oracle_torch_l2_norm, pinned to every golden norm by tests/test_stoch_golden.py) — bit for bit, on data
that exercises every branch of the phased kernels: binade crossings (every tensor's first tiles), ties
(integer and short-mantissa data, where R(p/u) lands on a half), misses of the grid predictor (a chain
whose values jump in scale), subnormal and overflowing squares, NaN and inf, empty tiles and the n % 8
tail, tensors below 8 elements. Also against the sequential one-wave kernel
(norms_batched NORM_L2_TORCH), across repeated launches and two layouts alternating.
"""

import numpy as np
import pytest
import torch

from golden_util import same_f32

import stoch_oracle as so

pytestmark = pytest.mark.gpu

from adfl_amd import ops, stoch  # noqa: E402

DEV = torch.device("cuda", 0)


def d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def h(t):
    return t.detach().cpu().numpy()


def _data(kind: str, n: int, rng) -> np.ndarray:
    f32 = np.float32
    if kind == "randn":
        return rng.standard_normal(n, dtype=f32)
    if kind == "grad":  # the bench's data
        return rng.standard_normal(n, dtype=f32) * f32(1e-3)
    if kind == "ints":  # exact squares, ties once the accumulator passes 2^24 ulps of 1
        return np.trunc(rng.standard_normal(n) * 20).astype(f32)
    if kind == "bf16":  # short mantissas: ties
        return (rng.standard_normal(n, dtype=f32).view(np.uint32) & np.uint32(0xffff0000)).view(f32)
    if kind == "const":
        return np.full(n, 0.6, f32)
    if kind == "quarters":
        return (rng.integers(0, 5, n) * 0.25).astype(f32) * (rng.random(n) > 0.15)
    if kind == "wide":  # scales over 2^+-60: crossings everywhere, predictor misses
        return (rng.standard_normal(n) * np.exp2(rng.integers(-60, 60, n))).astype(f32)
    if kind == "jump":  # a chain that changes scale mid-tensor: the fp64 predictor runs ahead of the chain
        x = rng.standard_normal(n, dtype=f32) * f32(1e-3)
        x[n // 3:] *= f32(4096.0)
        x[2 * n // 3:] *= f32(1.0 / 65536.0)
        return x
    if kind == "under":  # squares below the smallest subnormal
        return rng.standard_normal(n, dtype=f32) * f32(1e-23)
    if kind == "sub":  # subnormal inputs
        return rng.integers(0, 0x00800000, n, dtype=np.uint32).view(f32)
    if kind == "over":  # squares overflow: inf
        return rng.standard_normal(n, dtype=f32) * f32(1e19)
    if kind == "nan":
        x = rng.standard_normal(n, dtype=f32)
        x[rng.integers(0, n, max(1, n // 5000))] = np.nan
        return x
    if kind == "inf":
        x = rng.standard_normal(n, dtype=f32)
        x[rng.integers(0, n)] = np.inf
        return x
    if kind == "late_nan":  # inf first, NaN later in the same chain: NaN
        x = rng.standard_normal(n, dtype=f32)
        x[min(8, n - 1)] = -np.inf
        x[max(n - 9, 0)] = np.nan
        return x
    if kind == "zeros":
        return np.zeros(n, f32)
    raise ValueError(kind)


KINDS = ["randn", "grad", "ints", "bf16", "const", "quarters", "wide", "jump", "under", "sub", "over", "nan",
         "inf", "late_nan", "zeros"]
SIZES = [1, 3, 7, 8, 9, 15, 16, 63, 64, 65, 4095, 4096, 4097, 4103, 8192, 8199, 12289, 45663, 65536, 65537, 65541,
         100003, 200011]


def _bucket(xs, align):
    lay = ops.BucketLayout([x.size for x in xs], align=align)
    flat = np.zeros(lay.total, np.float32)
    for x, o in zip(xs, lay.offsets):
        flat[o:o + x.size] = x
    return lay, flat


def _check(xs, got, tag):
    for i, x in enumerate(xs):
        want = np.array([so.torch_l2_norm(x)], np.float32)
        assert same_f32(got[i:i + 1], want), (tag, i, x.size, got[i], want[0])


@pytest.mark.parametrize("align", [1, 64])
@pytest.mark.parametrize("kind", KINDS)
def test_torch_norms_match_reference_order(kind, align):
    rng = np.random.default_rng(KINDS.index(kind) * 2 + (align == 64))
    xs = [_data(kind, n, rng) for n in SIZES]
    lay, flat = _bucket(xs, align)
    xd = d(flat)
    got = h(stoch.torch_norms(xd, lay))
    _check(xs, got, kind)
    seq, _ = stoch.norms_batched(xd, lay, stoch.NORM_L2_TORCH)
    assert same_f32(got, h(seq))


@pytest.mark.parametrize("kind", ["grad", "randn", "bf16", "jump"])
def test_torch_norms_big_tensor(kind):
    """2^24 + 5 elements in one tensor: 4097 tiles, late binade crossings far from the tensor's start, the
    fp32 chain drifting below the fp64 prefix the predictor starts from."""
    rng = np.random.default_rng(5)
    x = _data(kind, (1 << 24) + 5, rng)
    lay = ops.BucketLayout([x.size], align=1)
    got = h(stoch.torch_norms(d(x), lay))
    _check([x], got, kind)


def test_torch_norms_repeat_and_alternate_layouts():
    """Repeated launches and two layouts of different tile counts alternating: every launch gives the same
    bits."""
    rng = np.random.default_rng(11)
    xa = [_data("grad", n, rng) for n in (45663,) * 40]
    xb = [_data("wide", n, rng) for n in SIZES]
    la, fa = _bucket(xa, 1)
    lb, fb = _bucket(xb, 64)
    da, db = d(fa), d(fb)
    ra = h(stoch.torch_norms(da, la))
    rb = h(stoch.torch_norms(db, lb))
    _check(xa, ra, "a")
    _check(xb, rb, "b")
    for _ in range(5):
        assert same_f32(h(stoch.torch_norms(da, la)), ra)
        assert same_f32(h(stoch.torch_norms(db, lb)), rb)


def test_torch_norms_c3_equal_layout():
    """C3's equal layout (256 tensors of 45,662-45,663 elements, packed back to back) at the bench data."""
    rng = np.random.default_rng(3)
    base, rem = divmod(11_689_512, 256)
    xs = [_data("grad", base + (1 if i < rem else 0), rng) for i in range(256)]
    lay, flat = _bucket(xs, 1)
    got = h(stoch.torch_norms(d(flat), lay))
    _check(xs, got, "c3")
