"""GPU: adfl_torch_norms (csrc/torch_norm.hip) — torch's CPU vector_norm(ord=2) of fp32 / bf16 / fp16 / fp64
buckets bit for bit, the reference's QSGD / CNAT norm in the tensor's own dtype (quant.py:226,512).

Every norm is compared with torch.linalg.vector_norm itself, run on this box's CPU (torch is the oracle's
own source here: the restatements in oracle/slq_oracle.c are pinned to it on CPU by
tests/test_torch_norm_dtypes.py), on data that exercises every branch of the phased kernels: binade
crossings, ties (short-mantissa and integer data), misses of the binade predictor (chains that jump in
scale, stagnating fp32 sums), subnormal and overflowing squares, NaN and inf, the tails (n % 8, n % 16,
n % 4), fp16's at::parallel_for split at 1 / 3 / 8 / 64 threads, short tensors (one phase) and long ones
(four), compact and aligned buckets; then single tensors of 2^20, 2^24 + 5 and 2^28 elements.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from adfl_amd import ops, stoch  # noqa: E402

DEV = torch.device("cuda", 0)
DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
_SUB_BITS = {torch.float32: (0x00800000, np.uint32), torch.float16: (0x0400, np.uint16),
             torch.bfloat16: (0x0080, np.uint16), torch.float64: (1 << 52, np.uint64)}


def _data(kind: str, n: int, rng, dtype) -> torch.Tensor:
    f = np.float64
    if kind == "randn":
        x = rng.standard_normal(n)
    elif kind == "grad":
        x = rng.standard_normal(n) * 1e-3
    elif kind == "ints":
        x = np.trunc(rng.standard_normal(n) * 20)
    elif kind == "short":  # few mantissa bits: ties
        x = np.round(rng.standard_normal(n) * 16) / 64
    elif kind == "tiny_short":  # low binades (u / 2 subnormal) with ties: x^2 near 2^-112, few mantissa bits
        x = np.round(rng.standard_normal(n) * 16) / 64 * 2.0 ** -56
    elif kind == "const":
        x = np.full(n, 0.6, f)
    elif kind == "wide":
        span = 60 if dtype in (torch.float32, torch.float64) else (7 if dtype == torch.float16 else 60)
        x = rng.standard_normal(n) * np.exp2(rng.integers(-span, span, n))
    elif kind == "jump":
        x = rng.standard_normal(n) * 1e-3
        x[n // 3:] *= 4096.0
        x[2 * n // 3:] /= 65536.0
    elif kind == "under":
        tiny = {torch.float32: 1e-23, torch.float16: 1e-5, torch.bfloat16: 1e-25, torch.float64: 1e-170}[dtype]
        x = rng.standard_normal(n) * tiny
    elif kind == "sub":  # subnormal values of the dtype
        hi, u = _SUB_BITS[dtype]
        signed = {np.uint16: np.int16, np.uint32: np.int32, np.uint64: np.int64}[u]
        return torch.from_numpy(rng.integers(0, hi, n).astype(u).view(signed).copy()).view(dtype)
    elif kind == "over":
        big = {torch.float32: 1e19, torch.float16: 300.0, torch.bfloat16: 1e19, torch.float64: 1e155}[dtype]
        x = rng.standard_normal(n) * big
    elif kind == "nan":
        x = rng.standard_normal(n)
        x[rng.integers(0, n, max(1, n // 5000))] = np.nan
    elif kind == "inf":
        x = rng.standard_normal(n)
        x[rng.integers(0, n)] = np.inf
    elif kind == "late_nan":
        x = rng.standard_normal(n)
        x[min(8, n - 1)] = -np.inf
        x[max(n - 9, 0)] = np.nan
    elif kind == "zeros":
        x = np.zeros(n, f)
    else:
        raise ValueError(kind)
    return torch.from_numpy(x).to(dtype)


KINDS = ["randn", "grad", "ints", "short", "tiny_short", "const", "wide", "jump", "under", "sub", "over", "nan", "inf",
         "late_nan", "zeros"]
SIZES = [1, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65, 1023, 1025, 4097, 8192, 8199, 12289, 32767, 32768,
         32769, 45663, 65536, 65537, 65541, 100003, 131075, 200011, 524288, 524291]  # fp32 short bound 2^19


def _torch_norm(x: torch.Tensor, threads: int) -> float:
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        return torch.linalg.vector_norm(x).item()
    finally:
        torch.set_num_threads(old)


def _same(a: float, b: float) -> bool:
    return (np.isnan(a) and np.isnan(b)) or np.float64(a).view(np.uint64) == np.float64(b).view(np.uint64)


def _bucket(xs, align, dtype):
    lay = ops.BucketLayout([x.numel() for x in xs], align=align)
    flat = torch.zeros(lay.total, dtype=dtype)
    for x, o in zip(xs, lay.offsets):
        flat[o:o + x.numel()] = x
    return lay, flat.to(DEV)


def _run(xs, align, dtype, threads, tag):
    lay, flat = _bucket(xs, align, dtype)
    n64, n32 = stoch.reference_norms(flat, lay, threads=threads, out32=torch.empty(lay.ntensors, device=DEV),
                                     out64=torch.empty(lay.ntensors, dtype=torch.float64, device=DEV))
    got = n64.cpu().numpy()
    got32 = n32.cpu().numpy()
    for i, x in enumerate(xs):
        want = _torch_norm(x, threads)
        assert _same(got[i], want), (tag, i, x.numel(), float(got[i]), want)
        assert _same(float(np.float32(got32[i])), float(np.float32(want))), (tag, i)


@pytest.mark.parametrize("align", [1, 64])
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("dt", list(DTYPES))
def test_reference_norms_every_dtype(dt, kind, align):
    dtype = DTYPES[dt]
    rng = np.random.default_rng(KINDS.index(kind) * 8 + list(DTYPES).index(dt) * 2 + (align == 64))
    xs = [_data(kind, n, rng, dtype) for n in SIZES]
    _run(xs, align, dtype, 8, (dt, kind))


@pytest.mark.parametrize("threads", [1, 3, 64])
@pytest.mark.parametrize("kind", ["grad", "short", "jump", "nan"])
def test_reference_norms_fp16_thread_split(kind, threads):
    rng = np.random.default_rng(threads)
    xs = [_data(kind, n, rng, torch.float16) for n in (32767, 32768, 65536, 65537, 100003, 300007, 1 << 20)]
    _run(xs, 1, torch.float16, threads, ("f16", kind, threads))


@pytest.mark.parametrize("dt", list(DTYPES))
def test_reference_norms_c3_like(dt):
    """ResNet-18-sized bucket (256 tensors, log-uniform sizes 64..2.4 M) in each dtype."""
    dtype = DTYPES[dt]
    rng = np.random.default_rng(33)
    sizes = np.exp(rng.uniform(np.log(64), np.log(2_400_000), 256)).astype(np.int64)
    xs = [_data("grad", int(n), rng, dtype) for n in sizes]
    _run(xs, 64, dtype, 8, (dt, "c3"))


@pytest.mark.parametrize("n", [1 << 20, (1 << 24) + 5, 1 << 28])
@pytest.mark.parametrize("dt", list(DTYPES))
def test_reference_norms_one_big_tensor(dt, n):
    """One tensor of 2^20 / 2^24 + 5 / 2^28 elements: the value torch.linalg.vector_norm gives on this box."""
    dtype = DTYPES[dt]
    g = torch.Generator().manual_seed(n % 1000 + len(dt))
    x = (torch.randn(n, generator=g, dtype=torch.float32) * 1e-3).to(dtype)
    lay = ops.BucketLayout([n], align=1)
    threads = torch.get_num_threads()
    n64, _ = stoch.reference_norms(x.to(DEV), lay, threads=threads)
    want = torch.linalg.vector_norm(x).item()
    assert _same(n64.item(), want), (dt, n, n64.item(), want)


@pytest.mark.parametrize("dt", list(DTYPES))
def test_reference_norms_many_threads(dt):
    """A host with more than 512 torch threads: fp32 / bf16 / fp64 do not depend on the count, fp16's split
    is at most ceil(n / 32768) pieces whatever it is (stoch.reference_norms clamps it)."""
    dtype = DTYPES[dt]
    rng = np.random.default_rng(5)
    xs = [_data("grad", n, rng, dtype) for n in (5, 32769, 100003, 300007)]
    lay, flat = _bucket(xs, 1, dtype)
    n64, _ = stoch.reference_norms(flat, lay, threads=1024)
    got = n64.cpu().numpy()
    for i, x in enumerate(xs):
        # torch itself at 16 threads splits these fp16 tensors as it would at 1024 (at most 10 pieces)
        assert _same(got[i], _torch_norm(x, 16)), (dt, i)


def test_reference_norms_abi_rejects_bad_arguments():
    from adfl_amd import _lib
    L = _lib.load()
    lay = ops.BucketLayout([100], align=1)
    x = torch.zeros(100, device=DEV)
    nrm = torch.empty(1, dtype=torch.float64, device=DEV)
    need = L.adfl_torch_norm_scratch_bytes(lay.nchunks, 1)
    assert need > 0 and L.adfl_torch_norm_scratch_bytes(-1, 1) < 0
    buf = torch.zeros(need + 256, dtype=torch.uint8, device=DEV)
    ch = lay.device_chunks(DEV).data_ptr()
    args = lambda **k: dict(dict(dtype=0, x=x.data_ptr(), ch=ch, nc=lay.nchunks, nt=1, kinds=0, threads=1,  # noqa: E731
                                 s=buf.data_ptr(), sb=need, n64=nrm.data_ptr(), n32=None), **k)
    call = lambda a: L.adfl_torch_norms(a["dtype"], a["x"], a["ch"], a["nc"], a["nt"], a["kinds"], a["threads"],  # noqa: E731
                                        a["s"], a["sb"], a["n64"], a["n32"], None)
    assert call(args()) == 0
    assert call(args(sb=need - 1)) == -4
    assert call(args(s=buf.data_ptr() + 8)) == -3
    assert call(args(x=None)) == -1
    assert call(args(dtype=7)) == -1
    assert call(args(threads=0)) == -1
    assert call(args(threads=513)) == 0            # fp32 does not use threads
    assert call(args(threads=1 << 20)) == 0
    x16 = torch.zeros(100, dtype=torch.float16, device=DEV)
    assert call(args(dtype=1, x=x16.data_ptr(), threads=512)) == 0
    assert call(args(dtype=1, x=x16.data_ptr(), threads=513)) == -1   # fp16: at most 512 pieces
    assert call(args(n64=None)) == -1
    assert call(args(nt=2)) == -1
    assert L.adfl_torch_norm_short_max() == 1 << 16
    # one block per tensor up to these sizes (k_tn_short / k_tn_short_bf16 / k_tn_short_f16; fp64: phase D)
    assert [L.adfl_torch_norm_short_max_dt(d) for d in (_lib.DTYPE_F32, _lib.DTYPE_BF16, _lib.DTYPE_F16,
                                                         _lib.DTYPE_F64)] == [1 << 19, 1 << 19, 1 << 16, 1 << 16]
    assert L.adfl_torch_norm_short_max_dt(7) < 0
    torch.cuda.synchronize()
