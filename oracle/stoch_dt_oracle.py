"""ORACLE — TEST INFRASTRUCTURE ONLY. numpy restatement of ADFL's stochastic codecs (QSGD / RQSGD / CNAT)
on fp16, bf16 and fp64 tensors.

Only ``tests/`` may import this module; the product package never does. Pinned against
``tests/golden/stoch_dt.npz`` (``tests/golden/make_golden_stoch_dt.py``: the reference channels EXECUTED in
place on fp16 / bf16 / fp64 tensors with ``torch.rand_like`` replaced by recorded uniforms of the tensor's
dtype, torch 2.10.0+rocm7.0).

The reference computes these codecs in the tensor's own dtype (``Src/ADFL/Channel/quant.py:223-240``,
``:364-382``, ``:509-534``): every elementwise op returns a tensor of that dtype. torch's CPU kernels for
fp16 / bf16 compute each op in fp32 and round the result to the dtype once; fp64 ops are fp64 ops. So,
with R() = round to the dtype (identity for fp64) and arithmetic in fp32 (fp64 for fp64):
  QSGD   scaled = R(R(s*|x|) / norm); l = floor(scaled); prob = R(scaled - l);
         q = u8(l + (u < prob))  (l + a fp32 0/1 tensor: fp32 for fp16 / bf16, fp64 for fp64);
         signs = i8(sign(x)).
  RQSGD  the same levels with norm = max|x|; min factor = min|x|.
  CNAT   v = R(|x| + eps_dtype); lg = fl_dtype(log2 v) (torch's fp16 / bf16 log2 is the correctly rounded
         value: tools/gen_cnat_dt_tables.py checks every value; fp64: numpy's log2, equal to torch's on the
         band windows); f, c = floor(lg), ceil(lg); prob = R(R(R(2^c) - |x|) / R(2^f));
         e = (u < prob) ? f : c, clamped; e = min_exp where x == 0; i8(e).
  Decode is the fp32 arithmetic of the fp32 codecs with scale = fp32(norm): ``scale * q.float()`` takes
  the Python float norm as an fp32 scalar (stoch_oracle.qsgd_dequantize etc. apply unchanged).
  Uniforms: torch.rand on these dtypes draws from a 2^-11 (fp16), 2^-8 (bf16) or 2^-53 (fp64) grid on
  [0, 1); the HIP codec's Philox stream draws from the same grids (``philox_uniforms_dt``).

Norms: the reference's fp16 / bf16 ``vector_norm`` squares and accumulates in fp32, takes an fp32 sqrt and
rounds to the dtype; here (and in the HIP kernels) the fp32 squares are accumulated in fp64, rounded
once to fp32, square-rooted (correctly rounded) and rounded to the dtype. fp64: fp64 squares summed in
fp64. Both differ from torch only by torch's own accumulation error; the golden tests inject the
reference's norm to check every byte.
"""

import numpy as np

import stoch_oracle as so

DT_F16, DT_BF16, DT_F64 = 1, 2, 3     # ADFL_DTYPE_* (include/adfl_stoch.h)
TORCH_NAME = {DT_F16: "float16", DT_BF16: "bfloat16", DT_F64: "float64"}
EPS = {DT_F16: 2.0 ** -10, DT_BF16: 2.0 ** -7, DT_F64: 2.0 ** -52}  # torch.finfo(dtype).eps (quant.py:522)
GRID_BITS = {DT_F16: 11, DT_BF16: 8, DT_F64: 53}


# ------------------------------------------------------------------------------------------------
# storage <-> compute values, rounding
# ------------------------------------------------------------------------------------------------
def rn_bf16(a: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (round to nearest even, NaN kept quiet), returned as fp32 values."""
    a = np.asarray(a, dtype=np.float32)
    b = a.view(np.uint32).astype(np.uint64)
    r = ((b + np.uint64(0x7FFF) + ((b >> np.uint64(16)) & np.uint64(1))) & np.uint64(0xFFFF0000)).astype(np.uint32)
    r = np.where(np.isnan(a), (b.astype(np.uint32) | np.uint32(0x00400000)) & np.uint32(0xFFFF0000), r)
    return r.astype(np.uint32).view(np.float32)


def rn_bf16_from_f64(a: np.ndarray) -> np.ndarray:
    """fp64 -> bf16 rounded ONCE (no fp32 step), for values in bf16's normal range, as fp32 values."""
    a = np.asarray(a, dtype=np.float64)
    b = a.view(np.uint64)
    r = (b + np.uint64((1 << 44) - 1) + ((b >> np.uint64(45)) & np.uint64(1))) & ~np.uint64((1 << 45) - 1)
    out = r.view(np.float64).astype(np.float32)   # exact: 8 significant bits
    return np.where(np.isfinite(a), out, a.astype(np.float32))


def R(a, dt):
    """Round compute values (fp32; fp64 for fp64) to the dtype; returns compute values."""
    if dt == DT_F16:
        return np.asarray(a, dtype=np.float32).astype(np.float16).astype(np.float32)
    if dt == DT_BF16:
        return rn_bf16(a)
    return np.asarray(a, dtype=np.float64)


def to_compute(raw: np.ndarray, dt) -> np.ndarray:
    """Stored values (uint16 bits for fp16 / bf16, float64) -> compute values (fp32 / fp64)."""
    raw = np.asarray(raw)
    if dt == DT_F16:
        return raw.view(np.uint16).view(np.float16).astype(np.float32)
    if dt == DT_BF16:
        return (raw.view(np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)
    return raw.view(np.float64).astype(np.float64)


def from_compute(v: np.ndarray, dt) -> np.ndarray:
    """Compute values already on the dtype's grid -> stored values (uint16 bits / float64)."""
    v = np.asarray(v)
    if dt == DT_F16:
        return v.astype(np.float16).view(np.uint16)
    if dt == DT_BF16:
        return (rn_bf16(v).view(np.uint32) >> np.uint32(16)).astype(np.uint16)
    return v.astype(np.float64)


def _ctype(dt):
    return np.float64 if dt == DT_F64 else np.float32


def _trunc_i64(v: np.ndarray) -> np.ndarray:
    """fp -> int32 as x86's truncating conversion: NaN and out-of-range -> INT32_MIN."""
    v = np.asarray(v, dtype=np.float64)
    out = np.full(v.shape, np.iinfo(np.int32).min, dtype=np.int64)
    ok = np.isfinite(v) & (v > -2147483648.0) & (v < 2147483648.0)
    out[ok] = np.trunc(v[ok]).astype(np.int64)
    return out


def to_u8(v):
    return (_trunc_i64(v) & 0xFF).astype(np.uint8)


def to_i8(v):
    return (_trunc_i64(v) & 0xFF).astype(np.uint8).view(np.int8)


def sign_i8(x):
    x = np.asarray(x)
    return ((x > 0).astype(np.int8) - (x < 0).astype(np.int8)).astype(np.int8)


# ------------------------------------------------------------------------------------------------
# norms (the HIP codec's definition; see the module docstring)
# ------------------------------------------------------------------------------------------------
def l2_norm(x_raw, dt) -> float:
    x = to_compute(x_raw, dt).reshape(-1)
    with np.errstate(over="ignore", invalid="ignore"):
        if dt == DT_F64:
            return float(np.sqrt(np.sum(x * x, dtype=np.float64)))
        sq = (x * x).astype(np.float64)
        s32 = np.float32(sq.sum())
        n32 = np.float32(np.sqrt(np.float64(s32)))
        return float(R(n32, dt))


def torch_l2_norm(x_raw, dt, threads: int = 1) -> float:
    """``torch.linalg.vector_norm(x, ord=2).item()`` on an fp16 / bf16 / fp64 CPU tensor bit for bit as torch
    2.10 computes it (the reference's QSGD / CNAT norm in the tensor's dtype, quant.py:226,512): the C
    restatements ``oracle_torch_l2_norm_{f16,bf16,f64}`` (oracle/slq_oracle.c), then torch's round-to-nearest
    conversion of the fp32 sqrt to the dtype. ``threads``: torch.get_num_threads() of the process whose
    norm is restated (fp16 tensors of >= 32768 elements are split across threads)."""
    import ctypes
    import slq_oracle
    L = slq_oracle.lib()
    raw = np.ascontiguousarray(np.asarray(x_raw).reshape(-1))
    if dt == DT_F64:
        fn = L.oracle_torch_l2_norm_f64
        fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int64], ctypes.c_double
        a = raw.view(np.float64)
        return float(fn(a.ctypes.data, a.size))
    a = raw.view(np.uint16)
    if dt == DT_BF16:
        fn = L.oracle_torch_l2_norm_bf16
        fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int64], ctypes.c_float
        return float(R(np.float32(fn(a.ctypes.data, a.size)), dt))
    fn = L.oracle_torch_l2_norm_f16
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32], ctypes.c_float
    return float(R(np.float32(fn(a.ctypes.data, a.size, int(threads))), dt))


def linf_norm(x_raw, dt) -> float:
    a = np.abs(to_compute(x_raw, dt).reshape(-1))
    return float("nan") if np.isnan(a).any() else float(a.max())


def lminf_norm(x_raw, dt) -> float:
    a = np.abs(to_compute(x_raw, dt).reshape(-1))
    return float("nan") if np.isnan(a).any() else float(a.min())


# ------------------------------------------------------------------------------------------------
# quantize (quant.py:223-240, :364-377, :509-534 in the tensor's dtype)
# ------------------------------------------------------------------------------------------------
def qsgd_quantize(x_raw, dt, bits: int, norm: float, u_raw):
    """QSGD / RQSGD levels (norm = L2 or max|x|) and signs. Returns (q u8, signs i8)."""
    x = to_compute(x_raw, dt)
    if norm == 0:
        return np.zeros(x.shape, np.uint8), np.ones(x.shape, np.int8)
    ct = _ctype(dt)
    s = ct(2 ** bits - 1)
    nrm = ct(norm)
    u = to_compute(u_raw, dt)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        a = R(s * np.abs(x), dt)
        scaled = R(a / nrm, dt)
        lo = np.floor(scaled)
        prob = R(scaled - lo, dt)
        up = (u < prob).astype(ct)
        q = to_u8(lo + up)
    return q, sign_i8(x)


def log2_dt(v: np.ndarray, dt) -> np.ndarray:
    """fl_dtype(log2 v): the correctly rounded value for fp16 / bf16 (torch's, checked on every value),
    numpy's fp64 log2 for fp64."""
    with np.errstate(divide="ignore", invalid="ignore"):
        lg = np.log2(np.asarray(v, dtype=np.float64))
    if dt == DT_F16:
        return lg.astype(np.float16).astype(np.float32)
    if dt == DT_BF16:
        return rn_bf16_from_f64(lg)
    return lg


def _pow2(k, dt):
    """torch's 2 ** k for integral k in the dtype: exact, inf past the dtype's range."""
    with np.errstate(over="ignore", invalid="ignore"):
        return R(np.exp2(np.asarray(k, dtype=np.float64)).astype(_ctype(dt)), dt)


def cnat_quantize(x_raw, dt, bits: int, norm: float, u_raw):
    """Returns (exponents i8 — u8 zeros on the norm == 0 branch, signs i8)."""
    x = to_compute(x_raw, dt)
    if norm == 0:
        return np.zeros(x.shape, np.uint8), np.ones(x.shape, np.int8)
    ct = _ctype(dt)
    min_exp, max_exp = -(2 ** (bits - 1)), 2 ** (bits - 1) - 1
    u = to_compute(u_raw, dt)
    xa = np.abs(x)
    with np.errstate(over="ignore", invalid="ignore"):
        v = R(xa + ct(EPS[dt]), dt)
        lg = log2_dt(v, dt).astype(ct)
        f, c = np.floor(lg), np.ceil(lg)
        prob = R(R(_pow2(c, dt) - xa, dt) / _pow2(f, dt), dt)
        lower = u < prob
        e = np.where(lower, f, c).astype(ct)
        e = np.where(np.isnan(e), e, np.clip(e, ct(min_exp), ct(max_exp)))
        e[x == 0] = ct(min_exp)
    return to_i8(e), sign_i8(x)


def quantize(codec: str, x_raw, dt, bits: int, norm: float, u_raw):
    if codec == "cnat":
        return cnat_quantize(x_raw, dt, bits, norm, u_raw)
    return qsgd_quantize(x_raw, dt, bits, norm, u_raw)


def encode(codec: str, x_raw, dt, bits: int, u_raw):
    """(q, signs, norm, min) with the HIP codec's norms."""
    if codec == "rqsgd":
        norm, mn = linf_norm(x_raw, dt), lminf_norm(x_raw, dt)
    else:
        norm, mn = l2_norm(x_raw, dt), 0.0
    q, sg = quantize(codec, x_raw, dt, bits, norm, u_raw)
    return q, sg, norm, mn


def decode(codec: str, q, signs, bits: int, norm: float, mn: float = 0.0) -> np.ndarray:
    """fp32 decode (the fp32 codecs' arithmetic with scale = fp32(norm), min = fp32(min))."""
    if codec == "qsgd":
        return so.qsgd_dequantize(q, signs, 2 ** bits - 1, np.float32(norm))
    if codec == "rqsgd":
        return so.rqsgd_dequantize(q, signs, 2 ** bits - 1, np.float32(norm), np.float32(mn))
    return so.cnat_dequantize(q.view(np.int8), signs, np.float32(norm))


# ------------------------------------------------------------------------------------------------
# Philox uniforms on the dtype's grid (the HIP codec's production stream for these dtypes)
# ------------------------------------------------------------------------------------------------
def philox_uniforms_dt(dt, n: int, seed: int, counter: int, start: int = 0) -> np.ndarray:
    """Stored uniforms for flat elements start .. start+n-1. fp16 / bf16: element e takes word e % 4 of
    Philox4x32-7 block (counter + e // 4), u = (word >> (32 - g)) * 2^-g with g = 11 / 8. fp64: element e
    takes words (2 (e % 2), 2 (e % 2) + 1) = (hi, lo) of block (counter + e // 2), u = ((hi:lo) >> 11) * 2^-53."""
    e = np.arange(start, start + n, dtype=np.uint64)
    if dt == DT_F64:
        blk = np.uint64(counter) + (e >> np.uint64(1))
        w = np.stack(so.philox4x32(blk & np.uint64(so.MASK32), blk >> np.uint64(32), seed), axis=0)
        odd = (e & np.uint64(1)).astype(np.int64)
        hi = w[2 * odd, np.arange(n)]
        lo = w[2 * odd + 1, np.arange(n)]
        bits53 = ((hi << np.uint64(32)) | lo) >> np.uint64(11)
        return (bits53.astype(np.float64) * 2.0 ** -53).astype(np.float64)
    g = GRID_BITS[dt]
    blk = np.uint64(counter) + (e >> np.uint64(2))
    w = np.stack(so.philox4x32(blk & np.uint64(so.MASK32), blk >> np.uint64(32), seed), axis=0)
    sel = w[(e & np.uint64(3)).astype(np.int64), np.arange(n)]
    u = (sel >> np.uint64(32 - g)).astype(np.float32) * np.float32(2.0 ** -g)
    return from_compute(u, dt)
