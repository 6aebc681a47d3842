"""ORACLE — TEST INFRASTRUCTURE ONLY. numpy restatement of ADFL's stochastic gradient codecs.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py`` may import this module; the product package
never does. Pinned against ``tests/golden/stoch.npz`` (``tests/golden/make_golden_stoch.py``: the reference
channels EXECUTED in place with ``torch.rand_like`` replaced by recorded uniforms, torch 2.10.0+rocm7.0).

Restated reference lines (``Src/ADFL/Channel/quant.py``):
  QSGD   ``_quantize_tensor`` :223-240, ``_dequantize_tensor`` :243-252   (levels = 2**bits - 1, :147)
  RQSGD  ``_quantize_tensor`` :364-382, ``_dequantize_tensor`` :385-398
  CNAT   ``_quantize_tensor`` :509-534, ``_dequantize_tensor`` :537-545

Every elementwise step is the fp32 operation torch performs (numpy float32 ops are IEEE correctly
rounded, as are torch's CPU kernels for these ops), in torch's operation order:
  QSGD   scaled = fl(fl(s*|x|) / norm); l = floor(scaled); prob = scaled - l (exact);
         q = u8(l + (u < prob)); signs = i8(sign(x)).
         decode: fl(fl(fl(norm*q) / s) * sign)
  RQSGD  same levels with norm = max|x|, min_factor = min|x|;
         decode: fl(fl(fl(norm*sign)*q) / s), and min_factor*sign where q == 0.
  CNAT   v = fl(|x| + 2^-23); lg = fl32(log2 v); f, c = floor(lg), ceil(lg);
         prob = fl(2^c - |x|) / 2^f; e = (u < prob) ? f : c, clamped to [-2^(b-1), 2^(b-1)-1];
         e = -2^(b-1) where x == 0; i8(e).   decode: fl(fl(norm*sign) * 2^e)
  Conversions float -> u8 / i8 are torch's: the low byte of the truncated int32, NaN -> 0.
  norm == 0 (all zeros): levels u8 zeros, signs ones, scale = tensor(0.), decode zeros.

Norms. torch's fp32 ``vector_norm`` (ord=2) squares in fp32 and accumulates in fp32 in an order that
cannot be parallelised (its error grows with n: -7e-4 relative at 2^24 elements). The restatement here —
and the HIP kernels — square in fp32 (so overflow / underflow of x^2 behave as torch's), accumulate
those squares in fp64, round the sum once to fp32 and take a correctly rounded fp32 sqrt. It differs
from torch only by torch's own accumulation error; the golden tests bound that difference and then
inject the reference's norm to check every level, sign and decoded float bit-exactly. ord=inf / -inf
(max|x|, min|x|, NaN-propagating) are exact.

CNAT's fp32 log2 is restated as the correctly rounded value (float64 log2 rounded once to fp32).
torch's CPU log2 (SLEEF, <= 1 ulp) makes the same floor/ceil decision on EVERY fp32 value >= 2^-23
(tools/check_log2_exhaustive.py: 1,266,679,808 values, 0 mismatches); tests/test_stoch_golden.py re-checks
the powers-of-two neighbourhoods. The HIP kernel uses the equivalent integer band rule of
ad-federatedlearning_amd/csrc/cnat_log2_table.h (tools/gen_cnat_table.py --verify: 0 mismatches).

Uniforms. The reference draws ``torch.rand_like`` from torch's CPU mt19937 stream. The HIP codec draws
from a counter-based Philox4x32-7 stream instead (``philox_uniforms`` below restates it bit-exactly) or
takes injected uniforms; with the same uniforms every output is bit-identical to the reference.
"""

import os

import numpy as np

F32 = np.float32
EPS32 = F32(np.finfo(np.float32).eps)  # torch.finfo(torch.float32).eps = 2^-23 (quant.py:522)


# ------------------------------------------------------------------------------------------------
# torch conversion semantics
# ------------------------------------------------------------------------------------------------
def _trunc_i32(v: np.ndarray) -> np.ndarray:
    """float32 -> int32 as x86 cvttss2si: truncation; NaN and out-of-range -> INT32_MIN."""
    v = np.asarray(v, dtype=np.float32)
    out = np.full(v.shape, np.iinfo(np.int32).min, dtype=np.int64)
    ok = np.isfinite(v) & (v > -2147483648.0) & (v < 2147483648.0)
    out[ok] = np.trunc(v[ok]).astype(np.int64)
    return out


def to_u8(v: np.ndarray) -> np.ndarray:
    """``Tensor.to(torch.uint8)`` on fp32 (quant.py:236): low byte of the truncated int32, NaN -> 0."""
    return (_trunc_i32(v) & 0xFF).astype(np.uint8)


def to_i8(v: np.ndarray) -> np.ndarray:
    """``Tensor.to(torch.int8)`` on fp32 (quant.py:238,534)."""
    return (_trunc_i32(v) & 0xFF).astype(np.uint8).view(np.int8)


def sign_i8(x: np.ndarray) -> np.ndarray:
    """``torch.sign(x).to(torch.int8)``: -1 / 0 / 1, NaN -> 0."""
    x = np.asarray(x, dtype=np.float32)
    return ((x > 0).astype(np.int8) - (x < 0).astype(np.int8)).astype(np.int8)


# ------------------------------------------------------------------------------------------------
# norms
# ------------------------------------------------------------------------------------------------
def l2_norm(x: np.ndarray) -> np.float32:
    """fp32 squares, fp64 accumulation, one rounding to fp32, correctly rounded fp32 sqrt."""
    x = np.asarray(x, dtype=np.float32).reshape(-1)
    with np.errstate(over="ignore", invalid="ignore"):
        sq = (x * x).astype(np.float64)
        s32 = np.float32(sq.sum())
    return np.float32(np.sqrt(np.float64(s32)))  # sqrt of an fp32 in fp64 rounded once = correctly rounded


def torch_l2_norm(x: np.ndarray) -> np.float32:
    """``torch.linalg.vector_norm(x, ord=2)`` bit for bit as torch 2.10's CPU kernel computes it (the
    reference's own QSGD / CNAT norm, quant.py:226,512): 8 fp32 FMA lane accumulators in order, left-to-
    right lane sum, then the n % 8 tail as torch's compiled loop runs it — a group of 4 rounded squares, then
    FMA (oracle/slq_oracle.c
    ``oracle_torch_l2_norm``; pinned to every golden L2 norm by tests/test_stoch_golden.py)."""
    import ctypes
    import slq_oracle
    L = slq_oracle.lib()
    fn = L.oracle_torch_l2_norm
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int64], ctypes.c_float
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32).reshape(-1))
    return np.float32(fn(a.ctypes.data, a.size))


def linf_norm(x: np.ndarray) -> np.float32:
    """``vector_norm(x, ord=inf)`` = max|x|, NaN if any element is NaN."""
    a = np.abs(np.asarray(x, dtype=np.float32).reshape(-1))
    return np.float32(np.nan) if np.isnan(a).any() else np.float32(a.max())


def lminf_norm(x: np.ndarray) -> np.float32:
    """``vector_norm(x, ord=-inf)`` = min|x|, NaN if any element is NaN (quant.py:380)."""
    a = np.abs(np.asarray(x, dtype=np.float32).reshape(-1))
    return np.float32(np.nan) if np.isnan(a).any() else np.float32(a.min())


# ------------------------------------------------------------------------------------------------
# QSGD / RQSGD
# ------------------------------------------------------------------------------------------------
def qsgd_quantize(x: np.ndarray, levels: int, norm, u: np.ndarray):
    """quant.py:223-240 (and :364-377 for RQSGD with norm = max|x|). Returns (q u8, signs i8)."""
    x = np.asarray(x, dtype=np.float32)
    norm = F32(norm)
    if norm == 0:
        return np.zeros(x.shape, np.uint8), np.ones(x.shape, np.int8)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        scaled = (F32(levels) * np.abs(x)) / norm
        lo = np.floor(scaled)
        prob = scaled - lo
        up = (np.asarray(u, dtype=np.float32) < prob).astype(np.float32)
        q = to_u8(lo + up)
    return q, sign_i8(x)


def qsgd_dequantize(q: np.ndarray, signs: np.ndarray, levels: int, norm) -> np.ndarray:
    """quant.py:243-252: (norm * q / levels) * sign, zeros when norm == 0."""
    norm = F32(norm)
    if norm == 0:
        return np.zeros(q.shape, np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        mag = (norm * q.astype(np.float32)) / F32(levels)
        return mag * signs.astype(np.float32)


def rqsgd_dequantize(q: np.ndarray, signs: np.ndarray, levels: int, norm, min_factor) -> np.ndarray:
    """quant.py:385-398: norm * sign * q / levels, then min_factor * sign where q == 0."""
    norm = F32(norm)
    if norm == 0:
        return np.zeros(q.shape, np.float32)
    sf = signs.astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        res = ((norm * sf) * q.astype(np.float32)) / F32(levels)
        zero = q == 0
        res[zero] = F32(min_factor) * sf[zero]
    return res


# ------------------------------------------------------------------------------------------------
# CNAT
# ------------------------------------------------------------------------------------------------
def log2_f32(v: np.ndarray) -> np.ndarray:
    """Correctly rounded fp32 log2 (float64 log2 rounded once)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.log2(np.asarray(v, dtype=np.float32).astype(np.float64)).astype(np.float32)


def cnat_bounds(x_abs: np.ndarray):
    """floor / ceil of fl32(log2(fl(|x| + eps))) (quant.py:523-526)."""
    with np.errstate(over="ignore", invalid="ignore"):
        lg = log2_f32(x_abs + EPS32)
    return np.floor(lg), np.ceil(lg)


def _pow2(k: np.ndarray) -> np.ndarray:
    """torch's 2 ** k for integral fp32 k: exact (2^128 -> inf; 2^-127, 2^-128 are fp32 denormals)."""
    with np.errstate(over="ignore", invalid="ignore"):
        return np.exp2(np.asarray(k, dtype=np.float64)).astype(np.float32)


def cnat_quantize(x: np.ndarray, bits: int, norm, u: np.ndarray):
    """quant.py:509-534. Returns (exponents i8 — or u8 zeros for the norm == 0 branch, signs i8)."""
    x = np.asarray(x, dtype=np.float32)
    if F32(norm) == 0:
        return np.zeros(x.shape, np.uint8), np.ones(x.shape, np.int8)
    min_exp, max_exp = -(2 ** (bits - 1)), 2 ** (bits - 1) - 1
    xa = np.abs(x)
    f, c = cnat_bounds(xa)
    with np.errstate(over="ignore", invalid="ignore"):
        prob = (_pow2(c) - xa) / _pow2(f)
        lower = np.asarray(u, dtype=np.float32) < prob
        e = np.where(lower, f, c).astype(np.float32)
        e = np.where(np.isnan(e), e, np.clip(e, F32(min_exp), F32(max_exp)))  # clamp_ keeps NaN
        e[x == 0] = F32(min_exp)
    return to_i8(e), sign_i8(x)


def cnat_dequantize(e: np.ndarray, signs: np.ndarray, norm) -> np.ndarray:
    """quant.py:537-545: norm * sign * 2^e (zeros when norm == 0)."""
    norm = F32(norm)
    if norm == 0:
        return np.zeros(e.shape, np.float32)
    with np.errstate(over="ignore", invalid="ignore"):
        return (norm * signs.astype(np.float32)) * _pow2(e)


# ------------------------------------------------------------------------------------------------
# Philox4x32-7 uniforms (the HIP codec's production stream, csrc/stoch_codec.hip kPhiloxRounds)
# ------------------------------------------------------------------------------------------------
PHILOX_M0, PHILOX_M1 = 0xD2511F53, 0xCD9E8D57
PHILOX_W0, PHILOX_W1 = 0x9E3779B9, 0xBB67AE85
# the codec's stream; 10 is Random123's / curand's default (known-answer vectors). ADFL_PHILOX_ROUNDS=10
# follows an opt-in 10-round build of the library (csrc/philox.h)
PHILOX_ROUNDS = int(os.environ.get("ADFL_PHILOX_ROUNDS", "7"))
MASK32 = 0xFFFFFFFF


def philox_round(c0, c1, c2, c3, k0: int, k1: int):
    """One Philox4x32 round (S-box multiply + key xor) on uint64 arrays holding 32-bit words."""
    p0 = c0 * np.uint64(PHILOX_M0)
    p1 = c2 * np.uint64(PHILOX_M1)
    hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK32)
    hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK32)
    return hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0


def philox4x32(ctr_lo: np.ndarray, ctr_hi: np.ndarray, seed: int, ctr2: int = 0, ctr3: int = 0,
               rounds: int = PHILOX_ROUNDS, first_round: int = 0, state=None):
    """Philox4x32-R (Salmon et al., SC'11) on counters (ctr_lo, ctr_hi, ctr2, ctr3), key = 64-bit seed (the
    codec always uses ctr2 = ctr3 = 0). Returns the four uint32 output words (arrays). `state` / `first_round`
    continue a computation: rounds first_round .. rounds-1 applied to the words `state` (the key schedule
    bumped first_round times), so philox4x32(..., 10) == 3 more rounds on philox4x32(..., 7)."""
    if state is None:
        c0 = np.asarray(ctr_lo, dtype=np.uint64) & MASK32
        c1 = np.asarray(ctr_hi, dtype=np.uint64) & MASK32
        c2 = np.full_like(c0, ctr2 & MASK32)
        c3 = np.full_like(c0, ctr3 & MASK32)
    else:
        c0, c1, c2, c3 = (np.asarray(w, dtype=np.uint64) for w in state)
    k0 = (seed + first_round * PHILOX_W0) & MASK32
    k1 = ((seed >> 32) + first_round * PHILOX_W1) & MASK32
    for _ in range(first_round, rounds):
        c0, c1, c2, c3 = philox_round(c0, c1, c2, c3, k0, k1)
        k0 = (k0 + PHILOX_W0) & MASK32
        k1 = (k1 + PHILOX_W1) & MASK32
    return c0, c1, c2, c3


def philox_uniforms(n: int, seed: int, counter: int, start: int = 0) -> np.ndarray:
    """Uniforms [0, 1) for flat elements start .. start+n-1 of a stream (seed, counter): element e takes
    word e % 4 of Philox block (counter + e // 4), as (word >> 8) * 2^-24 (24 random bits, the same
    resolution as torch.rand on fp32)."""
    e = np.arange(start, start + n, dtype=np.uint64)
    blk = np.uint64(counter) + (e >> np.uint64(2))
    w = philox4x32(blk & np.uint64(MASK32), blk >> np.uint64(32), seed)
    words = np.stack(w, axis=0)  # [4, n]
    sel = words[(e & np.uint64(3)).astype(np.int64), np.arange(n)]
    return ((sel >> np.uint64(8)).astype(np.float32) * F32(2.0 ** -24)).astype(np.float32)
