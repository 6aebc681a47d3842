"""ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatements of ADFL's SLQ codec used as the parity checker.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module; the product package never does (it fails loudly when its HIP library is missing instead).

Two independent restatements, both pinned against ``tests/golden/`` (vectors produced by executing
the reference ``Src/ADFL/Channel/quant.py`` in place, torch 2.10.0+rocm7.0, engine x86):

* ``C``     — ``oracle/slq_oracle.c`` through ctypes (``liboracle_slq.so``, built by ``oracle/Makefile``);
* ``numpy`` — the functions below with a ``np_`` prefix.

Reference lines restated: ``Src/ADFL/Channel/quant.py:97-104`` (encode), ``:107-112`` (decode),
``:74-94`` (per-tensor loop, passthrough of ``ndim<=1``), ``Src/ADFL/compression.py:35-66`` (int4),
``Examples/ray_ad.py:188`` (peer mean).

``aten_encode`` / ``aten_decode`` replay the reference's exact ATen op sequence
(``quant.py:100-103,110``) and are what ``bench.py`` times as the CPU baseline.
"""

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_slq.so")

_lib = None


def build() -> str:
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
        L.oracle_slq_absmax.argtypes, L.oracle_slq_absmax.restype = [P, I64], F
        L.oracle_slq_scale.argtypes, L.oracle_slq_scale.restype = [F, ctypes.c_int], F
        L.oracle_slq_quantize.argtypes, L.oracle_slq_quantize.restype = [P, I64, F, P], None
        L.oracle_slq_encode.argtypes, L.oracle_slq_encode.restype = [P, I64, ctypes.c_int, P], F
        L.oracle_slq_dequantize.argtypes, L.oracle_slq_dequantize.restype = [P, I64, F, P], None
        L.oracle_slq_encode_batched.argtypes = [P, P, P, I32, ctypes.c_int, P, P]
        L.oracle_slq_encode_batched.restype = None
        L.oracle_slq_dequantize_batched.argtypes = [P, P, P, I32, P, P]
        L.oracle_slq_dequantize_batched.restype = None
        L.oracle_pack_int4.argtypes, L.oracle_pack_int4.restype = [P, I64, P], I64
        L.oracle_unpack_int4.argtypes, L.oracle_unpack_int4.restype = [P, I64, P], None
        L.oracle_slq_dequantize_int4.argtypes, L.oracle_slq_dequantize_int4.restype = [P, I64, F, P], None
        L.oracle_slq_dequantize_mean.argtypes = [P, P, I32, I64, P]
        L.oracle_slq_dequantize_mean.restype = None
        L.oracle_slq_dequantize_mean_int4.argtypes = [P, P, I32, I64, P]
        L.oracle_slq_dequantize_mean_int4.restype = None
        L.oracle_slq_dequantize_mean_self.argtypes = [P, P, I32, I64, I32, P, I32, P]
        L.oracle_slq_dequantize_mean_self.restype = None
        L.oracle_torch_sum_col.argtypes, L.oracle_torch_sum_col.restype = [P, I32, I64, I64], F
        L.oracle_torch_mean_rows.argtypes, L.oracle_torch_mean_rows.restype = [P, I32, I64, P], None
        L.oracle_torch_sum_rows.argtypes, L.oracle_torch_sum_rows.restype = [P, I32, I64, P], None
        L.oracle_torch_sum_f32.argtypes, L.oracle_torch_sum_f32.restype = [P, I64, I32], F
        L.oracle_qerror_ref.argtypes, L.oracle_qerror_ref.restype = [P, P, P, I32, I32, P, P, P], None
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------- C restatement (ctypes) --------
def encode(x: np.ndarray, bits: int):
    """quant.py:97-104 -> (int8 payload shaped like x, fp32 scale)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    q = np.empty(x.shape, np.int8)
    s = lib().oracle_slq_encode(_ptr(x), x.size, bits, _ptr(q))
    return q, np.float32(s)


def decode(q: np.ndarray, scale) -> np.ndarray:
    """quant.py:107-112 for ndim>1."""
    q = np.ascontiguousarray(q, dtype=np.int8)
    out = np.empty(q.shape, np.float32)
    lib().oracle_slq_dequantize(_ptr(q), q.size, float(np.float32(scale)), _ptr(out))
    return out


def encode_batched(flat: np.ndarray, offsets, sizes, bits: int):
    flat = np.ascontiguousarray(flat, dtype=np.float32)
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    siz = np.ascontiguousarray(sizes, dtype=np.int64)
    q = np.zeros(flat.shape, np.int8)
    scales = np.empty(len(off), np.float32)
    lib().oracle_slq_encode_batched(_ptr(flat), _ptr(off), _ptr(siz), len(off), bits, _ptr(q), _ptr(scales))
    return q, scales


def pack_int4(q: np.ndarray) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.int8).reshape(-1)
    out = np.empty((q.size + 1) // 2, np.uint8)
    lib().oracle_pack_int4(_ptr(q), q.size, _ptr(out))
    return out


def unpack_int4(packed: np.ndarray, n: int) -> np.ndarray:
    packed = np.ascontiguousarray(packed).view(np.uint8).reshape(-1)
    out = np.empty(n, np.int8)
    lib().oracle_unpack_int4(_ptr(packed), n, _ptr(out))
    return out


def decode_int4(packed: np.ndarray, n: int, scale) -> np.ndarray:
    packed = np.ascontiguousarray(packed).view(np.uint8).reshape(-1)
    out = np.empty(n, np.float32)
    lib().oracle_slq_dequantize_int4(_ptr(packed), n, float(np.float32(scale)), _ptr(out))
    return out


def torch_sum_rows(rows) -> np.ndarray:
    """torch.sum(torch.stack(rows), dim=0) for K fp32 rows of one n-element tensor, in torch 2.10's CPU
    summation order (slq_oracle.c oracle_torch_sum_col; the sum simple_aggregate takes,
    Src/ADFL/model.py:229-231)."""
    m = np.ascontiguousarray(np.stack([np.asarray(r, np.float32).reshape(-1) for r in rows]), dtype=np.float32)
    out = np.empty(m.shape[1], np.float32)
    lib().oracle_torch_sum_rows(_ptr(m), m.shape[0], m.shape[1], _ptr(out))
    return out


def torch_mean_rows(rows) -> np.ndarray:
    """simple_aggregate of one tensor (Src/ADFL/model.py:229-231) = stack(rows).mean(0) (Examples/ray_ad.py:188):
    the torch-order sum, then a correctly rounded fp32 division by K."""
    m = np.ascontiguousarray(np.stack([np.asarray(r, np.float32).reshape(-1) for r in rows]), dtype=np.float32)
    out = np.empty(m.shape[1], np.float32)
    lib().oracle_torch_mean_rows(_ptr(m), m.shape[0], m.shape[1], _ptr(out))
    return out


def dequantize_mean(qs, scales) -> np.ndarray:
    qs = [np.ascontiguousarray(q, dtype=np.int8).reshape(-1) for q in qs]
    n = qs[0].size
    arr = (ctypes.c_void_p * len(qs))(*[q.ctypes.data for q in qs])
    sc = np.ascontiguousarray(scales, dtype=np.float32)
    out = np.empty(n, np.float32)
    lib().oracle_slq_dequantize_mean(arr, _ptr(sc), len(qs), n, _ptr(out))
    return out


def dequantize_mean_int4(packed_rows, scales, n: int) -> np.ndarray:
    ps = [np.ascontiguousarray(p).view(np.uint8).reshape(-1) for p in packed_rows]
    arr = (ctypes.c_void_p * len(ps))(*[p.ctypes.data for p in ps])
    sc = np.ascontiguousarray(scales, dtype=np.float32)
    out = np.empty(n, np.float32)
    lib().oracle_slq_dequantize_mean_int4(arr, _ptr(sc), len(ps), n, _ptr(out))
    return out


def dequantize_mean_self(rows, scales, n: int, self_row: int, self_x, packed: bool = False) -> np.ndarray:
    """Peer mean with the receiver's own update exact: rows (int8 payloads, or int4-packed with packed=True)
    other than self_row summed in order, self_x (fp32) added last, / K (async_peer.py:170-174)."""
    rs = [np.ascontiguousarray(r).view(np.uint8).reshape(-1) for r in rows]
    arr = (ctypes.c_void_p * len(rs))(*[r.ctypes.data for r in rs])
    sc = np.ascontiguousarray(scales, dtype=np.float32)
    sx = np.ascontiguousarray(self_x, dtype=np.float32).reshape(-1)
    out = np.empty(n, np.float32)
    lib().oracle_slq_dequantize_mean_self(arr, _ptr(sc), len(rs), n, int(self_row), _ptr(sx), int(packed), _ptr(out))
    return out


def dequantize_mean_batched(rows, scales, offsets, sizes, total: int, self_row: int = -1, self_x=None,
                            packed: bool = False) -> np.ndarray:
    """Peer mean of K bucketed int8 payloads with per-tensor scales: for each tensor t, dequantize_mean_self
    (self_row >= 0: the receiver's own fp32 values added last) or dequantize_mean over the rows' slices
    [offset_t, offset_t + size_t) with scales[r][t] (Examples/ray_ad.py:164-190 per tensor, quant.py:74-94).
    packed=True: int4-packed rows (even offsets; tensor t's bytes [offset_t / 2, ceil((offset_t + size_t) / 2)),
    compression.py:35-66), through the int4 mean restatements. Positions outside every tensor are 0."""
    out = np.zeros(total, np.float32)
    for t, (o, n) in enumerate(zip(offsets, sizes)):
        o, n = int(o), int(n)
        lo, hi = (o // 2, (o + n + 1) // 2) if packed else (o, o + n)
        rs = [np.ascontiguousarray(np.asarray(r).view(np.uint8).reshape(-1)[lo:hi]) for r in rows]
        sc = np.array([np.asarray(s, np.float32).reshape(-1)[t] for s in scales], np.float32)
        if self_row >= 0:
            out[o:o + n] = dequantize_mean_self(rs, sc, n, self_row, np.asarray(self_x, np.float32).reshape(-1)[o:o + n],
                                                packed=packed)
        elif packed:
            out[o:o + n] = dequantize_mean_int4(rs, sc, n)
        else:
            out[o:o + n] = dequantize_mean([r.view(np.int8) for r in rs], sc)
    return out


# ---------------------------------------------------------------- numpy restatement -------------
def np_encode(x: np.ndarray, bits: int):
    x = np.asarray(x, dtype=np.float32)
    qmax = np.float32(2 ** (bits - 1) - 1)
    absmax = np.max(np.abs(x))  # NaN propagates, as torch.max (quant.py:100)
    with np.errstate(all="ignore"):
        scale = np.float32(absmax) / qmax
        inv = np.float32(1.0) / scale
        y = x * inv
        y = np.where(np.isnan(y), np.float32(127), np.clip(y, np.float32(-128), np.float32(127)))
        q = np.rint(y).astype(np.int8)
    return q, np.float32(scale)


def np_decode(q: np.ndarray, scale) -> np.ndarray:
    with np.errstate(all="ignore"):
        return (np.float32(scale) * q.astype(np.float32)).astype(np.float32)


def np_pack_int4(q: np.ndarray) -> np.ndarray:
    q = np.asarray(q, dtype=np.int8).reshape(-1)
    if q.size & 1:
        q = np.concatenate([q, np.zeros(1, np.int8)])
    u = (q.astype(np.int16) + 8).astype(np.uint8)  # int8 wraparound
    return ((u[0::2] << 4).astype(np.uint8) | u[1::2]).astype(np.uint8)


def np_unpack_int4(packed: np.ndarray, n: int) -> np.ndarray:
    b = np.asarray(packed).view(np.uint8).reshape(-1)
    hi = ((b >> 4) & 0xF).astype(np.int8) - 8
    lo = (b & 0xF).astype(np.int8) - 8
    return np.stack([hi, lo], axis=1).reshape(-1)[:n].astype(np.int8)


# ---------------------------------------------------------------- reference ATen op sequence ----
def aten_encode(t, bits: int):
    """The exact op sequence of Src/ADFL/Channel/quant.py:99-104 (CPU baseline for bench.py)."""
    import torch
    q_max = 2 ** (bits - 1) - 1
    scale = torch.max(torch.abs(t)) / q_max
    q = torch.quantize_per_tensor(t, float(scale), 0, dtype=torch.qint8)
    return q, float(scale)


def aten_decode(q):
    """Src/ADFL/Channel/quant.py:110."""
    return q.dequantize()


def torch_sum_f32(x: np.ndarray, threads: int) -> float:
    """torch.sum of a contiguous fp32 tensor to a scalar, in torch 2.10's CPU order with `threads` threads
    (slq_oracle.c oracle_torch_sum_f32)."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    return float(lib().oracle_torch_sum_f32(_ptr(x), x.size, int(threads)))


def qerror_sums(xs, ds, threads: int):
    """Per-tensor fp32 sums e[t] = sum((x - d)^2), s[t] = sum(x^2) and the fp32 cosine sum over the
    concatenation (slq_oracle.c oracle_qerror_ref) for the ndim > 1 tensors xs / their decodes ds."""
    sizes = np.array([np.asarray(x).size for x in xs], dtype=np.int64)
    x = np.ascontiguousarray(np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in xs]))
    d = np.ascontiguousarray(np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in ds]))
    e = np.zeros(len(xs), np.float32)
    s = np.zeros(len(xs), np.float32)
    c = np.zeros(1, np.float32)
    lib().oracle_qerror_ref(_ptr(x), _ptr(d), _ptr(sizes), len(xs), int(threads), _ptr(e), _ptr(s), _ptr(c))
    return e, s, float(c[0])


def qerror_metrics(xs, ds, threads: int):
    """(parameter_relative_mse, parameter_cosine_similarity) as the reference returns them
    (Src/ADFL/model.py:256-323, exclude_bias=True over the ndim > 1 tensors xs, in dict order): Python-double
    sums of the fp32 per-tensor sums, each divided by the element count, then their ratio."""
    e, s, c = qerror_sums(xs, ds, threads)
    n = sum(int(np.asarray(x).size) for x in xs)
    num = 0.0
    den = 0.0
    for v in e.tolist():
        num += v
    for v in s.tolist():
        den += v
    num = num / n if n > 0 else 0.0
    den = den / n if n > 0 else 0.0
    return (num / den if den > 0 else 0.0), c
