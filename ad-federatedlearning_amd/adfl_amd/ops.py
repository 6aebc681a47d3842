"""Device-resident SLQ codec ops over the HIP C ABI (include/adfl_slq.h).

Every function here takes and returns CUDA (HIP) tensors, launches on the current stream and never
synchronises. Semantics are the reference's, bit for bit:

* ``encode``  — ``SLQChannel._quantize_tensor`` (Src/ADFL/Channel/quant.py:97-104)
* ``decode``  — ``SLQChannel._dequantize_tensor`` (quant.py:107-112)
* ``encode_batched`` / ``decode_batched`` — the per-tensor loop of ``_quantize_params`` / ``_receive``
  (quant.py:67-94) as one launch per pass over a whole bucketed state dict
* ``encode_int4`` / ``decode_int4`` / ``pack_int4`` / ``unpack_int4`` — Src/ADFL/compression.py:35-66
* ``dequantize_mean`` — the peer mean after the exchange (Examples/ray_ad.py:188); ``dequantize_mean_batched``
  the same over bucketed payloads with per-tensor scales

The same ops are registered as PyTorch custom ops ``torch.ops.adfl.*`` (with fake implementations, so
they trace under torch.compile) at the bottom of this file: slq_absmax, slq_encode / slq_decode,
slq_encode_int4 / slq_decode_int4, slq_encode_batched / slq_decode_batched and their _int4 variants over
caller-placed tensors (host offsets / sizes), pack_int4 / unpack_int4, slq_dequantize_mean and
slq_dequantize_mean_batched (+ _int4).
"""

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import ALIGN_ELEMS, Chunk, check

_TORCH_TYPE_NAMES = {
    torch.float64: "Double", torch.float16: "Half", torch.bfloat16: "BFloat16", torch.int64: "Long",
    torch.int32: "Int", torch.int16: "Short", torch.int8: "Char", torch.uint8: "Byte", torch.bool: "Bool",
    torch.complex64: "ComplexFloat", torch.complex128: "ComplexDouble",
}
EMPTY_MAX_MSG = ("max(): Expected reduction dim to be specified for input.numel() == 0. "
                 "Specify the reduction dim with the 'dim' argument.")


def require_quantizable(t: torch.Tensor) -> None:
    """Raise exactly what the reference raises for a tensor it cannot quantize (quant.py:100-103)."""
    if t.numel() == 0:
        raise RuntimeError(EMPTY_MAX_MSG)
    if t.dtype != torch.float32:
        name = _TORCH_TYPE_NAMES.get(t.dtype, str(t.dtype).replace("torch.", ""))
        raise RuntimeError(f"Quantize only works on Float Tensor, got {name}")


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _dev(t: torch.Tensor, what: str) -> torch.Tensor:
    """A contiguous, 16-byte aligned device view of t (copying only when it is not already one)."""
    if not t.is_cuda:
        raise ValueError(f"adfl_amd.ops: {what} must be a CUDA/HIP device tensor, got {t.device}")
    if not t.is_contiguous():
        t = t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def _f32_on(t: torch.Tensor, n: int, dev: torch.device, what: str) -> torch.Tensor:
    """An fp32 tensor of >= n elements on `dev` as a contiguous, 16-byte aligned device view (scales, self_x):
    a host tensor, another device, another dtype or a short tensor raises instead of reaching a kernel."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.device != dev:
        raise ValueError(f"adfl_amd.ops: {what} must be a device tensor on {dev}, got "
                         f"{getattr(t, 'device', type(t).__name__)}")
    if t.dtype != torch.float32:
        raise ValueError(f"adfl_amd.ops: {what} must be float32, got {t.dtype}")
    if t.numel() < n:
        raise ValueError(f"adfl_amd.ops: {what} needs >= {n} elements, got {t.numel()}")
    return _dev(t, what)


def _scale_rows(scales: torch.Tensor, k: int, ncols: int, dev: torch.device, what: str) -> torch.Tensor:
    """K rows of >= ncols fp32 scales with unit column stride (row r's scale for tensor t at [r, t])."""
    if not isinstance(scales, torch.Tensor) or not scales.is_cuda or scales.device != dev:
        raise ValueError(f"adfl_amd.ops: {what} must be a device tensor on {dev}")
    if scales.dtype != torch.float32:
        raise ValueError(f"adfl_amd.ops: {what} must be float32, got {scales.dtype}")
    if scales.numel() % k:
        raise ValueError(f"adfl_amd.ops: {what} has {scales.numel()} elements, not a multiple of K = {k}")
    sc = scales.reshape(k, -1)
    if sc.shape[1] < ncols:
        raise ValueError(f"adfl_amd.ops: {what} must be [K, >= {ncols}] fp32")
    if sc.stride(1) != 1 or sc.data_ptr() % 4:
        sc = sc.contiguous()
    return sc


def _dst(out: Optional[torch.Tensor], n: int, dtype: torch.dtype, dev: torch.device, what: str,
         zero: bool = False, align: int = 16) -> torch.Tensor:
    """A caller's output tensor checked (contiguous, `align`-byte aligned, dtype, >= n elements, on dev), or a
    new one."""
    if out is None:
        return (torch.zeros if zero else torch.empty)(n, dtype=dtype, device=dev)
    if (not out.is_cuda or out.device != dev or out.dtype != dtype or not out.is_contiguous()
            or out.numel() < n or out.data_ptr() % align):
        raise ValueError(f"adfl_amd.ops: {what} must be a contiguous, {align}-byte aligned {dtype} tensor of "
                         f">= {n} elements on {dev}")
    return out


def new_workspace(device) -> torch.Tensor:
    return torch.empty(_lib.workspace_bytes(), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------------------------------------
# flat codec
# ------------------------------------------------------------------------------------------------
def absmax(x: torch.Tensor, *, workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """torch.max(torch.abs(t)) (quant.py:100) on the device: fp32 tensor of shape [] (NaN propagates)."""
    require_quantizable(x)
    x = _dev(x, "x")
    ws = new_workspace(x.device) if workspace is None else workspace
    out = torch.empty((), dtype=torch.float32, device=x.device)
    lib, st = _lib.load(), _stream(x.device)
    check(lib.adfl_slq_absmax(x.data_ptr(), x.numel(), ws.data_ptr(), ws.numel(), st))
    check(lib.adfl_slq_absmax_value(ws.data_ptr(), out.data_ptr(), st))
    return out


def encode(x: torch.Tensor, bits: int, *, q: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None,
           workspace: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """quant.py:97-104 on the device: returns (int8 payload shaped like x, fp32 scale of shape [1])."""
    require_quantizable(x)
    x = _dev(x, "x")
    q = torch.empty(x.shape, dtype=torch.int8, device=x.device) if q is None else \
        _dst(q, x.numel(), torch.int8, x.device, "q")
    scale = _dst(scale, 1, torch.float32, x.device, "scale", align=4)
    ws = new_workspace(x.device) if workspace is None else workspace
    check(_lib.load().adfl_slq_encode(x.data_ptr(), x.numel(), bits, q.data_ptr(), scale.data_ptr(), ws.data_ptr(),
                                      ws.numel(), _stream(x.device)))
    return q, scale


def decode(q: torch.Tensor, scale: torch.Tensor, *, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """quant.py:110 ``q.dequantize()`` on the device: fp32(scale * q)."""
    q = _dev(q, "q")
    if q.dtype != torch.int8:
        raise TypeError(f"adfl_amd.ops.decode: payload must be int8, got {q.dtype}")
    out = torch.empty(q.shape, dtype=torch.float32, device=q.device) if out is None else \
        _dst(out, q.numel(), torch.float32, q.device, "out")
    scale = _f32_on(scale, 1, q.device, "scale")
    check(_lib.load().adfl_slq_dequantize(q.data_ptr(), q.numel(), scale.data_ptr(), out.data_ptr(),
                                          _stream(q.device)))
    return out


def encode_int4(x: torch.Tensor, bits: int = 4, *, packed: Optional[torch.Tensor] = None,
                scale: Optional[torch.Tensor] = None,
                workspace: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """SLQ encode fused with pack_4bit (compression.py:35-48): returns (uint8 [ceil(n/2)], fp32 [1])."""
    require_quantizable(x)
    x = _dev(x, "x")
    n = x.numel()
    packed = _dst(packed, (n + 1) // 2, torch.uint8, x.device, "packed")
    scale = _dst(scale, 1, torch.float32, x.device, "scale", align=4)
    ws = new_workspace(x.device) if workspace is None else workspace
    check(_lib.load().adfl_slq_encode_int4(x.data_ptr(), n, bits, packed.data_ptr(), scale.data_ptr(),
                                           ws.data_ptr(), ws.numel(), _stream(x.device)))
    return packed, scale


def decode_int4(packed: torch.Tensor, n: int, scale: torch.Tensor, *,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """unpack_4bit (compression.py:51-66) fused with dequantize: fp32 [n]."""
    packed = _dev(packed, "packed")
    if packed.numel() * packed.element_size() < (n + 1) // 2:
        raise ValueError(f"decode_int4: {n} elements need {(n + 1) // 2} packed bytes")
    out = _dst(out, n, torch.float32, packed.device, "out")
    scale = _f32_on(scale, 1, packed.device, "scale")
    check(_lib.load().adfl_slq_dequantize_int4(packed.data_ptr(), n, scale.data_ptr(), out.data_ptr(),
                                               _stream(packed.device)))
    return out


def pack_int4(q: torch.Tensor) -> torch.Tensor:
    """compression.py:35-48 ``pack_4bit`` on a device int8 tensor: uint8 [ceil(n/2)]."""
    q = _dev(q, "q")
    n = q.numel()
    packed = torch.empty((n + 1) // 2, dtype=torch.uint8, device=q.device)
    check(_lib.load().adfl_pack_int4(q.data_ptr(), n, packed.data_ptr(), _stream(q.device)))
    return packed


def unpack_int4(packed: torch.Tensor, shape: Sequence[int]) -> torch.Tensor:
    """compression.py:51-66 ``unpack_4bit`` on the device: int8 of `shape`."""
    packed = _dev(packed, "packed")
    n = int(np.prod(shape)) if len(shape) else 1
    q = torch.empty(tuple(shape), dtype=torch.int8, device=packed.device)
    check(_lib.load().adfl_unpack_int4(packed.data_ptr(), n, q.data_ptr(), _stream(packed.device)))
    return q


def dequantize_mean(q_rows: torch.Tensor, scales: torch.Tensor, n: int, *,
                    out: Optional[torch.Tensor] = None, self_row: int = -1,
                    self_x: Optional[torch.Tensor] = None, packed: bool = False) -> torch.Tensor:
    """Mean over K payload rows of one n-element tensor (Examples/ray_ad.py:188; simple_aggregate,
    Src/ADFL/model.py:221-234), summed in torch's CPU order (csrc/torch_sum_order.h), then / K: q_rows is
    [K, row_bytes] int8 (row_bytes >= n, a 16-byte multiple) — or, packed=True, uint8 int4-packed rows
    (row_bytes >= ceil(n/2), compression.py:35-48) — and scales is [K] or [K, stride] fp32 (column 0). With
    self_row >= 0 that row is replaced by the receiver's own fp32 update self_x, added last and exactly
    (async_peer.py:170-174)."""
    dt = torch.uint8 if packed else torch.int8
    if q_rows.dim() != 2 or q_rows.dtype != dt or not q_rows.is_contiguous() or not q_rows.is_cuda:
        raise ValueError(f"dequantize_mean: q_rows must be a contiguous [K, row_bytes] {dt} device tensor")
    k, row = q_rows.shape
    dev = q_rows.device
    if row < ((n + 1) // 2 if packed else n):
        raise ValueError("dequantize_mean: rows shorter than the tensor")
    sc = _scale_rows(scales, k, 1, dev, "scales")
    xp = None
    if self_row >= 0:
        self_x = _f32_on(self_x, n, dev, "self_x")
        if self_x.numel() != n:
            raise ValueError("dequantize_mean: self_x must be a contiguous fp32 tensor of n elements")
        xp = self_x.data_ptr()
    out = _dst(out, n, torch.float32, dev, "out")
    fn = _lib.load().adfl_slq_dequantize_mean_self_int4 if packed else _lib.load().adfl_slq_dequantize_mean_self
    check(fn(q_rows.data_ptr(), row, k, n, sc.data_ptr(), sc.stride(0), self_row, xp, out.data_ptr(), _stream(dev)))
    return out


# ------------------------------------------------------------------------------------------------
# bucketed codec (one launch per pass for a whole state dict)
# ------------------------------------------------------------------------------------------------
class BucketLayout:
    """Placement of T tensors in one flat buffer, plus the chunk table the bucketed kernels walk (one
    256-thread block per <= 8192-element chunk).

    align=64 (default) starts every tensor on a 64-element boundary (pads between tensors);
    align=1 packs them back to back (compact: what the Channel stages through host memory, so the
    host-side gather is one plain concatenation)."""

    def __init__(self, sizes: Sequence[int], align: int = ALIGN_ELEMS, offsets: Optional[Sequence[int]] = None):
        sizes = [int(s) for s in sizes]
        if not sizes or min(sizes) < 1:
            raise ValueError("BucketLayout: every tensor needs at least one element")
        if align < 1:
            raise ValueError("BucketLayout: align must be >= 1")
        self.sizes = np.asarray(sizes, dtype=np.int64)
        if offsets is None:
            self.align = align
            padded = (self.sizes + align - 1) // align * align
            self.padded = padded.astype(np.int64)  # per-tensor slot size (size rounded up to the alignment)
            self.offsets = np.concatenate([[0], np.cumsum(padded)[:-1]]).astype(np.int64)
            self.total = int(padded.sum())
        else:  # caller-placed tensors (the torch.ops.adfl batched ops): any order, no overlap
            self.offsets = np.asarray([int(o) for o in offsets], dtype=np.int64)
            if self.offsets.shape != self.sizes.shape or (self.offsets < 0).any():
                raise ValueError("BucketLayout: offsets must be one non-negative offset per tensor")
            order = np.argsort(self.offsets, kind="stable")
            ends = self.offsets[order] + self.sizes[order]
            if (self.offsets[order][1:] < ends[:-1]).any():
                raise ValueError("BucketLayout: tensors overlap")
            self.total = int(ends.max())
            self.padded = self.sizes.copy()
            nz = self.offsets[self.offsets > 0]
            self.align = int(np.gcd.reduce(nz)) if nz.size else ALIGN_ELEMS
        self.ntensors = len(sizes)
        lib = _lib.load()
        off_p, siz_p = self.offsets.ctypes.data, self.sizes.ctypes.data
        count = lib.adfl_slq_build_chunks(off_p, siz_p, self.ntensors, None, 0)
        if count < 0:
            check(int(count))
        self.chunks = (Chunk * count)()
        got = lib.adfl_slq_build_chunks(off_p, siz_p, self.ntensors, self.chunks, count)
        if got != count:
            check(int(got) if got < 0 else -1)
        self.nchunks = int(count)
        # the one-launch encode's work list (adfl_slq_build_encode_work): the first chunk of every tensor
        # when all of them fit one block's registers, else empty (the two-pass encode)
        nwork = lib.adfl_slq_build_encode_work(self.chunks, count, None, 0)
        if nwork < 0:
            raise ValueError(f"BucketLayout: encode work list failed ({nwork})")
        self.work = np.zeros(max(nwork, 1), dtype=np.int32)
        if nwork:
            lib.adfl_slq_build_encode_work(self.chunks, count, self.work.ctypes.data, nwork)
        self.nwork = int(nwork)
        self.max_tensor_chunks = int(max(c.nchunks for c in self.chunks))
        self._device_chunks = {}
        self._device_work = {}
        self._device_tfirst = {}

    def device_chunks(self, device: torch.device) -> torch.Tensor:
        key = (device.type, device.index)
        t = self._device_chunks.get(key)
        if t is None:
            host = torch.frombuffer(bytearray(bytes(self.chunks)), dtype=torch.uint8)
            t = host.to(device)
            self._device_chunks[key] = t
        return t

    def device_tfirst(self, device: torch.device) -> torch.Tensor:
        """Every tensor's first chunk (int32, one per tensor) on `device`: the short-tensor norm kernel's work
        list (adfl_torch_norms_work), cached like the chunk table."""
        key = (device.type, device.index)
        t = self._device_tfirst.get(key)
        if t is None:
            rec = np.frombuffer(bytes(self.chunks), dtype=np.dtype([("start", "<i8"), ("len", "<i4"), ("tensor", "<i4"),
                                                                    ("first_chunk", "<i4"), ("nchunks", "<i4")]))
            first = np.nonzero(rec["first_chunk"] == np.arange(self.nchunks))[0]
            tf = np.zeros(self.ntensors, dtype=np.int32)
            tf[rec["tensor"][first]] = first
            t = torch.from_numpy(tf).to(device)
            self._device_tfirst[key] = t
        return t

    def device_work(self, device: torch.device) -> torch.Tensor:
        key = (device.type, device.index)
        t = self._device_work.get(key)
        if t is None:
            t = torch.from_numpy(self.work).to(device)
            self._device_work[key] = t
        return t


# Bucketed SLQ encode: "resident" (one 1024-thread block per tensor; every tensor <= 8 chunks), "twopass"
# (absmax launch + quantize launch). "auto" (the product): resident when the layout allows it, else the two
# passes.
_ENCODE_MODES = ("auto", "resident", "twopass")


def _encode_mode() -> str:
    mode = os.environ.get("ADFL_SLQ_ENCODE", "auto")
    if mode not in _ENCODE_MODES:
        raise ValueError(f"ADFL_SLQ_ENCODE must be one of {_ENCODE_MODES}, got {mode!r}")
    return mode


def encode_batched(flat: torch.Tensor, layout: BucketLayout, bits: int, *, q: Optional[torch.Tensor] = None,
                   scales: Optional[torch.Tensor] = None,
                   partials: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Encode every tensor of a bucketed flat fp32 buffer with its own scale (quant.py:74-94)."""
    if flat.dtype != torch.float32:
        raise RuntimeError(f"Quantize only works on Float Tensor, got {_TORCH_TYPE_NAMES.get(flat.dtype, flat.dtype)}")
    flat = _dev(flat, "flat")
    if flat.numel() < layout.total:
        raise ValueError("encode_batched: flat buffer smaller than the layout")
    dev = flat.device
    q = _dst(q, layout.total, torch.int8, dev, "q")
    scales = _dst(scales, layout.ntensors, torch.float32, dev, "scales", align=4)
    partials = _dst(partials, layout.nchunks, torch.int32, dev, "partials", align=4)
    lib, st = _lib.load(), _stream(dev)
    nwork = 0 if _encode_mode() == "twopass" else layout.nwork
    check(lib.adfl_slq_encode_batched_work(flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                           layout.nchunks, layout.device_work(dev).data_ptr(),
                                           nwork, bits, q.data_ptr(),
                                           scales.data_ptr(), partials.data_ptr(), st))
    return q, scales


def decode_batched(q: torch.Tensor, scales: torch.Tensor, layout: BucketLayout, *,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decode a bucketed int8 payload with per-tensor scales (quant.py:67-71)."""
    q = _dev(q, "q")
    dev = q.device
    if q.numel() * q.element_size() < layout.total:
        raise ValueError("decode_batched: payload smaller than the layout")
    out = _dst(out, layout.total, torch.float32, dev, "out")
    scales = _f32_on(scales, layout.ntensors, dev, "scales")
    check(_lib.load().adfl_slq_dequantize_batched(q.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                  layout.nchunks, scales.data_ptr(), out.data_ptr(), _stream(dev)))
    return out


def qerror_batched(flat: torch.Tensor, q: torch.Tensor, scales: torch.Tensor,
                   layout: BucketLayout) -> Tuple[float, float, float, float]:
    """(sum (x-d)^2, sum x^2, sum x*d, sum d^2) over a bucket and its payload, d = fp32(scale*q), fp64
    sums (synchronises: returns Python floats)."""
    flat, q = _dev(flat, "flat"), _dev(q, "q")
    dev = flat.device
    scales = _f32_on(scales, layout.ntensors, dev, "scales")
    partials = torch.empty(layout.nchunks * 4, dtype=torch.float64, device=dev)
    check(_lib.load().adfl_slq_qerror_batched(flat.data_ptr(), q.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                              layout.nchunks, scales.data_ptr(), partials.data_ptr(),
                                              _stream(dev)))
    return tuple(partials.view(-1, 4).sum(0).tolist())


def qerror_batched_int4(flat: torch.Tensor, packed: torch.Tensor, scales: torch.Tensor,
                        layout: BucketLayout) -> Tuple[float, float, float, float]:
    """qerror_batched against an int4-packed bucket (layout offsets even; encode_batched_int4's payload)."""
    flat, packed = _dev(flat, "flat"), _dev(packed, "packed")
    if (layout.offsets % 2).any():
        raise ValueError("qerror_batched_int4: tensor offsets must be even (an int4 bucket layout)")
    dev = flat.device
    scales = _f32_on(scales, layout.ntensors, dev, "scales")
    partials = torch.empty(layout.nchunks * 4, dtype=torch.float64, device=dev)
    check(_lib.load().adfl_slq_qerror_batched_int4(flat.data_ptr(), packed.data_ptr(),
                                                   layout.device_chunks(dev).data_ptr(), layout.nchunks,
                                                   scales.data_ptr(), partials.data_ptr(), _stream(dev)))
    return tuple(partials.view(-1, 4).sum(0).tolist())


def _bucket_ptr_table(tensors, layout: BucketLayout, bucket: torch.Tensor, what: str, checked: bool,
                      ptrs: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Device int64 table of the tensors' data pointers, after checking them against the layout and bucket
    (checked=False: tensors the caller has just allocated to match, as the Channel's outputs are; ptrs: their
    pointers as a CPU int64 tensor when the caller already has them)."""
    dev = bucket.device
    if len(tensors) != layout.ntensors:
        raise ValueError(f"{what}: {len(tensors)} tensors for a layout of {layout.ntensors}")
    if ptrs is not None and not checked:
        return ptrs.to(dev, non_blocking=True)
    if checked:
        es = bucket.element_size()
        for t, (x, n) in enumerate(zip(tensors, layout.sizes.tolist())):
            if (not x.is_cuda or x.device != dev or not x.is_contiguous() or x.numel() != n
                    or x.element_size() != es):
                raise ValueError(f"{what}: tensor {t} must be a contiguous {es}-byte-element tensor of {n} "
                                 f"elements on {dev}")
    return torch.tensor([x.data_ptr() for x in tensors], dtype=torch.int64).to(dev, non_blocking=True)


def _check_bucket(bucket: torch.Tensor, layout: BucketLayout, what: str) -> torch.Tensor:
    bucket = _dev(bucket, "bucket")
    if not bucket.is_contiguous() or bucket.numel() < layout.total or bucket.element_size() not in (1, 2, 4, 8):
        raise ValueError(f"{what}: the bucket must be a contiguous device tensor of >= {layout.total} elements "
                         "of 1, 2, 4 or 8 bytes")
    return bucket


def bucket_gather(tensors, layout: BucketLayout, bucket: torch.Tensor, *, checked: bool = True,
                  ptrs: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Copy every tensor into its slot of the device bucket (tensor t at layout.offsets[t]), one launch
    (adfl_bucket_gather). Tensors: contiguous, on the bucket's device, of its element size (any dtype,
    quantized included); pads between slots are left as they are."""
    bucket = _check_bucket(bucket, layout, "bucket_gather")
    table = _bucket_ptr_table(tensors, layout, bucket, "bucket_gather", checked, ptrs)
    check(_lib.load().adfl_bucket_gather(bucket.data_ptr(), layout.device_chunks(bucket.device).data_ptr(),
                                         layout.nchunks, table.data_ptr(), bucket.element_size(),
                                         _stream(bucket.device)))
    return bucket


def bucket_scatter(bucket: torch.Tensor, layout: BucketLayout, tensors, *, checked: bool = True,
                   ptrs: Optional[torch.Tensor] = None) -> None:
    """Copy every slot of the device bucket into its own tensor (tensor t from layout.offsets[t]), one launch
    (adfl_bucket_scatter): the owned per-tensor outputs of a bucketed decode or encode."""
    bucket = _check_bucket(bucket, layout, "bucket_scatter")
    table = _bucket_ptr_table(tensors, layout, bucket, "bucket_scatter", checked, ptrs)
    check(_lib.load().adfl_bucket_scatter(bucket.data_ptr(), layout.device_chunks(bucket.device).data_ptr(),
                                          layout.nchunks, table.data_ptr(), bucket.element_size(),
                                          _stream(bucket.device)))


def dequantize_add_batched(q: torch.Tensor, scales: torch.Tensor, layout: BucketLayout, targets) -> None:
    """In place, for every model k and tensor t: targets[k][t] += fp32(scales[t] * q_t) (fp32 add) — decode
    once, accumulate into K device-resident models (Src/ADFL/Client/pool.py:62-75, model.py:337-347).

    targets: K sequences of T contiguous, 16-byte aligned fp32 device tensors, tensor t with
    layout.sizes[t] elements. Any layout: an aligned bucket's tensors take 16-byte accesses, a compact
    bucket's (offsets not multiples of 4) are decoded element-wise, with the same result."""
    q = _dev(q, "q")
    dev = q.device
    ptrs = []
    for k, model in enumerate(targets):
        if len(model) != layout.ntensors:
            raise ValueError(f"dequantize_add_batched: model {k} has {len(model)} tensors, layout {layout.ntensors}")
        for t, (x, n) in enumerate(zip(model, layout.sizes.tolist())):
            if (not x.is_cuda or x.device != dev or x.dtype != torch.float32 or not x.is_contiguous()
                    or x.numel() != n or x.data_ptr() % 16):
                raise ValueError(f"dequantize_add_batched: target {k}/{t} must be a contiguous, 16-byte aligned "
                                 f"fp32 tensor of {n} elements on {dev}")
            ptrs.append(x.data_ptr())
    table = torch.tensor(ptrs, dtype=torch.int64).to(dev, non_blocking=True)
    check(_lib.load().adfl_slq_dequantize_add_batched(q.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                      layout.nchunks, _f32_on(scales, layout.ntensors, dev, "scales").data_ptr(),
                                                      table.data_ptr(), layout.ntensors, len(targets),
                                                      _stream(dev)))
    # `table` may be freed on return: the caching allocator only reuses it for later work on this stream


def dequantize_mean_batched(q_rows: torch.Tensor, scales: torch.Tensor, layout: BucketLayout, *,
                            out: Optional[torch.Tensor] = None, self_row: int = -1,
                            self_x: Optional[torch.Tensor] = None, packed: bool = False) -> torch.Tensor:
    """Peer mean of K bucketed int8 payloads with per-tensor scales (SLQChannel's per-tensor codec over a
    whole state dict, averaged as Examples/ray_ad.py:164-190 averages every tensor). q_rows: [K, row_bytes]
    int8 (row_bytes >= layout.total, a 16-byte multiple), payload r in the layout; scales: [K, >= T] fp32
    (column t = tensor t). With self_row >= 0 that row is replaced by the receiver's own fp32 bucket self_x,
    added last and exactly (async_peer.py:170-174). packed=True: the rows are int4-packed bucket payloads
    (encode_batched_int4's: uint8, row_bytes >= ceil(layout.total / 2), even tensor offsets) -- the
    PackedSLQChannel exchange. Returns the flat fp32 bucket; positions outside every tensor are zero when
    `out` is None (left untouched otherwise)."""
    dt = torch.uint8 if packed else torch.int8
    if q_rows.dim() != 2 or q_rows.dtype != dt or not q_rows.is_contiguous() or not q_rows.is_cuda:
        raise ValueError(f"dequantize_mean_batched: q_rows must be a contiguous [K, row_bytes] {dt} device tensor")
    k, row = q_rows.shape
    if packed:
        _require_even_offsets(layout)
    if row < ((layout.total + 1) // 2 if packed else layout.total):
        raise ValueError("dequantize_mean_batched: rows shorter than the bucket layout")
    dev = q_rows.device
    sc = _scale_rows(scales, k, layout.ntensors, dev, "scales")
    xp = None
    if self_row >= 0:
        self_x = _f32_on(self_x, layout.total, dev, "self_x")
        xp = self_x.data_ptr()
    out = _dst(out, layout.total, torch.float32, dev, "out", zero=True)
    fn = _lib.load().adfl_slq_dequantize_mean_batched_int4 if packed else _lib.load().adfl_slq_dequantize_mean_batched
    check(fn(q_rows.data_ptr(), row, k, layout.device_chunks(dev).data_ptr(), layout.nchunks, sc.data_ptr(),
             sc.stride(0), self_row, xp, out.data_ptr(), _stream(dev)))
    return out


def _require_even_offsets(layout: BucketLayout) -> None:
    if layout.align % 2 or (layout.offsets % 2).any():
        raise ValueError("int4 buckets need even tensor offsets (BucketLayout(align=2) or a multiple of 2)")


def encode_batched_int4(flat: torch.Tensor, layout: BucketLayout, bits: int = 4, *,
                        packed: Optional[torch.Tensor] = None, scales: Optional[torch.Tensor] = None,
                        partials: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-tensor SLQ encode fused with pack_4bit over a bucket: packed byte e/2 holds flat elements
    e, e+1 (ceil(layout.total / 2) bytes); per-tensor fp32 scales."""
    if flat.dtype != torch.float32:
        raise RuntimeError(f"Quantize only works on Float Tensor, got {_TORCH_TYPE_NAMES.get(flat.dtype, flat.dtype)}")
    _require_even_offsets(layout)
    flat = _dev(flat, "flat")
    if flat.numel() < layout.total:
        raise ValueError("encode_batched_int4: flat buffer smaller than the layout")
    dev = flat.device
    packed = _dst(packed, (layout.total + 1) // 2, torch.uint8, dev, "packed")
    scales = _dst(scales, layout.ntensors, torch.float32, dev, "scales", align=4)
    partials = _dst(partials, layout.nchunks, torch.int32, dev, "partials", align=4)
    check(_lib.load().adfl_slq_encode_batched_int4_work(flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                        layout.nchunks, layout.device_work(dev).data_ptr(),
                                                        layout.nwork, bits, packed.data_ptr(), scales.data_ptr(),
                                                        partials.data_ptr(), _stream(dev)))
    return packed, scales


def decode_batched_int4(packed: torch.Tensor, scales: torch.Tensor, layout: BucketLayout, *,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """unpack_4bit + dequantize over a bucket (layout of encode_batched_int4)."""
    _require_even_offsets(layout)
    packed = _dev(packed, "packed")
    dev = packed.device
    if packed.numel() * packed.element_size() < (layout.total + 1) // 2:
        raise ValueError("decode_batched_int4: packed / scales / out smaller than the layout needs")
    out = _dst(out, layout.total, torch.float32, dev, "out")
    scales = _f32_on(scales, layout.ntensors, dev, "scales")
    check(_lib.load().adfl_slq_dequantize_batched_int4(packed.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                       layout.nchunks, scales.data_ptr(), out.data_ptr(),
                                                       _stream(dev)))
    return out


# ------------------------------------------------------------------------------------------------
# torch.ops.adfl.* custom ops (device tensors; fake impls for tracing / meta shapes)
# ------------------------------------------------------------------------------------------------
@torch.library.custom_op("adfl::slq_encode", mutates_args=())
def slq_encode_op(x: torch.Tensor, bits: int) -> Tuple[torch.Tensor, torch.Tensor]:
    return encode(x, bits)


@slq_encode_op.register_fake
def _(x, bits):
    return x.new_empty(x.shape, dtype=torch.int8), x.new_empty((1,), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_decode", mutates_args=())
def slq_decode_op(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return decode(q, scale)


@slq_decode_op.register_fake
def _(q, scale):
    return q.new_empty(q.shape, dtype=torch.float32)


@torch.library.custom_op("adfl::slq_encode_int4", mutates_args=())
def slq_encode_int4_op(x: torch.Tensor, bits: int) -> Tuple[torch.Tensor, torch.Tensor]:
    return encode_int4(x, bits)


@slq_encode_int4_op.register_fake
def _(x, bits):
    return x.new_empty(((x.numel() + 1) // 2,), dtype=torch.uint8), x.new_empty((1,), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_decode_int4", mutates_args=())
def slq_decode_int4_op(packed: torch.Tensor, n: int, scale: torch.Tensor) -> torch.Tensor:
    return decode_int4(packed, n, scale)


@slq_decode_int4_op.register_fake
def _(packed, n, scale):
    return packed.new_empty((n,), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_absmax", mutates_args=())
def slq_absmax_op(x: torch.Tensor) -> torch.Tensor:
    return absmax(x)


@slq_absmax_op.register_fake
def _(x):
    return x.new_empty((), dtype=torch.float32)


# Batched ops over caller-placed tensors: `offsets` / `sizes` are host (CPU) int64 tensors, tensor t owning
# flat[offsets[t] : offsets[t] + sizes[t]] (any order, no overlap; quant.py:74-94's loop over a state dict
# in one launch per pass). Outputs are shaped like the flat input; positions no tensor owns are zero.
_LAYOUT_CACHE: "dict" = {}
_LAYOUT_CACHE_MAX = 64


def layout_for(offsets: torch.Tensor, sizes: torch.Tensor) -> BucketLayout:
    """The BucketLayout (host chunk table + its device copies) for caller-placed tensors, cached by value so a
    repeated state-dict layout pays the table build and its H2D copy once."""
    if offsets.device.type != "cpu" or sizes.device.type != "cpu":
        raise ValueError("adfl batched ops: offsets and sizes must be host (CPU) int64 tensors")
    key = (tuple(offsets.tolist()), tuple(sizes.tolist()))
    lay = _LAYOUT_CACHE.pop(key, None)
    if lay is None:
        lay = BucketLayout(key[1], offsets=key[0])
    _LAYOUT_CACHE[key] = lay                       # most recently used last
    while len(_LAYOUT_CACHE) > _LAYOUT_CACHE_MAX:
        _LAYOUT_CACHE.pop(next(iter(_LAYOUT_CACHE)))
    return lay


def _filled(n: int, dtype, device, lay: BucketLayout) -> torch.Tensor:
    """Output buffer of n elements: zeros when some element belongs to no tensor (gaps, or a buffer longer
    than the layout), so the op's result is deterministic; otherwise left for the kernel to fill."""
    covered = int(lay.sizes.sum()) == n
    return (torch.empty if covered else torch.zeros)(n, dtype=dtype, device=device)


@torch.library.custom_op("adfl::slq_encode_batched", mutates_args=())
def slq_encode_batched_op(flat: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                          bits: int) -> Tuple[torch.Tensor, torch.Tensor]:
    lay = layout_for(offsets, sizes)
    flat = flat.reshape(-1)
    if flat.numel() < lay.total:
        raise ValueError("slq_encode_batched: flat buffer smaller than the layout")
    q = _filled(flat.numel(), torch.int8, flat.device, lay)
    return encode_batched(flat, lay, bits, q=q)


@slq_encode_batched_op.register_fake
def _(flat, offsets, sizes, bits):
    return flat.new_empty((flat.numel(),), dtype=torch.int8), flat.new_empty((sizes.numel(),), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_decode_batched", mutates_args=())
def slq_decode_batched_op(q: torch.Tensor, scales: torch.Tensor, offsets: torch.Tensor,
                          sizes: torch.Tensor) -> torch.Tensor:
    lay = layout_for(offsets, sizes)
    q = q.reshape(-1)
    if q.numel() < lay.total:
        raise ValueError("slq_decode_batched: payload smaller than the layout")
    return decode_batched(q, scales, lay, out=_filled(q.numel(), torch.float32, q.device, lay))


@slq_decode_batched_op.register_fake
def _(q, scales, offsets, sizes):
    return q.new_empty((q.numel(),), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_encode_batched_int4", mutates_args=())
def slq_encode_batched_int4_op(flat: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor,
                               bits: int) -> Tuple[torch.Tensor, torch.Tensor]:
    lay = layout_for(offsets, sizes)
    flat = flat.reshape(-1)
    if flat.numel() < lay.total:
        raise ValueError("slq_encode_batched_int4: flat buffer smaller than the layout")
    nbytes = (flat.numel() + 1) // 2
    gap = int(lay.sizes.sum()) != flat.numel()
    packed = (torch.zeros if gap else torch.empty)(nbytes, dtype=torch.uint8, device=flat.device)
    return encode_batched_int4(flat, lay, bits, packed=packed)


@slq_encode_batched_int4_op.register_fake
def _(flat, offsets, sizes, bits):
    return (flat.new_empty(((flat.numel() + 1) // 2,), dtype=torch.uint8),
            flat.new_empty((sizes.numel(),), dtype=torch.float32))


@torch.library.custom_op("adfl::slq_decode_batched_int4", mutates_args=())
def slq_decode_batched_int4_op(packed: torch.Tensor, scales: torch.Tensor, offsets: torch.Tensor,
                               sizes: torch.Tensor, n: int) -> torch.Tensor:
    lay = layout_for(offsets, sizes)
    if n < lay.total or packed.numel() < (lay.total + 1) // 2:
        raise ValueError("slq_decode_batched_int4: n / packed smaller than the layout")
    gap = int(lay.sizes.sum()) != n
    out = (torch.zeros if gap else torch.empty)(n, dtype=torch.float32, device=packed.device)
    return decode_batched_int4(packed.reshape(-1), scales, lay, out=out)


@slq_decode_batched_int4_op.register_fake
def _(packed, scales, offsets, sizes, n):
    return packed.new_empty((n,), dtype=torch.float32)


@torch.library.custom_op("adfl::pack_int4", mutates_args=())
def pack_int4_op(q: torch.Tensor) -> torch.Tensor:
    return pack_int4(q)


@pack_int4_op.register_fake
def _(q):
    return q.new_empty(((q.numel() + 1) // 2,), dtype=torch.uint8)


@torch.library.custom_op("adfl::unpack_int4", mutates_args=())
def unpack_int4_op(packed: torch.Tensor, shape: List[int]) -> torch.Tensor:
    return unpack_int4(packed, shape)


@unpack_int4_op.register_fake
def _(packed, shape):
    return packed.new_empty(tuple(shape), dtype=torch.int8)


@torch.library.custom_op("adfl::slq_dequantize_mean", mutates_args=())
def slq_dequantize_mean_op(q_rows: torch.Tensor, scales: torch.Tensor, n: int, self_row: int = -1,
                           self_x: Optional[torch.Tensor] = None) -> torch.Tensor:
    return dequantize_mean(q_rows, scales, n, self_row=self_row, self_x=self_x)


@slq_dequantize_mean_op.register_fake
def _(q_rows, scales, n, self_row=-1, self_x=None):
    return q_rows.new_empty((n,), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_dequantize_mean_batched", mutates_args=())
def slq_dequantize_mean_batched_op(q_rows: torch.Tensor, scales: torch.Tensor, offsets: torch.Tensor,
                                   sizes: torch.Tensor, n: int, self_row: int = -1,
                                   self_x: Optional[torch.Tensor] = None) -> torch.Tensor:
    lay = layout_for(offsets, sizes)
    if n < lay.total:
        raise ValueError("slq_dequantize_mean_batched: n smaller than the layout")
    out = torch.zeros(n, dtype=torch.float32, device=q_rows.device)
    return dequantize_mean_batched(q_rows, scales, lay, out=out, self_row=self_row, self_x=self_x)


@slq_dequantize_mean_batched_op.register_fake
def _(q_rows, scales, offsets, sizes, n, self_row=-1, self_x=None):
    return q_rows.new_empty((n,), dtype=torch.float32)


@torch.library.custom_op("adfl::slq_dequantize_mean_batched_int4", mutates_args=())
def slq_dequantize_mean_batched_int4_op(packed_rows: torch.Tensor, scales: torch.Tensor, offsets: torch.Tensor,
                                        sizes: torch.Tensor, n: int, self_row: int = -1,
                                        self_x: Optional[torch.Tensor] = None) -> torch.Tensor:
    """slq_dequantize_mean_batched over int4-packed rows (uint8 [K, row_bytes], even offsets)."""
    lay = layout_for(offsets, sizes)
    if n < lay.total:
        raise ValueError("slq_dequantize_mean_batched_int4: n smaller than the layout")
    out = torch.zeros(n, dtype=torch.float32, device=packed_rows.device)
    return dequantize_mean_batched(packed_rows, scales, lay, out=out, self_row=self_row, self_x=self_x, packed=True)


@slq_dequantize_mean_batched_int4_op.register_fake
def _(packed_rows, scales, offsets, sizes, n, self_row=-1, self_x=None):
    return packed_rows.new_empty((n,), dtype=torch.float32)
