"""Device-resident stochastic codec ops (QSGD / RQSGD / CNAT) over the HIP C ABI (include/adfl_stoch.h).

Every function takes and returns CUDA (HIP) tensors over a bucketed flat buffer described by an
``ops.BucketLayout``, launches on the current stream and never synchronises:

* ``qsgd_encode_batched`` / ``qsgd_decode_batched``   — QSGDChannel._quantize_tensor / _dequantize_tensor
  (Src/ADFL/Channel/quant.py:223-252)
* ``rqsgd_encode_batched`` / ``rqsgd_decode_batched`` — RQSGDChannel (quant.py:364-398)
* ``cnat_encode_batched`` / ``cnat_decode_batched``   — CNATChannel (quant.py:509-545)
* ``norms_batched`` — per-tensor ||x||_2 or (max|x|, min|x|); ``qsgd_quantize_batched`` — levels from
  given norms (what the parity tests use to inject the reference's own norm)

Randomness: pass ``uniforms`` (fp32 plane indexed like x, values in [0, 1)) to inject the reference's
``torch.rand_like`` draws, or leave it None to draw from the Philox4x32-7 stream ``(seed, counter)``.
``RngStream`` hands out (seed, counter) pairs seeded from torch's default CPU generator, so
``torch.manual_seed`` makes a run reproducible the way it does for the reference.
"""

import os
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import (CODEC_CNAT, CODEC_QSGD, CODEC_RQSGD, DTYPE_BF16, DTYPE_F16, DTYPE_F32, DTYPE_F64, NORM_L2, NORM_L2_TORCH,
                   NORM_LINF, check)
from .ops import BucketLayout, _dev, _stream

__all__ = ["RngStream", "norms_batched", "qsgd_quantize_batched", "qsgd_encode_batched", "rqsgd_encode_batched",
           "qsgd_decode_batched", "rqsgd_decode_batched", "cnat_encode_batched", "cnat_decode_batched",
           "philox_uniforms", "workspace", "torch_norms", "NORM_L2", "NORM_LINF", "NORM_L2_TORCH", "DT_DTYPES", "encode_batched_dt",
           "quantize_batched_dt", "norms_batched_dt", "philox_uniforms_dt", "dequantize_mean_batched"]


class RngStream:
    """(seed, counter) pairs for successive encode calls. The seed is drawn from torch's default CPU
    generator at construction (the generator the reference's torch.rand_like consumes); each call
    advances the counter past the uniforms it used, so no two calls share a uniform."""

    def __init__(self, seed: Optional[int] = None):
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
        self.seed = int(seed) & (2 ** 64 - 1)
        self.counter = 0

    def take(self, numel: int) -> Tuple[int, int]:
        c = self.counter
        self.counter += (int(numel) + 3) // 4
        return self.seed, c


def workspace(layout: BucketLayout, device) -> torch.Tensor:
    return torch.empty(int(_lib.load().adfl_stoch_workspace_bytes(layout.nchunks)), dtype=torch.uint8, device=device)


def _check_flat(flat: torch.Tensor, layout: BucketLayout) -> torch.Tensor:
    if flat.dtype != torch.float32:
        raise ValueError(f"adfl_amd.stoch: the HIP stochastic codecs take fp32 buckets, got {flat.dtype}")
    flat = _dev(flat, "flat")
    if flat.numel() < layout.total:
        raise ValueError("adfl_amd.stoch: flat buffer smaller than the layout")
    return flat


def _uniforms(u: Optional[torch.Tensor], layout: BucketLayout) -> int:
    if u is None:
        return 0
    if u.dtype != torch.float32 or u.numel() < layout.total:
        raise ValueError("adfl_amd.stoch: uniforms must be an fp32 plane covering the layout")
    if not u.is_cuda or not u.is_contiguous() or u.data_ptr() % 16:
        raise ValueError("adfl_amd.stoch: uniforms must be a contiguous, 16-byte aligned device tensor")
    return u.data_ptr()


def _ws(ws: Optional[torch.Tensor], layout: BucketLayout, dev) -> torch.Tensor:
    return workspace(layout, dev) if ws is None else ws


def _work(layout: BucketLayout, dev, resident: Optional[bool] = None):
    """(work list pointer, count) for the *_encode_batched_work entries: the one-launch register-resident
    encode when every tensor of the layout fits a block (layout.nwork > 0), else (any, 0) = multi-launch.
    ADFL_STOCH_RESIDENT=0 in the environment forces the multi-launch path (A/B runs)."""
    if resident is None:
        resident = os.environ.get("ADFL_STOCH_RESIDENT", "1") != "0"
    if not resident or layout.nwork == 0:
        return 0, 0
    return layout.device_work(dev).data_ptr(), layout.nwork


def norms_batched(flat: torch.Tensor, layout: BucketLayout, mode: int = NORM_L2, *,
                  norms: Optional[torch.Tensor] = None, mins: Optional[torch.Tensor] = None,
                  ws: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Per-tensor ||x||_2 (mode NORM_L2: fp64 accumulation, correctly rounded; NORM_L2_TORCH: torch's own
    fp32 reduction order, bit-identical to the reference's norm, sequential per tensor) or
    (max|x|, min|x|) (NORM_LINF)."""
    flat = _check_flat(flat, layout)
    dev = flat.device
    norms = torch.empty(layout.ntensors, dtype=torch.float32, device=dev) if norms is None else norms
    if mode == NORM_LINF and mins is None:
        mins = torch.empty(layout.ntensors, dtype=torch.float32, device=dev)
    ws = _ws(ws, layout, dev)
    check(_lib.load().adfl_stoch_norms_batched(flat.data_ptr(), layout.device_chunks(dev).data_ptr(), layout.nchunks,
                                               mode, ws.data_ptr(), ws.numel(), norms.data_ptr(),
                                               mins.data_ptr() if mins is not None else None, _stream(dev)))
    return norms, mins


def torch_norms(flat: torch.Tensor, layout: BucketLayout, *, norms: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-tensor ||x||_2 of an fp32 bucket bit-identical to torch's CPU vector_norm (the reference's QSGD /
    CNAT norm, quant.py:226,512): reference_norms' fp32 output. Same bits as norms_batched(...,
    NORM_L2_TORCH), the in-order kernel."""
    flat = _check_flat(flat, layout)
    norms = torch.empty(layout.ntensors, dtype=torch.float32, device=flat.device) if norms is None else norms
    reference_norms(flat, layout, out32=_dev(norms, "norms"))
    return norms


_REF_NORM_DTYPES = {torch.float32: DTYPE_F32, torch.float16: DTYPE_F16, torch.bfloat16: DTYPE_BF16,
                    torch.float64: DTYPE_F64}


def reference_norms(flat: torch.Tensor, layout: BucketLayout, *, threads: Optional[int] = None,
                    out64: Optional[torch.Tensor] = None, out32: Optional[torch.Tensor] = None):
    """Per-tensor ``torch.linalg.vector_norm(x, ord=2)`` of an fp32 / fp16 / bf16 / fp64 bucket, bit-identical
    to torch 2.10's CPU kernel — the reference's QSGD / CNAT norm in the tensor's own dtype (quant.py:226,512)
    — by adfl_torch_norms (csrc/torch_norm.hip: phases with no cross-block waits).

    threads: the torch.get_num_threads() whose fp16 split is reproduced (default: this process's, which is
    what the reference's own call would use). Returns (out64, out32): fp64 norms (the dtype's exact value)
    and fp32 ones; pass either to fill it (the other stays None unless passed too); with neither, out64 is
    allocated."""
    if flat.dtype not in _REF_NORM_DTYPES:
        raise ValueError(f"adfl_amd.stoch: reference_norms takes fp32 / fp16 / bf16 / fp64 buckets, got {flat.dtype}")
    flat = _dev(flat, "flat")
    if flat.numel() < layout.total:
        raise ValueError("adfl_amd.stoch: flat buffer smaller than the layout")
    dev = flat.device
    if out64 is None and out32 is None:
        out64 = torch.empty(layout.ntensors, dtype=torch.float64, device=dev)
    for o, dt in ((out64, torch.float64), (out32, torch.float32)):
        if o is not None and (o.dtype != dt or o.numel() < layout.ntensors or not o.is_contiguous() or o.device != dev):
            raise ValueError(f"adfl_amd.stoch: norm outputs must be contiguous {dt} device tensors of >= ntensors")
    if layout.nchunks == 0:
        return out64, out32
    L = _lib.load()
    threads = torch.get_num_threads() if threads is None else int(threads)
    if flat.dtype == torch.float16:   # at::parallel_for splits a tensor into at most ceil(n / GRAIN) pieces
        threads = min(threads, max(1, -(-int(max(layout.sizes)) // 32768)))
    elif threads < 1:
        raise ValueError("adfl_amd.stoch: threads must be >= 1")
    short_max = L.adfl_torch_norm_short_max_dt(_REF_NORM_DTYPES[flat.dtype])
    kinds = (1 if min(layout.sizes) <= short_max else 0) | (2 if max(layout.sizes) > short_max else 0)
    need = L.adfl_torch_norm_scratch_bytes(layout.nchunks, layout.ntensors)
    scratch = torch.empty(need, dtype=torch.uint8, device=dev)  # stream-ordered: no initialisation needed
    check(L.adfl_torch_norms_work(_REF_NORM_DTYPES[flat.dtype], flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                  layout.nchunks, layout.device_tfirst(dev).data_ptr(), layout.ntensors, kinds, threads,
                                  scratch.data_ptr(), need, out64.data_ptr() if out64 is not None else None,
                                  out32.data_ptr() if out32 is not None else None, _stream(dev)))
    return out64, out32


def _planes(layout, dev, levels, signs, ldtype):
    levels = torch.empty(layout.total, dtype=ldtype, device=dev) if levels is None else levels
    signs = torch.empty(layout.total, dtype=torch.int8, device=dev) if signs is None else signs
    return levels, signs


def qsgd_quantize_batched(flat: torch.Tensor, layout: BucketLayout, bits: int, norms: torch.Tensor, *,
                          uniforms: Optional[torch.Tensor] = None, seed: int = 0, counter: int = 0,
                          levels: Optional[torch.Tensor] = None,
                          signs: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Levels + signs from given per-tensor norms (QSGD: L2 norms; RQSGD: max|x|)."""
    flat = _check_flat(flat, layout)
    dev = flat.device
    levels, signs = _planes(layout, dev, levels, signs, torch.uint8)
    check(_lib.load().adfl_qsgd_quantize_batched(flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                 layout.nchunks, bits, _dev(norms, "norms").data_ptr(),
                                                 _uniforms(uniforms, layout), seed, counter, levels.data_ptr(),
                                                 signs.data_ptr(), _stream(dev)))
    return levels, signs


def qsgd_encode_batched(flat: torch.Tensor, layout: BucketLayout, bits: int, *,
                        uniforms: Optional[torch.Tensor] = None, seed: int = 0, counter: int = 0,
                        levels: Optional[torch.Tensor] = None, signs: Optional[torch.Tensor] = None,
                        norms: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
                        torch_norm: bool = False, resident: Optional[bool] = None):
    """QSGD encode of every tensor of a bucket: (levels u8, signs i8, L2 norms f32). torch_norm=True takes
    the norm in torch's reduction order (the reference's norm bit for bit: reference_norms, then the
    given-norm quantize); False, the one-launch encode's correctly rounded norm.
    resident: None = the one-launch register-resident encode whenever the layout allows it (same bytes as
    the multi-launch path), False = always the multi-launch path."""
    flat = _check_flat(flat, layout)
    dev = flat.device
    levels, signs = _planes(layout, dev, levels, signs, torch.uint8)
    norms = torch.empty(layout.ntensors, dtype=torch.float32, device=dev) if norms is None else norms
    ws = _ws(ws, layout, dev)
    if torch_norm:
        reference_norms(flat, layout, out32=norms)
        qsgd_quantize_batched(flat, layout, bits, norms, uniforms=uniforms, seed=seed, counter=counter,
                              levels=levels, signs=signs)
        return levels, signs, norms
    check(_lib.load().adfl_qsgd_encode_batched_work(flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                    layout.nchunks, *_work(layout, dev, resident), bits,
                                                    _uniforms(uniforms, layout), seed, counter, ws.data_ptr(),
                                                    ws.numel(), levels.data_ptr(), signs.data_ptr(), norms.data_ptr(),
                                                    _stream(dev)))
    return levels, signs, norms


def rqsgd_encode_batched(flat: torch.Tensor, layout: BucketLayout, bits: int, *,
                         uniforms: Optional[torch.Tensor] = None, seed: int = 0, counter: int = 0,
                         levels: Optional[torch.Tensor] = None, signs: Optional[torch.Tensor] = None,
                         norms: Optional[torch.Tensor] = None, mins: Optional[torch.Tensor] = None,
                         ws: Optional[torch.Tensor] = None, resident: Optional[bool] = None):
    """RQSGD encode: (levels u8, signs i8, max|x| norms f32, min|x| factors f32). resident as for QSGD."""
    flat = _check_flat(flat, layout)
    dev = flat.device
    levels, signs = _planes(layout, dev, levels, signs, torch.uint8)
    norms = torch.empty(layout.ntensors, dtype=torch.float32, device=dev) if norms is None else norms
    mins = torch.empty(layout.ntensors, dtype=torch.float32, device=dev) if mins is None else mins
    ws = _ws(ws, layout, dev)
    check(_lib.load().adfl_rqsgd_encode_batched_work(flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                     layout.nchunks, *_work(layout, dev, resident), bits,
                                                     _uniforms(uniforms, layout), seed, counter, ws.data_ptr(),
                                                     ws.numel(), levels.data_ptr(), signs.data_ptr(),
                                                     norms.data_ptr(), mins.data_ptr(), _stream(dev)))
    return levels, signs, norms, mins


def qsgd_decode_batched(levels: torch.Tensor, signs: torch.Tensor, norms: torch.Tensor, layout: BucketLayout,
                        bits: int, *, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    levels, signs = _dev(levels, "levels"), _dev(signs, "signs")
    dev = levels.device
    out = torch.empty(layout.total, dtype=torch.float32, device=dev) if out is None else out
    check(_lib.load().adfl_qsgd_dequantize_batched(levels.data_ptr(), signs.data_ptr(),
                                                   layout.device_chunks(dev).data_ptr(), layout.nchunks, bits,
                                                   _dev(norms, "norms").data_ptr(), out.data_ptr(), _stream(dev)))
    return out


def rqsgd_decode_batched(levels: torch.Tensor, signs: torch.Tensor, norms: torch.Tensor, mins: torch.Tensor,
                         layout: BucketLayout, bits: int, *, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    levels, signs = _dev(levels, "levels"), _dev(signs, "signs")
    dev = levels.device
    out = torch.empty(layout.total, dtype=torch.float32, device=dev) if out is None else out
    check(_lib.load().adfl_rqsgd_dequantize_batched(levels.data_ptr(), signs.data_ptr(),
                                                    layout.device_chunks(dev).data_ptr(), layout.nchunks, bits,
                                                    _dev(norms, "norms").data_ptr(), _dev(mins, "mins").data_ptr(),
                                                    out.data_ptr(), _stream(dev)))
    return out


def cnat_encode_batched(flat: torch.Tensor, layout: BucketLayout, bits: int, *,
                        uniforms: Optional[torch.Tensor] = None, seed: int = 0, counter: int = 0,
                        exps: Optional[torch.Tensor] = None, signs: Optional[torch.Tensor] = None,
                        norms: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
                        torch_norm: bool = False, resident: Optional[bool] = None):
    """CNAT encode (x read once; resident as for QSGD): (exponents i8, signs i8, L2 norms f32). A tensor
    whose norm is 0 gets the reference's zero-branch bytes (0 / 1). torch_norm=True then replaces the norms
    with torch's own (the exponents do not depend on the norm; both norms are 0 for exactly the same tensors)."""
    flat = _check_flat(flat, layout)
    dev = flat.device
    exps, signs = _planes(layout, dev, exps, signs, torch.int8)
    norms = torch.empty(layout.ntensors, dtype=torch.float32, device=dev) if norms is None else norms
    ws = _ws(ws, layout, dev)
    check(_lib.load().adfl_cnat_encode_batched_work(flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                    layout.nchunks, *_work(layout, dev, resident), bits,
                                                    _uniforms(uniforms, layout), seed, counter, ws.data_ptr(),
                                                    ws.numel(), exps.data_ptr(), signs.data_ptr(), norms.data_ptr(),
                                                    _stream(dev)))
    if torch_norm:
        reference_norms(flat, layout, out32=norms)
    return exps, signs, norms


def cnat_decode_batched(exps: torch.Tensor, signs: torch.Tensor, norms: torch.Tensor, layout: BucketLayout, *,
                        out: Optional[torch.Tensor] = None) -> torch.Tensor:
    exps, signs = _dev(exps, "exps"), _dev(signs, "signs")
    dev = exps.device
    out = torch.empty(layout.total, dtype=torch.float32, device=dev) if out is None else out
    check(_lib.load().adfl_cnat_dequantize_batched(exps.data_ptr(), signs.data_ptr(),
                                                   layout.device_chunks(dev).data_ptr(), layout.nchunks,
                                                   _dev(norms, "norms").data_ptr(), out.data_ptr(), _stream(dev)))
    return out


def philox_uniforms(n: int, seed: int, counter: int, start: int = 0, *, device=None) -> torch.Tensor:
    """The uniforms elements start .. start+n-1 of stream (seed, counter) draw."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    check(_lib.load().adfl_philox_uniforms(out.data_ptr(), n, start, seed & (2 ** 64 - 1), counter, _stream(dev)))
    return out


# ------------------------------------------------------------------------------------------------
def dequantize_mean_batched(codec: str, levels: torch.Tensor, signs: torch.Tensor, norms: torch.Tensor,
                            layout: BucketLayout, bits: int, *, mins: Optional[torch.Tensor] = None,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """simple_aggregate of K clients' decodes in one launch (adfl_stoch_dequantize_mean_batched): levels /
    signs are [K, row] byte planes (uint8 / int8; row >= layout.total, a multiple of 16), norms (RQSGD: mins)
    [K, ntensors] fp32. Returns the fp32 mean bucket."""
    if codec not in _CODEC_IDS:
        raise ValueError(f"adfl_amd.stoch: codec must be one of {sorted(_CODEC_IDS)}, got {codec!r}")
    levels, signs, norms = _dev(levels, "levels"), _dev(signs, "signs"), _dev(norms, "norms")
    if levels.dim() != 2 or signs.shape != levels.shape or levels.element_size() != 1 or signs.element_size() != 1:
        raise ValueError("adfl_amd.stoch: levels / signs must be [K, row] byte planes of one shape")
    k, row = levels.shape
    if row < layout.total or not levels.is_contiguous() or not signs.is_contiguous():
        raise ValueError(f"adfl_amd.stoch: rows of {row} bytes cannot hold the {layout.total}-element bucket")
    if norms.shape != (k, layout.ntensors) or norms.dtype != torch.float32 or not norms.is_contiguous():
        raise ValueError(f"adfl_amd.stoch: norms must be contiguous fp32 [{k}, {layout.ntensors}]")
    if codec == "rqsgd":
        if mins is None:
            raise ValueError("adfl_amd.stoch: RQSGD needs mins")
        mins = _dev(mins, "mins")
        if mins.shape != norms.shape or mins.dtype != torch.float32 or not mins.is_contiguous():
            raise ValueError("adfl_amd.stoch: mins must match norms")
    dev = levels.device
    out = torch.empty(layout.total, dtype=torch.float32, device=dev) if out is None else out
    if out.dtype != torch.float32 or out.numel() < layout.total or not out.is_contiguous() or out.device != dev:
        raise ValueError(f"adfl_amd.stoch: out must be a contiguous fp32 device tensor of >= {layout.total}")
    check(_lib.load().adfl_stoch_dequantize_mean_batched(
        _CODEC_IDS[codec], levels.data_ptr(), signs.data_ptr(), row, k, layout.device_chunks(dev).data_ptr(),
        layout.nchunks, bits, norms.data_ptr(), mins.data_ptr() if mins is not None else None, layout.ntensors,
        out.data_ptr(), _stream(dev)))
    return out


# fp16 / bf16 / fp64 buckets (include/adfl_stoch.h *_dt): the reference's arithmetic in the tensor's dtype
# ------------------------------------------------------------------------------------------------
DT_DTYPES = {torch.float16: DTYPE_F16, torch.bfloat16: DTYPE_BF16, torch.float64: DTYPE_F64}
_CODEC_IDS = {"qsgd": CODEC_QSGD, "rqsgd": CODEC_RQSGD, "cnat": CODEC_CNAT}


def _check_flat_dt(flat: torch.Tensor, layout: BucketLayout) -> Tuple[torch.Tensor, int]:
    if flat.dtype not in DT_DTYPES:
        raise ValueError(f"adfl_amd.stoch: the *_dt codecs take fp16 / bf16 / fp64 buckets, got {flat.dtype}")
    flat = _dev(flat, "flat")
    if flat.numel() < layout.total:
        raise ValueError("adfl_amd.stoch: flat buffer smaller than the layout")
    return flat, DT_DTYPES[flat.dtype]


def _uniforms_dt(u: Optional[torch.Tensor], layout: BucketLayout, dtype: torch.dtype) -> int:
    if u is None:
        return 0
    if u.dtype != dtype or u.numel() < layout.total:
        raise ValueError(f"adfl_amd.stoch: uniforms must be a {dtype} plane covering the layout")
    if not u.is_cuda or not u.is_contiguous() or u.data_ptr() % 16:
        raise ValueError("adfl_amd.stoch: uniforms must be a contiguous, 16-byte aligned device tensor")
    return u.data_ptr()


def norms_batched_dt(flat: torch.Tensor, layout: BucketLayout, mode: int = NORM_L2, *,
                     ws: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Per-tensor norms of an fp16 / bf16 / fp64 bucket as fp64 values of the dtype's norm: L2 (fp16 / bf16:
    fp32 squares summed in fp64, rounded to fp32, sqrt, rounded to the dtype; fp64: fp64 sum) or
    (max|x|, min|x|) with mode NORM_LINF."""
    flat, dt = _check_flat_dt(flat, layout)
    dev = flat.device
    norms = torch.empty(layout.ntensors, dtype=torch.float64, device=dev)
    mins = torch.empty(layout.ntensors, dtype=torch.float64, device=dev) if mode == NORM_LINF else None
    ws = _ws(ws, layout, dev)
    check(_lib.load().adfl_stoch_norms_batched_dt(dt, flat.data_ptr(), layout.device_chunks(dev).data_ptr(),
                                                  layout.nchunks, mode, ws.data_ptr(), ws.numel(), norms.data_ptr(),
                                                  mins.data_ptr() if mins is not None else None, _stream(dev)))
    return norms, mins


def quantize_batched_dt(codec: str, flat: torch.Tensor, layout: BucketLayout, bits: int, norms: torch.Tensor, *,
                        uniforms: Optional[torch.Tensor] = None, seed: int = 0, counter: int = 0,
                        levels: Optional[torch.Tensor] = None,
                        signs: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Levels (QSGD / RQSGD; uint8) or exponents (CNAT; int8) + signs of an fp16 / bf16 / fp64 bucket from
    given fp64 per-tensor norms (the parity tests inject the reference's)."""
    flat, dt = _check_flat_dt(flat, layout)
    dev = flat.device
    levels, signs = _planes(layout, dev, levels, signs, torch.int8 if codec == "cnat" else torch.uint8)
    norms = _dev(norms, "norms")
    if norms.dtype != torch.float64 or norms.numel() < layout.ntensors:
        raise ValueError("adfl_amd.stoch: norms must be fp64, one per tensor")
    check(_lib.load().adfl_stoch_quantize_batched_dt(_CODEC_IDS[codec], dt, flat.data_ptr(),
                                                     layout.device_chunks(dev).data_ptr(), layout.nchunks, bits,
                                                     norms.data_ptr(), _uniforms_dt(uniforms, layout, flat.dtype),
                                                     seed, counter, levels.data_ptr(), signs.data_ptr(), _stream(dev)))
    return levels, signs


def encode_batched_dt(codec: str, flat: torch.Tensor, layout: BucketLayout, bits: int, *,
                      uniforms: Optional[torch.Tensor] = None, seed: int = 0, counter: int = 0,
                      levels: Optional[torch.Tensor] = None, signs: Optional[torch.Tensor] = None,
                      ws: Optional[torch.Tensor] = None):
    """QSGD / RQSGD / CNAT encode of an fp16 / bf16 / fp64 bucket in the dtype's arithmetic
    (quant.py:223-240, :364-382, :509-534): (levels, signs, norms f64, mins f64 or None)."""
    flat, dt = _check_flat_dt(flat, layout)
    dev = flat.device
    levels, signs = _planes(layout, dev, levels, signs, torch.int8 if codec == "cnat" else torch.uint8)
    norms = torch.empty(layout.ntensors, dtype=torch.float64, device=dev)
    mins = torch.empty(layout.ntensors, dtype=torch.float64, device=dev) if codec == "rqsgd" else None
    ws = _ws(ws, layout, dev)
    check(_lib.load().adfl_stoch_encode_batched_dt(_CODEC_IDS[codec], dt, flat.data_ptr(),
                                                   layout.device_chunks(dev).data_ptr(), layout.nchunks, bits,
                                                   _uniforms_dt(uniforms, layout, flat.dtype), seed, counter,
                                                   ws.data_ptr(), ws.numel(), levels.data_ptr(), signs.data_ptr(),
                                                   norms.data_ptr(), mins.data_ptr() if mins is not None else None,
                                                   _stream(dev)))
    return levels, signs, norms, mins


def philox_uniforms_dt(dtype: torch.dtype, n: int, seed: int, counter: int, start: int = 0, *,
                       device=None) -> torch.Tensor:
    """The uniforms (in `dtype`) elements start .. start+n-1 of stream (seed, counter) draw."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    out = torch.empty(n, dtype=dtype, device=dev)
    check(_lib.load().adfl_philox_uniforms_dt(DT_DTYPES[dtype], out.data_ptr(), n, start, seed & (2 ** 64 - 1),
                                              counter, _stream(dev)))
    return out


# ------------------------------------------------------------------------------------------------
# torch.ops.adfl stochastic ops over caller-placed tensors (offsets / sizes: host int64, as the SLQ batched
# ops take them, ops.layout_for): QSGDChannel / RQSGDChannel / CNATChannel's per-tensor loops
# (quant.py:223-252, :364-398, :509-545) as traceable ops. Positions no tensor owns are zero.
# ------------------------------------------------------------------------------------------------
def _check_codec(codec: str) -> None:
    if codec not in _CODEC_IDS:
        raise ValueError(f"adfl stochastic ops: codec must be one of {sorted(_CODEC_IDS)}, got {codec!r}")


@torch.library.custom_op("adfl::stoch_encode_batched", mutates_args=())
def stoch_encode_batched_op(flat: torch.Tensor, offsets: torch.Tensor, sizes: torch.Tensor, codec: str, bits: int,
                            seed: int, counter: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """(levels — uint8, CNAT: int8 exponents —, signs int8, norms f32, mins f32 — RQSGD's min|x|, else 0) of
    a flat buffer; uniforms from the Philox stream (seed, counter). fp32 buffers take the fp32 kernels;
    fp16 / bf16 / fp64 ones are encoded in their own dtype's arithmetic, as the reference computes them
    (encode_batched_dt), and their norms / mins come back as the fp32 values the decode multiplies by (the
    channels' Python-float norm as an fp32 scalar; exact for fp16 / bf16 norms)."""
    from .ops import _filled, layout_for
    _check_codec(codec)
    lay = layout_for(offsets, sizes)
    flat = flat.reshape(-1)
    if flat.numel() < lay.total:
        raise ValueError("stoch_encode_batched: flat buffer smaller than the layout")
    dev = flat.device
    lv = _filled(flat.numel(), torch.int8 if codec == "cnat" else torch.uint8, dev, lay)
    sg = _filled(flat.numel(), torch.int8, dev, lay)
    mins = torch.zeros(lay.ntensors, dtype=torch.float32, device=dev)
    if flat.dtype in DT_DTYPES:
        lv, sg, nr, mn = encode_batched_dt(codec, flat, lay, bits, seed=seed, counter=counter, levels=lv, signs=sg)
        return lv, sg, nr.float(), (mn.float() if mn is not None else mins)
    if codec == "qsgd":
        lv, sg, nr = qsgd_encode_batched(flat, lay, bits, seed=seed, counter=counter, levels=lv, signs=sg)
    elif codec == "rqsgd":
        lv, sg, nr, mins = rqsgd_encode_batched(flat, lay, bits, seed=seed, counter=counter, levels=lv, signs=sg,
                                                mins=mins)
    else:
        lv, sg, nr = cnat_encode_batched(flat, lay, bits, seed=seed, counter=counter, exps=lv, signs=sg)
    return lv, sg, nr, mins


@stoch_encode_batched_op.register_fake
def _(flat, offsets, sizes, codec, bits, seed, counter):
    n, t = flat.numel(), sizes.numel()
    return (flat.new_empty((n,), dtype=torch.int8 if codec == "cnat" else torch.uint8),
            flat.new_empty((n,), dtype=torch.int8), flat.new_empty((t,), dtype=torch.float32),
            flat.new_empty((t,), dtype=torch.float32))


@torch.library.custom_op("adfl::stoch_decode_batched", mutates_args=())
def stoch_decode_batched_op(levels: torch.Tensor, signs: torch.Tensor, norms: torch.Tensor, mins: torch.Tensor,
                            offsets: torch.Tensor, sizes: torch.Tensor, codec: str, bits: int) -> torch.Tensor:
    """fp32 decode of stoch_encode_batched's planes (mins used by RQSGD only)."""
    from .ops import _filled, layout_for
    _check_codec(codec)
    lay = layout_for(offsets, sizes)
    levels, signs = levels.reshape(-1), signs.reshape(-1)
    if levels.numel() < lay.total or signs.numel() < lay.total:
        raise ValueError("stoch_decode_batched: planes smaller than the layout")
    out = _filled(levels.numel(), torch.float32, levels.device, lay)
    if codec == "qsgd":
        return qsgd_decode_batched(levels.view(torch.uint8), signs, norms, lay, bits, out=out)
    if codec == "rqsgd":
        return rqsgd_decode_batched(levels.view(torch.uint8), signs, norms, mins, lay, bits, out=out)
    return cnat_decode_batched(levels.view(torch.int8), signs, norms, lay, out=out)


@stoch_decode_batched_op.register_fake
def _(levels, signs, norms, mins, offsets, sizes, codec, bits):
    return levels.new_empty((levels.numel(),), dtype=torch.float32)
