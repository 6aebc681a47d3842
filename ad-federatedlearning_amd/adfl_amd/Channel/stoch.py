"""Stochastic-rounding channels backed by the MI355X HIP codec — drop-in for
``Src/ADFL/Channel/quant.py:140-570`` (QSGD, UQSGD, RQSGD, URQSGD, CNAT, UCNAT).

Same names, constructor (``bits``; ``levels = 2**bits - 1``), six-method surface, ``to_json`` output,
``simulate_bandwidth`` formulas and payload layout as the reference:

* ``QuantParameter.data`` = levels (uint8; CNAT: int8 exponents), ``signs`` = int8 sign plane,
  ``scale`` = the norm as a Python float (``norm.item()``), ``scale_2`` = RQSGD's min|x|;
* all-zero tensors take the reference's norm == 0 branch: uint8 zeros, int8 ones, ``scale`` = the 0-dim
  fp32 tensor ``tensor(0.)`` (quant.py:227-228,368-369,513-514);
* ``ndim <= 1`` tensors pass through (same object) with ``signs = zeros(1, uint8)`` and scale 0;
* ``size`` counts only the level / exponent bytes, as the reference does (quant.py:218,359,504);
* decode returns owned, writable fp32 tensors.

What changes is where the arithmetic runs: the whole state dict is staged once into one flat bucket on
the GPU and encoded / decoded by a few HIP launches for all tensors together (include/adfl_stoch.h).

Randomness: the reference draws ``torch.rand_like`` from torch's CPU generator. Here each encode draws a
fresh 62-bit seed from that same generator (so ``torch.manual_seed`` reproduces a run) and the kernels
generate their uniforms from a Philox4x32-7 stream keyed by it. The uniforms are not the reference's
mt19937 draws, so individual rounding decisions differ from a reference run; their distribution is the
same (and with injected uniforms the codec is bit-identical: tests/test_gpu_stoch.py).

Norms: the L2 norm (QSGD, CNAT) is the reference's own, bit for bit: torch 2.10's CPU
``torch.linalg.vector_norm`` order in the tensor's dtype (fp32 / bf16 / fp16 / fp64; fp16's split over
``torch.get_num_threads()`` as the reference's call would make it), by csrc/torch_norm.hip. ADFL_STOCH_NORM=fp64
in the environment switches to the correctly rounded norm (fp64 accumulation of the squares: faster on very
large tensors, within torch's own summation error of the reference's). RQSGD's max / min norms are exact either
way. There is no CPU fallback: without the HIP library these raise.

fp16 / bf16 / fp64 tensors are encoded as the reference encodes them, in their own dtype's arithmetic (each
op rounded to the dtype; uniforms on torch.rand's grid for the dtype): one bucket per dtype through the
*_dt kernels (csrc/stoch_dtype.hip). Their payloads decode like fp32 ones (the reference decodes to fp32).
"""

import ctypes
import os
import time
from typing import Dict, List, Tuple

import numpy as np
import torch

from .. import _lib, _torchhost, hostcopy, ops
from .. import stoch as sops
from .._lib import check
from ..model import CompressedParameters, Parameters, QuantParameter, QuantParameters, get_parameter_info
from .channel import Channel, IdentityChannel
from . import quant as _quant
from .quant import (_PendingD2H, _aggregate_entries, _chunk_meta, _drain, _hand_out, _host_heap, _ph,
                    _range_copies, _ranges, _serialized, _stage_in, _stage_rows, _staging, device_mean_order_ok)

_CODECS = ("qsgd", "rqsgd", "cnat")


def reference_norm() -> bool:
    """The L2 norm mode of the QSGD / CNAT channels: True (default) = the reference's own norm, torch's CPU
    order bit for bit; ADFL_STOCH_NORM=fp64 = the correctly rounded norm (fp64 accumulation)."""
    mode = os.environ.get("ADFL_STOCH_NORM", "torch").lower()
    if mode not in ("torch", "fp64"):
        raise ValueError(f"ADFL_STOCH_NORM must be 'torch' (the reference's norm) or 'fp64', got {mode!r}")
    return mode == "torch"


def _require_codable(name: str, t: torch.Tensor, cls: str) -> None:
    """fp32 / fp16 / bf16 / fp64 tensors are encoded (each in its own dtype's arithmetic, as the reference
    computes them). Anything else fails as the reference's first op on it fails: torch.linalg.vector_norm
    raises for integer and bool tensors (quant.py:226,367,512)."""
    if t.dtype == torch.float32 or t.dtype in sops.DT_DTYPES:
        return
    if not (t.is_floating_point() or t.is_complex()):
        torch.linalg.vector_norm(t.reshape(-1)[:0])   # raises the reference's RuntimeError
    raise ValueError(f"{cls}: '{name}' is {t.dtype}; the HIP stochastic codecs take fp32 / fp16 / bf16 / fp64")


def _owned(parts: List[torch.Tensor], shapes: List[torch.Size]) -> List[torch.Tensor]:
    """Per-tensor copies: each payload tensor owns its bytes (it is pickled on its own; the staging
    buffers are reused by the next call)."""
    return [p.view(s).clone() for p, s in zip(parts, shapes)]


_DTYPE_CODE = {torch.uint8: 0, torch.int8: 1, torch.float32: 2}   # adfl_torchhost.empty_like_dtype


def _owned_dev(buf: torch.Tensor, lay, shapes: List[torch.Size], like=None) -> List[torch.Tensor]:
    """_owned for a device dict: fresh tensors filled from the bucket by one launch (ops.bucket_scatter); with
    `like` (the dict's tensors, all on the bucket's device) created by one native call."""
    code = _DTYPE_CODE.get(buf.dtype)
    if like is not None and code is not None:
        outs, ptrs = _torchhost.get().empty_like_dtype(like, code)
        ops.bucket_scatter(buf, lay, outs, checked=False, ptrs=ptrs)
        return outs
    outs = [torch.empty(s, dtype=buf.dtype, device=buf.device) for s in shapes]
    ops.bucket_scatter(buf, lay, outs, checked=False)
    return outs


def _owned_host(buf: torch.Tensor, offsets, shapes: List[torch.Size]) -> List[torch.Tensor]:
    """_owned for a host bucket: fresh tensors filled by one native parallel scatter."""
    outs = [torch.empty(s, dtype=buf.dtype) for s in shapes]
    hostcopy.advise_huge(outs)
    hostcopy.scatter(buf, outs, offsets)
    return outs


@_serialized
def _encode_stoch(params: Parameters, names: List[str], codec: str, bits: int, uniforms=None, seed=None,
                  torch_norm: bool = True, emit=None, idle=None):
    """Encode the ndim > 1 fp32 tensors `names` of `params` in one bucketed pass.

    Returns {name: (data, signs, scale, scale_2)} with CPU tensors for CPU inputs (device tensors for
    device inputs). `uniforms`: optional fp32 device plane over the compact bucket (tests). For a dict of
    contiguous CPU tensors the outputs are built while the copies run (_encode_stoch_host): emit(k, data,
    signs) is called for each as soon as its planes exist (the scale follows in the return value) and idle()
    (True while it has work left) between the ranges."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    # every tensor's size, and whether all are contiguous CPU fp32 storages (their pointers), in one native call
    th = _torchhost.get()
    host_ok, numel, hptrs = th.host_bytes(tensors, 4)
    lay = st.layout(tuple(numel.tolist()))
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    if host_ok and _quant._PIPELINE:
        return _encode_stoch_host(tensors, names, hptrs.numpy().view(np.uint64), lay, st, codec, bits, uniforms,
                                  seed, torch_norm, emit or (lambda k, d, g: None), idle or (lambda: False))
    x_dev = _stage_in(tensors, lay, st, "x", torch.float32, host_ptrs=hptrs.numpy().view(np.uint64) if host_ok else None)
    ws = st.buf("stoch_ws", lay.nchunks * 16, torch.uint8)
    # staging buffers are cached by name: the level plane is always uint8 (CNAT views it as int8)
    levels, signs = st.buf("s_levels", lay.total, torch.uint8), st.buf("s_signs", lay.total, torch.int8)
    norms = st.buf("s_norms", lay.ntensors, torch.float32)
    mins = st.buf("s_mins", lay.ntensors, torch.float32) if codec == "rqsgd" else None
    lv, sg = _codec_encode(codec, x_dev, lay, bits, uniforms, seed, levels, signs, norms, mins, ws, torch_norm)
    nm_host = st.buf("s_norms_host", 2 * lay.ntensors, torch.float32, pinned=True)
    nm_host[:lay.ntensors].copy_(norms, non_blocking=True)
    if mins is not None:
        nm_host[lay.ntensors:].copy_(mins, non_blocking=True)
    if host_ok:
        # as SLQ's encode: both planes' D2H enqueued right behind the norms, the owned outputs of both planes
        # created by one native call each while they run, each range scattered as it lands
        norms_ready = torch.cuda.Event()
        norms_ready.record(torch.cuda.current_stream(dev))
        pend_lv = _PendingD2H(lv.view(torch.uint8), lay, st, "s_levels")
        pend_sg = _PendingD2H(sg, lay, st, "s_signs")
        lv_parts, lv_p = th.empty_like_dtype(tensors, 1 if lv.dtype == torch.int8 else 0)
        sg_parts, sg_p = th.empty_like_dtype(tensors, 1)
        big = np.nonzero(lay.sizes >= (4 << 20))[0].tolist()
        if big:
            hostcopy.advise_huge([lv_parts[i] for i in big] + [sg_parts[i] for i in big])
        pend_lv.finish(lv_parts, lv_p.numpy().view(np.uint64))
        pend_sg.finish(sg_parts, sg_p.numpy().view(np.uint64))
        norms_ready.synchronize()
        return _payloads(names, lv_parts, sg_parts, nm_host.tolist(), lay.ntensors, codec)
    on_cpu = [not t.is_cuda for t in tensors]
    if all(on_cpu):
        # non-contiguous CPU tensors: the same, one output at a time
        norms_ready = torch.cuda.Event()
        norms_ready.record(torch.cuda.current_stream(dev))
        pend_lv = _PendingD2H(lv.view(torch.uint8), lay, st, "s_levels")
        pend_sg = _PendingD2H(sg, lay, st, "s_signs")
        shapes = [t.shape for t in tensors]
        lv_parts = [torch.empty(s_, dtype=lv.dtype) for s_ in shapes]
        sg_parts = [torch.empty(s_, dtype=torch.int8) for s_ in shapes]
        hostcopy.advise_huge(lv_parts + sg_parts)
        norms_ready.synchronize()
        nm = nm_host.tolist()
        pend_lv.finish([t.view(torch.uint8) for t in lv_parts])
        pend_sg.finish(sg_parts)
        return _payloads(names, lv_parts, sg_parts, nm, lay.ntensors, codec)
    if any(on_cpu):
        lv_h = st.buf("s_levels_host", lay.total, torch.uint8, pinned=True).view(lv.dtype)
        sg_h = st.buf("s_signs_host", lay.total, torch.int8, pinned=True)
        lv_h.copy_(lv, non_blocking=True)
        sg_h.copy_(sg, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    nm = nm_host.tolist()
    sizes, shapes = lay.sizes.tolist(), [t.shape for t in tensors]
    split = lambda buf: [p[:n] for p, n in zip(torch.split(buf, lay.padded.tolist()), sizes)]  # noqa: E731
    lv_parts = _owned_host(lv_h, lay.offsets, shapes) if any(on_cpu) else None
    sg_parts = _owned_host(sg_h, lay.offsets, shapes) if any(on_cpu) else None
    if not any(on_cpu):   # device dict: one scatter launch per plane
        same = _torchhost.get().device_ptrs(tensors, dev.index, 4)[0]   # all on the staging's device
        lv_dev = _owned_dev(lv, lay, shapes, like=tensors if same else None)
        sg_dev = _owned_dev(sg, lay, shapes, like=tensors if same else None)
    else:
        lv_dev = _owned(split(lv), shapes) if not all(on_cpu) else None
        sg_dev = _owned(split(sg), shapes) if not all(on_cpu) else None
    datas = [(lv_parts if cpu else lv_dev)[i] for i, cpu in enumerate(on_cpu)]
    signs = [(sg_parts if cpu else sg_dev)[i] for i, cpu in enumerate(on_cpu)]
    return _payloads(names, datas, signs, nm, lay.ntensors, codec)


def _codec_encode(codec: str, x_dev, lay, bits: int, uniforms, seed: int, levels, signs, norms, mins, ws,
                  torch_norm: bool):
    """The codec's encode over `lay` (a whole bucket, or a caller-placed sub-layout of some of its tensors at
    their bucket offsets: every kernel indexes x, the planes and the uniforms by absolute element, and the
    norms by the layout's own tensor index, so `norms` / `mins` are then views at the first tensor). Returns
    the (levels, signs) planes in the codec's dtypes."""
    if codec == "qsgd":
        lv, sg, _ = sops.qsgd_encode_batched(x_dev, lay, bits, uniforms=uniforms, seed=seed, counter=0, levels=levels,
                                             signs=signs, norms=norms, ws=ws, torch_norm=torch_norm)
    elif codec == "rqsgd":
        lv, sg, _, _ = sops.rqsgd_encode_batched(x_dev, lay, bits, uniforms=uniforms, seed=seed, counter=0,
                                                 levels=levels, signs=signs, norms=norms, mins=mins, ws=ws)
    else:
        lv, sg, _ = sops.cnat_encode_batched(x_dev, lay, bits, uniforms=uniforms, seed=seed, counter=0,
                                             exps=levels.view(torch.int8), signs=signs, norms=norms, ws=ws,
                                             torch_norm=torch_norm)
    return lv, sg


def _range_encode_args(sub, dev) -> Tuple[int, int, int, int, int, int]:
    """A sub-layout's fixed arguments for _range_encode (cached on it): (chunk table, nchunks, tfirst list,
    ntensors, norm kinds, norm scratch bytes)."""
    cache = sub.__dict__.setdefault("_range_encode_args", {})
    a = cache.get(dev.index)
    if a is None:
        L = _lib.load()
        short_max = L.adfl_torch_norm_short_max_dt(sops.DTYPE_F32)
        kinds = (1 if int(sub.sizes.min()) <= short_max else 0) | (2 if int(sub.sizes.max()) > short_max else 0)
        a = cache[dev.index] = (sub.device_chunks(dev).data_ptr(), sub.nchunks, sub.device_tfirst(dev).data_ptr(),
                                sub.ntensors, kinds, int(L.adfl_torch_norm_scratch_bytes(sub.nchunks, sub.ntensors)))
    return a


def _range_encode(codec: str, x_dev, sub, bits: int, seed: int, levels, signs, norms, made: int, ws, st) -> None:
    """_codec_encode of QSGD / CNAT with the reference's norm and Philox uniforms for one staging range, as
    direct native calls on the sub-layout's cached arguments: the same launches (adfl_torch_norms_work, then
    adfl_qsgd_quantize_batched / adfl_cnat_encode_batched_work) and bytes as the sops wrappers, without their
    per-call checks and allocations (~60 -> ~15 us of host time per range)."""
    L = _lib.load()
    dev = x_dev.device
    sh = torch.cuda.current_stream(dev).cuda_stream
    cp, nc, tp, nt, kinds, need = _range_encode_args(sub, dev)
    nd = norms.data_ptr() + 4 * made
    xd = x_dev.data_ptr()
    if codec == "cnat":   # the exponents do not depend on the norm: encode, then the reference's norms over it
        wp, nw = sops._work(sub, dev)
        check(L.adfl_cnat_encode_batched_work(xd, cp, nc, wp, nw, bits, 0, seed, 0, ws.data_ptr(), ws.numel(),
                                              levels.data_ptr(), signs.data_ptr(), nd, sh))
    scratch = st.buf("tn_scratch", need, torch.uint8)   # stream-ordered reuse: every range runs on this stream
    check(L.adfl_torch_norms_work(sops.DTYPE_F32, xd, cp, nc, tp, nt, kinds, 1, scratch.data_ptr(), need, None, nd, sh))
    if codec == "qsgd":
        check(L.adfl_qsgd_quantize_batched(xd, cp, nc, bits, nd, 0, seed, 0, levels.data_ptr(), signs.data_ptr(), sh))


def _sub_layout(lay, t0: int, t1: int):
    """Tensors [t0, t1) of `lay` at their bucket offsets, as a layout of their own (cached on `lay`: the staging
    ranges of a layout complete the same tensor runs every call)."""
    cache = lay.__dict__.setdefault("_sub_layouts", {})
    sub = cache.get((t0, t1))
    if sub is None:
        sub = cache[(t0, t1)] = ops.BucketLayout(lay.sizes[t0:t1].tolist(), offsets=lay.offsets[t0:t1].tolist())
    return sub


def _encode_stoch_host(tensors, names, hptrs: np.ndarray, lay, st, codec: str, bits: int, uniforms, seed: int,
                       torch_norm: bool, emit, idle):
    """A CPU fp32 dict's QSGD / RQSGD / CNAT encode, pipelined range by range as SLQ's host encode is: the
    gathers into the pinned bucket queued on the native pool at once; as range r lands its H2D is enqueued
    (adfl_stage_encode_range with no kernel), and the tensors whose every byte is now staged are encoded at
    once by the codec's kernels over a sub-layout of just those tensors (_codec_encode: the same bytes as the
    whole-bucket encode, norms included), their level and sign bytes go back D2H on the side stream behind an
    event (adfl_stage_d2h), their outputs are created (one native call per plane) and the scatter of both
    planes queued on the pool behind the event — so the planes' D2H overlaps the next ranges' H2D. The H2D
    runs on a stream of its own, enqueued as soon as each gather lands, so a range's kernels and outputs
    (longer on the calling thread than a range's copy) never hold the link back."""
    with _ph("enc.heap"):
        _host_heap(lay)
    dev = st.device
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    lib = _lib.load()
    th = _torchhost.get()
    x_dev = st.buf("x", lay.total, torch.float32)
    host = st.buf("x_host", lay.total, torch.float32, pinned=True)
    ws = st.buf("stoch_ws", lay.nchunks * 16, torch.uint8)
    levels, signs = st.buf("s_levels", lay.total, torch.uint8), st.buf("s_signs", lay.total, torch.int8)
    lv_host = st.buf("s_levels_host", lay.total, torch.uint8, pinned=True)
    sg_host = st.buf("s_signs_host", lay.total, torch.int8, pinned=True)
    norms = st.buf("s_norms", lay.ntensors, torch.float32)
    mins = st.buf("s_mins", lay.ntensors, torch.float32) if codec == "rqsgd" else None
    nm_host = st.buf("s_norms_host", 2 * lay.ntensors, torch.float32, pinned=True)
    ranges = _ranges(lay, 4)
    evs = st.events(2 * len(ranges))
    d2h_h = st.d2h_stream().cuda_stream
    hx, dx = host.data_ptr(), x_dev.data_ptr()
    ld, lh, gd, gh = levels.data_ptr(), lv_host.data_ptr(), signs.data_ptr(), sg_host.data_ptr()
    with _ph("enc.gather_submit"):
        jobs = [hostcopy.submit_pieces(*_range_copies(hptrs, lay, hx, 4, lo, hi, to_bucket=True), keep=host)
                for lo, hi in ranges]
    ends = lay.offsets + lay.sizes
    code = 1 if codec == "cnat" else 0
    fast = torch_norm and codec in ("qsgd", "cnat") and uniforms is None   # _range_encode's case
    lv_parts: List[torch.Tensor] = []
    sg_parts: List[torch.Tensor] = []
    lv_ptrs = np.zeros(lay.ntensors, dtype=np.uint64)
    sg_ptrs = np.zeros(lay.ntensors, dtype=np.uint64)
    copies = (ctypes.c_void_p * 2)(), (ctypes.c_void_p * 2)(), (ctypes.c_int64 * 2)()
    scatters = []
    h2d = st.h2d_stream()
    h2d_h = h2d.cuda_stream
    h2d.wait_stream(stream)   # the staging buffers' last readers
    landed = [torch.cuda.Event() for _ in ranges]
    made = 0
    r_h2d = 0
    try:
        for r, (lo, hi) in enumerate(ranges):
            # every range whose gather has landed goes to the link at once, on its own stream (the compute
            # stream waits only for the ranges its kernels read); block on a gather only when range r's is next
            while r_h2d < len(ranges) and (r_h2d == r or jobs[r_h2d].done()):
                with _ph("enc.gather_wait"):
                    jobs[r_h2d].wait()
                with _ph("enc.h2d_launch"):
                    a, b = ranges[r_h2d]
                    check(lib.adfl_stage_encode_range(hx, dx, a, b, None, None, 0, 0, 0, None, None, None, 0, 0, h2d_h,
                                                      None, None, None))
                    landed[r_h2d].record(h2d)
                r_h2d += 1
            done = int(np.searchsorted(ends, hi, side="right"))   # tensors whose every byte is staged
            if done <= made:
                continue
            with _ph("enc.kernel_launch"):
                stream.wait_event(landed[r])
                if fast:
                    _range_encode(codec, x_dev, _sub_layout(lay, made, done), bits, seed, levels, signs, norms, made,
                                  ws, st)
                else:
                    _codec_encode(codec, x_dev, _sub_layout(lay, made, done), bits, uniforms, seed, levels, signs,
                                  norms[made:], mins[made:] if mins is not None else None, ws, torch_norm)
                e0, e1 = int(lay.offsets[made]), int(ends[done - 1])
                src, dst, nb = copies
                src[0], src[1], dst[0], dst[1] = ld + e0, gd + e0, lh + e0, gh + e0
                nb[0] = nb[1] = e1 - e0
                check(lib.adfl_stage_d2h(src, dst, nb, 2, sh, d2h_h, evs[2 * r], evs[2 * r + 1]))
            with _ph("enc.outputs"):
                lts, lpt = th.empty_like_dtype(tensors[made:done], code)
                gts, gpt = th.empty_like_dtype(tensors[made:done], 1)
                lv_parts.extend(lts)
                sg_parts.extend(gts)
                lv_ptrs[made:done] = lpt.numpy().view(np.uint64)
                sg_ptrs[made:done] = gpt.numpy().view(np.uint64)
            with _ph("enc.scatter_submit"):
                a = _range_copies(lv_ptrs, lay, lh, 1, e0, e1, to_bucket=False)
                b = _range_copies(sg_ptrs, lay, gh, 1, e0, e1, to_bucket=False)
                scatters.append(hostcopy.submit_pieces(*(np.concatenate([u, v]) for u, v in zip(a, b)), stream=True,
                                                       event=evs[2 * r + 1], keep=(lv_host, sg_host)))
            with _ph("enc.passthrough"):
                for k in range(made, done):   # the caller's payload objects, their scales filled in at the end
                    emit(k, lv_parts[k], sg_parts[k])
                made = done
                idle()
        nm_host[:lay.ntensors].copy_(norms, non_blocking=True)
        if mins is not None:
            nm_host[lay.ntensors:].copy_(mins, non_blocking=True)
        norms_ready = torch.cuda.Event()
        norms_ready.record(stream)
        with _ph("enc.passthrough"):
            while idle():   # the caller's remaining objects, while the last copies land
                pass
    except BaseException:
        _drain(h2d, stream, st.d2h_stream())
        raise
    finally:
        for j in jobs:
            j.wait()
        with _ph("enc.scatter_wait"):
            for j in scatters:
                j.wait()
    with _ph("enc.norms_wait"):
        norms_ready.synchronize()
    with _ph("enc.payloads"):
        return _payloads(names, lv_parts, sg_parts, nm_host.tolist(), lay.ntensors, codec)


# Philox block-counter base of each dtype bucket: one seed serves an fp32 bucket and every fp16 / bf16 / fp64
# bucket of the same call, and each draws from its own disjoint part of the stream (2^40 blocks = 2^42
# uniforms each), so no two buckets' rounding decisions share a uniform.
COUNTER_BASE = {torch.float32: 0, torch.float16: 1 << 40, torch.bfloat16: 2 << 40, torch.float64: 3 << 40}


@_serialized
def _encode_stoch_dt(params: Parameters, names: List[str], codec: str, bits: int, uniforms=None, seed=None,
                     torch_norm: bool = True):
    """Encode the ndim > 1 tensors `names` (all of one dtype: fp16 / bf16 / fp64) in one bucketed pass, in
    that dtype's arithmetic (adfl_stoch_encode_batched_dt). Same return as _encode_stoch; the norms are the
    dtype's values as Python floats (norm.item() of the reference's 0-dim norm tensor)."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    dtype = tensors[0].dtype
    tag = str(dtype).replace("torch.", "")
    lay = st.layout(tuple(int(t.numel()) for t in tensors))
    x_dev = _stage_in(tensors, lay, st, "x_" + tag, dtype)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    ws = st.buf("stoch_ws", lay.nchunks * 16, torch.uint8)
    u = uniforms if uniforms is not None and uniforms.dtype == dtype else None
    levels = st.buf("s_levels", lay.total, torch.uint8).view(torch.int8 if codec == "cnat" else torch.uint8)
    signs = st.buf("s_signs", lay.total, torch.int8)
    if codec != "rqsgd" and torch_norm:  # the reference's norm in the dtype, then the given-norm quantize
        norms, _ = sops.reference_norms(x_dev, lay, out64=st.buf("s_norms64", lay.ntensors, torch.float64))
        lv, sg = sops.quantize_batched_dt(codec, x_dev, lay, bits, norms, uniforms=u, seed=seed,
                                          counter=COUNTER_BASE[dtype], levels=levels, signs=signs)
        mins = None
    else:
        lv, sg, norms, mins = sops.encode_batched_dt(codec, x_dev, lay, bits, uniforms=u, seed=seed,
                                                     counter=COUNTER_BASE[dtype], levels=levels, signs=signs, ws=ws)
    nm = torch.cat([norms, mins]) if mins is not None else norms
    on_cpu = [not t.is_cuda for t in tensors]
    shapes = [t.shape for t in tensors]
    if any(on_cpu):
        lv_h = st.buf("s_levels_host", lay.total, torch.uint8, pinned=True).view(lv.dtype)
        sg_h = st.buf("s_signs_host", lay.total, torch.int8, pinned=True)
        lv_h.copy_(lv, non_blocking=True)
        sg_h.copy_(sg, non_blocking=True)
    nm = nm.cpu().tolist()   # synchronises: the planes' D2H has landed too
    sizes = lay.sizes.tolist()
    split = lambda buf: [p[:n] for p, n in zip(torch.split(buf, lay.padded.tolist()), sizes)]  # noqa: E731
    lv_parts = _owned_host(lv_h, lay.offsets, shapes) if any(on_cpu) else None
    sg_parts = _owned_host(sg_h, lay.offsets, shapes) if any(on_cpu) else None
    if not any(on_cpu):   # device dict: one scatter launch per plane
        lv_dev, sg_dev = _owned_dev(lv, lay, shapes), _owned_dev(sg, lay, shapes)
    else:
        lv_dev = _owned(split(lv), shapes) if not all(on_cpu) else None
        sg_dev = _owned(split(sg), shapes) if not all(on_cpu) else None
    datas = [(lv_parts if cpu else lv_dev)[i] for i, cpu in enumerate(on_cpu)]
    signs = [(sg_parts if cpu else sg_dev)[i] for i, cpu in enumerate(on_cpu)]
    return _payloads(names, datas, signs, nm, lay.ntensors, codec, dtype)


def _payloads(names, datas, signs, nm, ntensors: int, codec: str, dtype: torch.dtype = torch.float32):
    """{name: (data, signs, scale, scale_2)} as the reference's _quantize_tensor returns them."""
    out = {}
    for i, name in enumerate(names):
        data, norm = datas[i], nm[i]
        if norm == 0.0:  # the reference's norm == 0 branch: uint8 zeros, the 0-dim norm tensor as scale
            scale = torch.tensor(0.0, dtype=dtype)
            data = data.view(torch.uint8)
            scale_2 = 0
        else:
            scale = norm
            scale_2 = nm[ntensors + i] if codec == "rqsgd" else 0
        out[name] = (data, signs[i], scale, scale_2)
    return out


@_serialized
def _decode_stoch(items: List[Tuple[str, QuantParameter]], codec: str, bits: int) -> Dict[str, torch.Tensor]:
    """Decode (levels, signs, norm[, min]) payloads of ndim > 1 tensors in one bucketed pass."""
    st = _staging()
    if _quant._PIPELINE:
        th = _torchhost.get()
        datas = [p.data for _, p in items]
        signs = [p.signs for _, p in items]
        ok_l, numel, lptrs = th.host_bytes(datas, 1)
        ok_s, numel_s, sptrs = th.host_bytes(signs, 1)
        if ok_l and ok_s and torch.equal(numel, numel_s):   # CPU payloads: range-pipelined (_decode_stoch_host)
            decoded = _decode_stoch_host(st, items, datas, numel, lptrs.numpy().view(np.uint64),
                                         sptrs.numpy().view(np.uint64), codec, bits)
            return {name: t for (name, _), t in zip(items, decoded)}
    lay, out_dev = _decode_stoch_bucket(st, items, codec, bits)
    datas = [p.data for _, p in items]
    on_cpu = [not d.is_cuda for d in datas]
    # CPU payloads: the fp32 outputs (shaped like the level planes) made in one native call per range
    decoded = _hand_out(out_dev, lay, [d.shape for d in datas], on_cpu, st, "d_out", like=datas)
    return {name: t for (name, _), t in zip(items, decoded)}


_CODEC_ID = {"qsgd": 0, "rqsgd": 1, "cnat": 2}   # ADFL_CODEC_* (include/adfl_stoch.h)


def _decode_stoch_host(st, items, datas, numel: torch.Tensor, lptrs: np.ndarray, sptrs: np.ndarray, codec: str,
                       bits: int) -> List[torch.Tensor]:
    """CPU level / sign planes -> owned CPU fp32 tensors, pipelined range by range as SLQ's host decode
    (quant._decode_host_dict): both planes' byte gathers queued on the native pool at once; as range r lands,
    one native call (adfl_stage_stoch_decode_range) enqueues its two H2Ds, the codec's dequantize of the chunks
    it completes and their floats' D2H on the side stream behind an event; the outputs those chunks reach are
    created (one native call) and their scatter queued on the pool behind the event. Bit-identical to the
    one-launch decode (each chunk is decoded by the same kernel)."""
    lay = st.layout(tuple(numel.tolist()))
    with _ph("dec.heap"):
        _host_heap(lay)
    dev = st.device
    sh = torch.cuda.current_stream(dev).cuda_stream
    lib = _lib.load()
    lv_dev = st.buf("d_levels", lay.total, torch.uint8)
    sg_dev = st.buf("d_signs", lay.total, torch.int8)
    lv_host = st.buf("d_levels_host", lay.total, torch.uint8, pinned=True)
    sg_host = st.buf("d_signs_host", lay.total, torch.int8, pinned=True)
    out_dev = st.buf("d_out", lay.total, torch.float32)
    out_host = st.buf("d_out_host", lay.total, torch.float32, pinned=True)
    ntens = len(items)
    sc = torch.tensor([float(p.scale) for _, p in items] + ([float(p.scale_2) for _, p in items]
                                                            if codec == "rqsgd" else []), dtype=torch.float32)
    s_dev = sc.to(dev, non_blocking=True)
    nd = s_dev.data_ptr()
    md = nd + 4 * ntens if codec == "rqsgd" else 0
    chunks_ptr = lay.device_chunks(dev).data_ptr()
    d2h_h = st.d2h_stream().cuda_stream
    cm = _chunk_meta(lay)
    th = _torchhost.get()
    ranges = _ranges(lay, 4)
    evs = st.events(2 * len(ranges))
    lh, ld, gh, gd = lv_host.data_ptr(), lv_dev.data_ptr(), sg_host.data_ptr(), sg_dev.data_ptr()
    od, oh = out_dev.data_ptr(), out_host.data_ptr()
    cid = _CODEC_ID[codec]
    jobs = []
    with _ph("dec.gather_submit"):
        for lo, hi in ranges:
            a = _range_copies(lptrs, lay, lh, 1, lo, hi, to_bucket=True)
            b = _range_copies(sptrs, lay, gh, 1, lo, hi, to_bucket=True)
            jobs.append(hostcopy.submit_pieces(*(np.concatenate([x, y]) for x, y in zip(a, b)),
                                               keep=(lv_host, sg_host)))
    offs = lay.offsets
    outs: List[torch.Tensor] = []
    out_ptrs = np.zeros(lay.ntensors, dtype=np.uint64)
    scatters = []
    c_made = t_made = 0
    try:
        for r, ((lo, hi), job) in enumerate(zip(ranges, jobs)):
            with _ph("dec.gather_wait"):
                job.wait()
            with _ph("dec.kernel_launch"):
                c_end = int(np.searchsorted(cm.end, hi, side="right"))   # chunks whose every byte is staged
                if c_end <= c_made:
                    check(lib.adfl_stage_stoch_decode_range(cid, bits, lh, ld, gh, gd, lo, hi, chunks_ptr, 0, 0, nd, md,
                                                            od, oh, 0, 0, sh, d2h_h, evs[2 * r], evs[2 * r + 1]))
                    continue
                e0, e1 = int(cm.start[c_made]), int(cm.end[c_end - 1])
                check(lib.adfl_stage_stoch_decode_range(cid, bits, lh, ld, gh, gd, lo, hi, chunks_ptr, c_made,
                                                        c_end - c_made, nd, md, od, oh, e0, e1, sh, d2h_h, evs[2 * r],
                                                        evs[2 * r + 1]))
                c_made = c_end
            with _ph("out.alloc"):
                t_end = int(np.searchsorted(offs, e1, side="left"))    # tensors starting below e1
                if t_end > t_made:
                    ts, pt = th.empty_f32_like(datas[t_made:t_end])
                    outs.extend(ts)
                    out_ptrs[t_made:t_end] = pt.numpy().view(np.uint64)
                    for j in np.nonzero(lay.sizes[t_made:t_end] * 4 >= (4 << 20))[0].tolist():
                        hostcopy.advise_huge([ts[j]])
                    t_made = t_end
            with _ph("out.scatter_submit"):
                scatters.append(hostcopy.submit_pieces(
                    *_range_copies(out_ptrs, lay, oh, 4, e0, e1, to_bucket=False),
                    stream=True, event=evs[2 * r + 1], keep=out_host))
    except BaseException:
        _drain(torch.cuda.current_stream(dev), st.d2h_stream())
        raise
    finally:
        for j in jobs:
            j.wait()
        with _ph("out.scatter_wait"):
            for j in scatters:
                j.wait()
    return outs


@_serialized
def _decode_add_stoch(items: List[Tuple[str, QuantParameter]], codec: str, bits: int,
                      targets: List[List[torch.Tensor]]) -> None:
    """Decode the payloads once into the device bucket and add it into every model (targets[k][j] += decode of
    item j, fp32 adds: add_parameters_inpace's mul_(1).add_(d, alpha=1), model.py:337-347)."""
    st = _staging()
    lay, out_dev = _decode_stoch_bucket(st, items, codec, bits)
    views = [out_dev[o:o + n].view(p.data.shape)
             for o, n, (_, p) in zip(lay.offsets.tolist(), lay.sizes.tolist(), items)]
    with torch.no_grad():
        for model in targets:
            torch._foreach_add_(model, views)
    # the next call's staging rewrites the pinned buffers this call's H2D read and the bucket it decoded into
    torch.cuda.current_stream(st.device).synchronize()


def _decode_stoch_bucket(st, items: List[Tuple[str, QuantParameter]], codec: str, bits: int):
    """Both planes staged as one bucket on the device and decoded by one launch: (layout, fp32 bucket)."""
    dev = st.device
    lay = st.layout(tuple(int(p.data.numel()) for _, p in items))
    lv_dev = _stage_in([p.data.view(torch.uint8) for _, p in items], lay, st, "d_levels", torch.uint8)
    sg_dev = _stage_in([p.signs.view(torch.int8) for _, p in items], lay, st, "d_signs", torch.int8)
    scales = [float(p.scale) for _, p in items]
    ntens = len(items)
    sc = torch.tensor(scales + ([float(p.scale_2) for _, p in items] if codec == "rqsgd" else []),
                      dtype=torch.float32).to(dev, non_blocking=True)
    out_dev = st.buf("d_out", lay.total, torch.float32)
    if codec == "qsgd":
        sops.qsgd_decode_batched(lv_dev, sg_dev, sc[:ntens], lay, bits, out=out_dev)
    elif codec == "rqsgd":
        sops.rqsgd_decode_batched(lv_dev, sg_dev, sc[:ntens], sc[ntens:], lay, bits, out=out_dev)
    else:
        sops.cnat_decode_batched(lv_dev.view(torch.int8), sg_dev, sc[:ntens], lay, out=out_dev)
    return lay, out_dev


@_serialized
def _decode_mean_stoch(all_c_params: List[QuantParameters], names: List[str], codec: str,
                       bits: int) -> List[torch.Tensor]:
    """simple_aggregate over K payloads of the entries `names` (every client's entry decodable by
    _decode_stoch, one shape): both byte planes of every client staged as device rows, one launch of
    adfl_stoch_dequantize_mean_batched, one owned fp32 tensor per entry (CPU when the payloads are)."""
    st = _staging()
    dev = st.device
    first = all_c_params[0].params
    lay = st.layout(tuple(int(first[n].data.numel()) for n in names))
    lv_rows = _stage_rows([[c.params[n].data for n in names] for c in all_c_params], lay, st, "sm_levels")
    sg_rows = _stage_rows([[c.params[n].signs for n in names] for c in all_c_params], lay, st, "sm_signs")
    norms = torch.tensor([[float(c.params[n].scale) for n in names] for c in all_c_params],
                         dtype=torch.float32).to(dev, non_blocking=True)
    mins = (torch.tensor([[float(c.params[n].scale_2) for n in names] for c in all_c_params],
                         dtype=torch.float32).to(dev, non_blocking=True) if codec == "rqsgd" else None)
    out_dev = sops.dequantize_mean_batched(codec, lv_rows, sg_rows, norms, lay, bits, mins=mins,
                                           out=st.buf("sm_out", lay.total, torch.float32))
    on_cpu = [not any(c.params[n].data.is_cuda for c in all_c_params) for n in names]
    return _hand_out(out_dev, lay, [first[n].data.shape for n in names], on_cpu, st, "sm_out")


@_serialized
def _decode_mean_stoch_host(like: List[torch.Tensor], numel: torch.Tensor, lv_ptrs: List[np.ndarray],
                            sg_ptrs: List[np.ndarray], norms: torch.Tensor, mins, codec: str,
                            bits: int) -> List[torch.Tensor]:
    """_decode_mean_stoch for K CPU updates already checked (_StochChannel._mean_host_updates): both planes of
    every client gathered straight from the storages into pinned rows (one native gather per client and
    plane, each row's H2D enqueued as soon as it is staged), one decode-mean launch, the fp32 means handed
    back as owned CPU tensors shaped like `like`, created by one native call per staging range."""
    st = _staging()
    dev = st.device
    lay = st.layout(tuple(numel.tolist()))
    _host_heap(lay)
    k = len(lv_ptrs)
    row = (lay.total + 15) // 16 * 16
    rows = {}
    for key, ptrs, dt in (("sm_levels", lv_ptrs, torch.uint8), ("sm_signs", sg_ptrs, torch.int8)):
        d = st.buf(key, k * row, torch.uint8).view(k, row)
        h = st.buf(key + "_host", k * row, torch.uint8, pinned=True).view(k, row)
        for r in range(k):
            hostcopy.copy_pieces(*_range_copies(ptrs[r], lay, h[r].data_ptr(), 1, 0, lay.total, to_bucket=True))
            d[r].copy_(h[r], non_blocking=True)
        rows[key] = d if dt == torch.uint8 else d.view(torch.int8)
    nd = norms.to(dev, non_blocking=True)
    md = mins.to(dev, non_blocking=True) if mins is not None else None
    out_dev = sops.dequantize_mean_batched(codec, rows["sm_levels"], rows["sm_signs"], nd, lay, bits, mins=md,
                                           out=st.buf("sm_out", lay.total, torch.float32))
    return _hand_out(out_dev, lay, [None] * len(like), [True] * len(like), st, "sm_out", like=like)


class _StochChannel(Channel):
    """Shared body of the three bi-directional stochastic channels."""

    CODEC = "qsgd"
    NORM_BYTES = 4  # per quantized tensor: the norm (RQSGD: norm + minimum factor)

    def __init__(self, bits: int) -> None:
        """The reference's constructor (quant.py:145-147): the L2 norm is the reference's own (see the module
        docstring; ADFL_STOCH_NORM=fp64 selects the correctly rounded one instead)."""
        self.bits = bits
        self.levels = 2 ** bits - 1

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return self._send(params)

    def on_server_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return self._receive(c_params)

    def on_client_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return self._send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return self._receive(c_params)

    def to_json(self) -> Dict:
        return {"name": self.__class__.__name__, "bits": self.bits}

    def simulate_bandwidth(self, params: Parameters, mbps: float) -> float:
        """self.bits + 1 for weights and signs, 32 bits for biases, norms (quant.py:173-184,313-324,459-470)."""
        p_info = get_parameter_info(params)
        num_bytes = p_info.num_non_bias_w * (self.bits + 1) / 8
        num_bytes += p_info.num_bias_w * 4
        num_bytes += p_info.num_non_bias_t * self.NORM_BYTES
        transfer_time = num_bytes / (mbps * 1_000_000 / 8)
        time.sleep(transfer_time)
        return transfer_time

    def _send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        s_time = time.perf_counter()
        q_params = self._quantize_params(params, self.bits)
        return q_params, time.perf_counter() - s_time

    def _receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        assert isinstance(c_params, QuantParameters)
        s_time = time.perf_counter()
        names = list(c_params.params.keys())
        ps = list(c_params.params.values())
        datas = [p.data for p in ps]
        th = _torchhost.get()
        ndim, numel, _, _ = (a.numpy() for a in th.tensor_meta(datas))   # every entry in one native call
        coded = (ndim > 1) & (numel > 0)
        ci = np.nonzero(coded)[0].tolist()
        decoded = _decode_stoch([(names[i], ps[i]) for i in ci], self.CODEC, self.bits) if ci else {}
        vals = [None] * len(names)
        for i in ci:
            vals[i] = decoded[names[i]]
        for i in np.nonzero(~coded & (ndim > 1))[0].tolist():   # empty tensor: the reference's scale == 0 branch
            vals[i] = torch.zeros_like(datas[i], dtype=torch.float32)
        pi = np.nonzero(ndim <= 1)[0].tolist()
        for i, t in zip(pi, th.variable_data([datas[i] for i in pi])):
            vals[i] = t  # passthrough: q_param.data.data
        return dict(zip(names, vals)), time.perf_counter() - s_time

    def receive_mean(self, all_c_params: List[CompressedParameters]) -> Tuple[Parameters, float]:
        """``simple_aggregate([self.on_server_receive(c)[0] for c in all_c_params])`` — a synchronous server
        decoding K client updates and averaging them (Src/ADFL/Strategy/simple.py:83-89 over
        Src/ADFL/model.py:221-234). Returns (aggregate, seconds).

        Entries encoded in every update are decoded and averaged on the device in one launch (each client's
        level and sign planes read once, no decoded copy materialised): summed in torch's CPU order for
        ``torch.sum(torch.stack(...), dim=0)`` (csrc/torch_sum_order.h), then / K, bit-identical to
        simple_aggregate of the decoded CPU tensors at every K (tests/golden/aggregate.npz: the reference's
        own payloads and aggregates at K = 5, 8, 16, 20). Everything else (biases, running statistics, empty
        tensors) is decoded and aggregated as the reference does, on the host."""
        if not all_c_params:
            raise AssertionError("receive_mean: no updates")   # simple_aggregate asserts len > 0
        for c in all_c_params:
            assert isinstance(c, QuantParameters)
        s_time = time.perf_counter()
        names = list(all_c_params[0].params.keys())
        order_ok = device_mean_order_ok()
        out: Parameters = {}
        fast = self._mean_host_updates(all_c_params, names) if order_ok else None
        if fast is not None:   # every update a CPU dict of the same entries: classified in native calls
            fused, decoded = fast
            out.update(zip(fused, decoded))
        else:
            fused = [n for n in names if all(n in c.params and self._fusable(c.params[n]) for c in all_c_params)
                     and len({tuple(c.params[n].data.shape) for c in all_c_params}) == 1] if order_ok else []
            if fused:
                out.update(zip(fused, _decode_mean_stoch(all_c_params, fused, self.CODEC, self.bits)))
        rest = [n for n in names if n not in out]
        if rest:
            parts = [self._receive(QuantParameters({n: c.params[n] for n in rest}, 0))[0] for c in all_c_params]
            out.update(_aggregate_entries(rest, parts))
        return {n: out[n] for n in names}, time.perf_counter() - s_time

    def receive_add_(self, c_params: CompressedParameters, targets: List[Parameters]) -> float:
        """``on_client_receive(c_params)`` followed by ``add_parameters_inpace(t, decoded, 1, 1, False)`` for
        every ``t`` in ``targets`` — the client pool's ``add_to_model`` / ``add_to_model_all``
        (Src/ADFL/Client/pool.py:62-75) and QAFeL's hidden-state update (Src/ADFL/Server/qafel.py:176-179),
        bit-identical to them. Returns the seconds spent.

        Encoded tensors whose targets are all fp32 device tensors are decoded once, into device memory, and
        added into every model there (no decoded tensor crosses PCIe). Everything else takes the reference's
        route: decode, then ``mul_(1).add_(decoded, alpha=1)``."""
        assert isinstance(c_params, QuantParameters)
        for t in targets:
            assert set(t.keys()) == set(c_params.params.keys())  # add_parameters_inpace, model.py:340
        s_time = time.perf_counter()
        fused = [n for n, p in c_params.params.items()
                 if self._fusable(p) and all(t[n].is_cuda and t[n].dtype == torch.float32 for t in targets)]
        if fused and targets:
            dev = targets[0][fused[0]].device   # the staging's device (the current one) for the whole set
            if dev.index == torch.cuda.current_device() and all(t[n].device == dev for t in targets for n in fused):
                _decode_add_stoch([(n, c_params.params[n]) for n in fused], self.CODEC, self.bits,
                                  [[t[n] for n in fused] for t in targets])
            else:
                fused = []
        rest = QuantParameters({n: p for n, p in c_params.params.items() if n not in fused}, 0)
        if rest.params:
            decoded, _ = self.on_client_receive(rest)
            with torch.no_grad():
                for t in targets:
                    for n, d in decoded.items():
                        t[n].mul_(1).add_(d.to(t[n].device), alpha=1)
        return time.perf_counter() - s_time

    def _mean_host_updates(self, all_c_params: List[QuantParameters], names: List[str]):
        """receive_mean's common case in a few native calls: K updates of one model whose entries come in the
        same order and whose every non-empty ndim > 1 entry is a pair of contiguous CPU byte planes of one
        element count and, across updates, one shape. Returns (those names, their means), or None when the
        updates are anything else (receive_mean then classifies entry by entry)."""
        if any(list(c.params.keys()) != names for c in all_c_params):
            return None
        th = _torchhost.get()
        ps = [list(c.params.values()) for c in all_c_params]
        datas = [[p.data for p in c] for c in ps]
        metas = [th.tensor_meta(d) for d in datas]
        ndim, numel = metas[0][0].numpy(), metas[0][1].numpy()
        if any(not (torch.equal(m[0], metas[0][0]) and torch.equal(m[1], metas[0][1])) for m in metas):
            return None
        idx = np.nonzero((ndim > 1) & (numel > 0))[0].tolist()
        if not idx:
            return [], []
        lv = [[d[i] for i in idx] for d in datas]
        sg = [[c[i].signs for i in idx] for c in ps]
        lvm = [th.byte_planes(x) for x in lv]
        sgm = [th.byte_planes(x) for x in sg]
        n0 = lvm[0][1]
        if not all(a[0] and b[0] and torch.equal(a[1], n0) and torch.equal(b[1], n0) for a, b in zip(lvm, sgm)):
            return None
        if not th.shapes_equal(lv):
            return None
        norms = torch.tensor([[float(c[i].scale) for i in idx] for c in ps], dtype=torch.float32)
        mins = (torch.tensor([[float(c[i].scale_2) for i in idx] for c in ps], dtype=torch.float32)
                if self.CODEC == "rqsgd" else None)
        means = _decode_mean_stoch_host(lv[0], n0, [m[2].numpy().view(np.uint64) for m in lvm],
                                        [m[2].numpy().view(np.uint64) for m in sgm], norms, mins, self.CODEC,
                                        self.bits)
        return [names[i] for i in idx], means

    @staticmethod
    def _fusable(p: QuantParameter) -> bool:
        """An entry _receive decodes (_decode_stoch's inputs: byte planes of one size, a numeric norm)."""
        d, g = p.data, p.signs
        return (isinstance(d, torch.Tensor) and isinstance(g, torch.Tensor) and d.ndim > 1 and d.numel() > 0
                and d.element_size() == 1 and not d.is_quantized and not d.is_floating_point()
                and g.numel() == d.numel() and g.element_size() == 1 and not g.is_floating_point()
                and d.is_cuda == g.is_cuda)

    def _quantize_params(self, params: Parameters, bits: int, uniforms=None, seed=None) -> QuantParameters:
        """Biases and running metrics (ndim <= 1) are not quantized."""
        items = list(params.items())
        # every entry's ndim / numel / dtype in one native call (adfl_torchhost.tensor_meta)
        ndim, numel, is_f32, _ = (a.numpy() for a in _torchhost.get().tensor_meta([t for _, t in items]))
        coded = (ndim > 1) & (numel > 0)
        names = [items[i][0] for i in np.nonzero(coded)[0].tolist()]
        f32 = [items[i][0] for i in np.nonzero(coded & is_f32)[0].tolist()]
        for i in np.nonzero(coded & ~is_f32)[0].tolist():
            _require_codable(items[i][0], items[i][1], self.__class__.__name__)
        if uniforms is not None and {params[n].dtype for n in names} - {uniforms.dtype}:
            raise ValueError(f"{self.__class__.__name__}: injected uniforms ({uniforms.dtype}) cover one dtype bucket; "
                             f"this dict also holds {sorted(str(d) for d in {params[n].dtype for n in names})}")
        tn = reference_norm()
        qp = QuantParameter
        made: Dict[str, QuantParameter] = {}
        size = [0]
        f32_numel = numel[coded & is_f32].tolist()

        def emit(k, data, signs):   # an encoded fp32 entry, built as soon as its planes exist; scale set below
            n = f32[k]
            p = params[n]
            made[n] = qp(data, bits, 0, signs, p.shape, p.dtype, data.dtype, 0)
            size[0] += f32_numel[k]   # one byte per element

        pass_signs = torch.zeros(1, dtype=torch.uint8)  # passthrough entries' unused signs, one per call
        rest = iter([items[i] for i in np.nonzero(ndim <= 1)[0].tolist()])

        def idle(batch=32):   # passthrough entries, a batch per staging range
            for _ in range(batch):
                e = next(rest, None)
                if e is None:
                    return False
                t = e[1]
                made[e[0]] = qp(t, bits, 0, pass_signs, t.shape, t.dtype, t.dtype, 0)
                size[0] += t.nbytes
            return True

        encoded = (_encode_stoch(params, f32, self.CODEC, bits, uniforms if uniforms is None or
                                 uniforms.dtype == torch.float32 else None, seed, tn, emit=emit, idle=idle)
                   if f32 else {})
        if len(f32) < len(names):
            for dtype in sops.DT_DTYPES:   # fp16 / bf16 / fp64: one bucket per dtype, in that dtype's arithmetic
                group = [n for n in names if params[n].dtype == dtype]
                if group:
                    encoded.update(_encode_stoch_dt(params, group, self.CODEC, bits, uniforms, seed, tn))
        for name, param in items:
            o = made.get(name)
            e = encoded.get(name)
            if e is not None:
                data, signs, scale, scale_2 = e
                if o is None:
                    made[name] = qp(data, bits, scale, signs, param.shape, param.dtype, data.dtype, scale_2)
                    size[0] += data.nbytes
                else:   # built while the copies ran: its scale now (and the zero-norm branch's uint8 view)
                    if data is not o.data:
                        o.data, o.q_dtype = data, data.dtype
                    o.scale, o.scale_2 = scale, scale_2
            elif o is None:
                if param.ndim > 1:  # empty: vector_norm is 0 -> zero branch
                    _require_codable(name, param, self.__class__.__name__)
                    data = torch.zeros_like(param, dtype=torch.uint8)
                    made[name] = qp(data, bits, torch.tensor(0.0, dtype=param.dtype),
                                    torch.ones_like(param, dtype=torch.int8), param.shape, param.dtype, data.dtype, 0)
                else:
                    made[name] = qp(param, bits, 0, pass_signs, param.shape, param.dtype, param.dtype, 0)
                size[0] += made[name].data.nbytes
        return QuantParameters({name: made[name] for name in params}, size[0])


class QSGDChannel(_StochChannel):
    """Bi-directional QSGD (quant.py:140-252) on the MI355X HIP codec."""

    CODEC = "qsgd"


class RQSGDChannel(_StochChannel):
    """Bi-directional revised QSGD (quant.py:280-398): infinity norm, minimum factor for zero levels."""

    CODEC = "rqsgd"
    NORM_BYTES = 8


class CNATChannel(_StochChannel):
    """Bi-directional natural compression (quant.py:426-545): stochastic power-of-two exponents."""

    CODEC = "cnat"


class _Unidirectional:
    """Only client -> server is compressed; server -> client and the client's receive use the identity
    channel (quant.py:255-277,401-423,548-570)."""

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return IdentityChannel(no_compute_time=True).on_server_send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return IdentityChannel(no_compute_time=True).on_client_receive(c_params)


class UQSGDChannel(_Unidirectional, QSGDChannel):
    """Uni-directional QSGD (quant.py:255-277)."""


class URQSGDChannel(_Unidirectional, RQSGDChannel):
    """Uni-directional RQSGD (quant.py:401-423)."""


class UCNATChannel(_Unidirectional, CNATChannel):
    """Uni-directional CNAT (quant.py:548-570)."""
