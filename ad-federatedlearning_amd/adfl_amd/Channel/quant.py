"""SLQ channels backed by the MI355X HIP codec — drop-in for ``Src/ADFL/Channel/quant.py:15-137``.

``SLQChannel`` / ``USLQChannel`` keep the reference's names, constructor, six-method surface,
``to_json`` output, ``simulate_bandwidth`` formula, payload types and error behaviour. What changes is
where the arithmetic runs: the reference loops over the state dict calling ATen CPU ops per tensor
(quant.py:74-112); here the whole dict is packed back to back into one flat buffer, moved to
the GPU once, encoded by two HIP launches (absmax partials -> scale + quantize, per-tensor scales),
and the int8 payload comes back in one copy. Decode is one HIP launch. Output is bit-identical to the
reference: int8 payload, fp32 scale and dequantized floats (tests/golden).

Contract kept from the reference:
* inputs are CPU tensors (callers ``.cpu()``, Src/ADFL/model.py:195-197) — CUDA tensors are also
  accepted and then stay on the device;
* ``ndim <= 1`` tensors pass through untouched with ``scale = 1`` (quant.py:80-81, same object);
* ``QuantParameter.data`` is a ``torch.qint8`` tensor (zero point 0) and ``scale`` a Python float;
* decode returns new, owned, writable fp32 tensors (strategies mutate them in place);
* a non-fp32 ``ndim > 1`` tensor raises ``RuntimeError: Quantize only works on Float Tensor, got …``;
  an empty one raises torch.max's ``RuntimeError``; ``_receive`` asserts ``QuantParameters``;
* the channel object holds no device state (it is pickled into every Ray actor): buffers live in a
  per-process, per-device cache created lazily on first use.

There is no CPU fallback: without a GPU and the built HIP library these methods raise.
"""

import ctypes
import os
import threading
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _lib, _torchhost, hostcopy, ops, qerror, sum_order
from .._lib import check
from ..model import (CompressedParameters, Parameters, QuantParameter, QuantParameters, get_parameter_info)
from .channel import Channel, IdentityChannel

_LAYOUT_CACHE_MAX = 16


class _DeviceStaging:
    """Per-process, per-device reusable buffers (pinned host + device), grown on demand."""

    def __init__(self, device: torch.device):
        self.device = device
        self.cpus = hostcopy.bind_to_device(device)   # the copy pool on the GPU's NUMA node
        self.lock = threading.RLock()
        self._bufs: Dict[str, torch.Tensor] = {}
        self.layouts: "OrderedDict[Tuple[int, ...], ops.BucketLayout]" = OrderedDict()
        self._d2h: Optional[torch.cuda.Stream] = None
        self._h2d: Optional[torch.cuda.Stream] = None
        self._events: List[int] = []

    def d2h_stream(self) -> torch.cuda.Stream:
        """The range-pipelined host paths' copy-back stream: a range's D2H runs here, behind an event on the
        compute stream, so it overlaps the next range's H2D (one stream would serialise them)."""
        if self._d2h is None:
            self._d2h = torch.cuda.Stream(self.device)
        return self._d2h

    def h2d_stream(self) -> torch.cuda.Stream:
        """The stochastic host encode's staging stream: each range's H2D runs here and the compute stream waits
        only for the ranges its kernels read, so the copies run at the link's rate however long the calling
        thread spends on a range's kernels and outputs."""
        if self._h2d is None:
            self._h2d = torch.cuda.Stream(self.device)
        return self._h2d

    def events(self, n: int) -> List[int]:
        """n hipEvent_t handles (timing-free, on this device) for the range-pipelined host paths: a range's
        kernel-done and copied-back events (adfl_stage_*_range). Kept for the staging's life: every call waits
        for all its ranges' scatters before it returns, so the next call may record them again."""
        if len(self._events) < n:
            more = n - len(self._events)
            arr = (ctypes.c_void_p * more)()
            with torch.cuda.device(self.device):
                check(_lib.load().adfl_stage_events_create(more, arr))
            self._events.extend(int(a) for a in arr)
        return self._events

    def buf(self, key: str, numel: int, dtype: torch.dtype, pinned: bool = False) -> torch.Tensor:
        t = self._bufs.get(key)
        if t is None or t.numel() < numel:
            numel = max(numel, 1)
            if pinned:
                with hostcopy.on_cpus(self.cpus):   # pages on the GPU's NUMA node
                    t = torch.empty(numel, dtype=dtype, pin_memory=True)
            else:
                t = torch.empty(numel, dtype=dtype, device=self.device)
            self._bufs[key] = t
        return t[:numel]

    def layout(self, sizes: Tuple[int, ...], align: int = 1) -> ops.BucketLayout:
        """align=1: compact (the host gather is one concatenation); align=2 for packed int4 buckets."""
        key = (sizes, align)
        lay = self.layouts.get(key)
        if lay is None:
            lay = ops.BucketLayout(sizes, align=align)
            self.layouts[key] = lay
            if len(self.layouts) > _LAYOUT_CACHE_MAX:
                self.layouts.popitem(last=False)
        else:
            self.layouts.move_to_end(key)
        return lay


_STAGING: Dict[int, _DeviceStaging] = {}


_STAGING_LOCK = threading.Lock()


def _staging() -> _DeviceStaging:
    idx = torch.cuda.current_device()
    with _STAGING_LOCK:
        st = _STAGING.get(idx)
        if st is None:
            st = _DeviceStaging(torch.device("cuda", idx))
            _STAGING[idx] = st
    return st


def _serialized(fn):
    """Staging buffers are per device and reused: calls from several threads of one actor (ADFL's peer
    clients receive on one thread while training on another, Examples/ray_ad.py) take turns. (Running the
    calling thread on the GPU's NUMA node as well, not only the copy pool, measured no faster:
    profiles/r04/host_channel/caller_*.json.)"""
    def wrapper(*args, **kwargs):
        with _staging().lock:
            return fn(*args, **kwargs)
    wrapper.__name__, wrapper.__doc__ = fn.__name__, fn.__doc__
    return wrapper


def _gather(tensors: List[torch.Tensor], lay: ops.BucketLayout, out: torch.Tensor) -> None:
    """Copy `tensors` (all on out's device) into the 1-D bucket `out` at lay.offsets with ONE torch.cat
    (zero pads between tensors only for an aligned layout; the Channel's compact layout has none)."""
    if lay.align == 1:
        torch.cat([t.reshape(-1) for t in tensors], out=out)
        return
    zeros = torch.zeros(lay.align, dtype=out.dtype, device=out.device)
    pieces = []
    for t, n, padded in zip(tensors, lay.sizes.tolist(), lay.padded.tolist()):
        pieces.append(t.reshape(-1))
        if padded > n:
            pieces.append(zeros[:padded - n])
    torch.cat(pieces, out=out)


_PIECE_BYTES = 4 << 20  # staging pieces of at least this size: one gather + one H2D each
_PIECES = 8             # ... and at most this many per bucket


def _ranges(lay: ops.BucketLayout, elem_bytes: int) -> List[Tuple[int, int]]:
    """The bucket split into element ranges [lo, hi) of about max(_PIECE_BYTES, total / _PIECES) bytes.
    Ranges may cut through a tensor (one 1 GiB tensor still stages in pipelined pieces). Eight pieces: the
    copy engine starts after the first eighth is gathered, and the last eighth's copy is the exposed tail."""
    step = max(_PIECE_BYTES // elem_bytes, -(-lay.total // _PIECES))
    return [(lo, min(lo + step, lay.total)) for lo in range(0, lay.total, step)]


class _RangePlan:
    """For one layout and staging range [lo, hi): which tensor each copy piece belongs to, where it starts in
    that tensor and in the bucket, and its length — everything but the call's pointers, computed once per
    (layout, range) and cached on the layout (the per-call numpy work was ~20 us per range)."""

    __slots__ = ("k", "t_off", "b_off", "n", "ku")

    def __init__(self, lay: ops.BucketLayout, lo: int, hi: int):
        a = np.maximum(lay.offsets, lo)
        b = np.minimum(lay.offsets + lay.sizes, hi)
        k = np.nonzero(a < b)[0]
        self.k = k
        self.ku = k.astype(np.uint64)
        self.t_off = (a[k] - lay.offsets[k]).astype(np.uint64)
        self.b_off = a[k].astype(np.uint64)
        self.n = (b[k] - a[k]).astype(np.int64)

    def copies(self, ptrs: np.ndarray, base: int, es: int, to_bucket: bool):
        t_ptr = ptrs[self.k] + self.t_off * np.uint64(es)
        b_ptr = np.uint64(base) + self.b_off * np.uint64(es)
        nbytes = self.n * es
        return (b_ptr, t_ptr, nbytes) if to_bucket else (t_ptr, b_ptr, nbytes)


def _plan(lay: ops.BucketLayout, lo: int, hi: int) -> _RangePlan:
    cache = lay.__dict__.setdefault("_range_plans", {})
    p = cache.get((lo, hi))
    if p is None:
        p = cache[(lo, hi)] = _RangePlan(lay, lo, hi)
    return p


def _range_copies(ptrs: np.ndarray, lay: ops.BucketLayout, base: int, es: int, lo: int, hi: int, to_bucket: bool,
                  with_tensors: bool = False):
    """Byte-copy lists moving bucket elements [lo, hi) between the host bucket at `base` and the tensors
    whose data pointers are `ptrs` (tensor k at lay.offsets[k]; pads are never copied). with_tensors: the
    tensor index of every piece is returned too."""
    p = _plan(lay, lo, hi)
    out = p.copies(ptrs, base, es, to_bucket)
    return out + (p.k,) if with_tensors else out


ctypes_chunk_bytes = 24  # sizeof(adfl_slq_chunk)
_CHUNK_DT = np.dtype([("start", "<i8"), ("len", "<i4"), ("tensor", "<i4"), ("first_chunk", "<i4"),
                      ("nchunks", "<i4")])


class _ChunkMeta:
    """A layout's chunk table as arrays (cached on the layout): every chunk's [start, end) and, per tensor, its
    first chunk and one past its last — what the range-pipelined host paths launch chunk ranges with."""

    __slots__ = ("start", "end", "first", "cend")

    def __init__(self, lay: ops.BucketLayout):
        c = np.frombuffer(lay.chunks, dtype=_CHUNK_DT)
        self.start = c["start"].astype(np.int64)
        self.end = self.start + c["len"]
        t_first = np.zeros(lay.ntensors, dtype=np.int64)
        t_first[c["tensor"][c["first_chunk"] == np.arange(len(c))]] = np.nonzero(c["first_chunk"] == np.arange(len(c)))[0]
        self.first = t_first
        self.cend = t_first + c["nchunks"][t_first]


def _chunk_meta(lay: ops.BucketLayout) -> _ChunkMeta:
    m = lay.__dict__.get("_chunk_meta")
    if m is None:
        m = lay.__dict__["_chunk_meta"] = _ChunkMeta(lay)
    return m


def _ptrs(tensors: List[torch.Tensor]) -> np.ndarray:
    return np.fromiter((t.data_ptr() for t in tensors), dtype=np.uint64, count=len(tensors))


def _host_heap(lay: ops.BucketLayout) -> None:
    """A host-resident call: the process heap sized for this layout's fp32 outputs (hostcopy.keep_host_heap:
    raised only as layouts grow; ADFL_KEEP_HOST_HEAP=0 leaves the allocator alone). Device-resident callers
    never change the allocator."""
    hostcopy.keep_host_heap(4 * lay.total, 4 * int(lay.sizes.max()))


def _stage_in(tensors: List[torch.Tensor], lay: ops.BucketLayout, st: _DeviceStaging, key: str,
              dtype: torch.dtype, host_ptrs: Optional[np.ndarray] = None) -> torch.Tensor:
    """The bucket on the device: one gather + one H2D for CPU tensors, one device gather otherwise.
    host_ptrs: the tensors' data pointers when the caller knows them all to be contiguous CPU tensors of the
    bucket's element size (adfl_torchhost.qint8_meta checked them in one call)."""
    dev_buf = st.buf(key, lay.total, dtype)
    if host_ptrs is None and tensors and tensors[0].is_cuda:
        # a device dict: its pointers and sizes checked in one native call, then one gather launch
        ok, numel, dptrs = _torchhost.get().device_ptrs(tensors, st.device.index, dev_buf.element_size())
        if ok and np.array_equal(numel.numpy(), lay.sizes):
            ops.bucket_gather(tensors, lay, dev_buf, checked=False, ptrs=dptrs)
            return dev_buf
    kinds = {False} if host_ptrs is not None else {t.is_cuda for t in tensors}
    if kinds == {False}:
        _host_heap(lay)
        host = st.buf(key + "_host", lay.total, dtype, pinned=True)
        es = host.element_size()
        if host_ptrs is not None or all(t.is_contiguous() and t.element_size() == es for t in tensors):
            # Native parallel gather (csrc/host_copy.cpp) in element ranges, each range's H2D enqueued as
            # soon as it is staged so the copy engine overlaps the next range's host copy. Pads of an
            # aligned layout are never read.
            ptrs = _ptrs(tensors) if host_ptrs is None else host_ptrs
            for lo, hi in _ranges(lay, es):
                hostcopy.copy_pieces(*_range_copies(ptrs, lay, host.data_ptr(), es, lo, hi, to_bucket=True))
                dev_buf[lo:hi].copy_(host[lo:hi], non_blocking=True)
        else:
            _gather(tensors, lay, host)
            dev_buf.copy_(host, non_blocking=True)
    elif kinds == {True}:
        es = dev_buf.element_size()
        if all(t.device == st.device and t.is_contiguous() and t.element_size() == es and t.numel() == n
               for t, n in zip(tensors, lay.sizes.tolist())):
            # one launch; quantized payloads read from their storage (checked just above)
            ops.bucket_gather(tensors, lay, dev_buf, checked=False)
        else:
            _gather([t.to(st.device) for t in tensors], lay, dev_buf)
    else:  # mixed host / device dict: per-tensor copies (rare)
        for t, off, n in zip(tensors, lay.offsets.tolist(), lay.sizes.tolist()):
            dev_buf[off:off + n].view(t.shape).copy_(t)
    return dev_buf


_PIPELINE = os.environ.get("ADFL_HOST_PIPELINE", "1") != "0"


def _drain(*streams) -> None:
    """A pipelined host path that fails part-way (an output allocation, a caller's emit / idle callback, a
    native call) may leave H2D copies reading, and kernels and D2H copies writing, the staging buffers it
    shares with the next call (the pinned buckets, the device buckets): wait for every stream it enqueued on
    before the exception leaves, so the next call's gathers cannot overwrite a buffer still in use."""
    for s in streams:
        if s is not None:
            try:
                s.synchronize()
            except Exception:   # the original exception is the one to report
                pass


class PhaseClock:
    """Wall milliseconds the calling thread spends in each phase of the host-to-host path (exclusive, no extra
    synchronisation): filled while a `phase_clock()` block is active, e.g. bench.py's channel_c3_dict."""

    def __init__(self):
        self.ms: Dict[str, float] = {}


_CLOCK: Optional[PhaseClock] = None


class _Phase:
    __slots__ = ("name", "t0")

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        c = _CLOCK
        if c is not None:
            c.ms[self.name] = c.ms.get(self.name, 0.0) + (time.perf_counter() - self.t0) * 1e3


class _NoPhase:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return None


_NO_PHASE = _NoPhase()


def _ph(name: str):
    return _NO_PHASE if _CLOCK is None else _Phase(name)


class phase_clock:
    """`with phase_clock() as c:` — c.ms holds the phase split of the channel calls made inside."""

    def __enter__(self) -> PhaseClock:
        global _CLOCK
        self.prev = _CLOCK
        _CLOCK = PhaseClock()
        return _CLOCK

    def __exit__(self, *exc):
        global _CLOCK
        _CLOCK = self.prev


class _PendingD2H:
    """D2H of a device bucket into the reused pinned staging, enqueued range by range with an event each;
    finish() scatters every range into the per-tensor CPU storages as soon as its copy lands (the native
    pool copies while the copy engine moves the next range). Whatever the caller does between the two —
    allocating the output tensors — overlaps the copies."""

    def __init__(self, dev_buf: torch.Tensor, lay: ops.BucketLayout, st: _DeviceStaging, key: str):
        self.host = st.buf(key + "_host", lay.total, dev_buf.dtype, pinned=True)
        self.lay = lay
        stream = torch.cuda.current_stream(st.device)
        self.stream = stream
        self.ranges = _ranges(lay, self.host.element_size())
        self.events = []
        for lo, hi in self.ranges:
            self.host[lo:hi].copy_(dev_buf[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            self.events.append(ev)

    def finish_building(self, make, count: int, make_batch=None) -> List[torch.Tensor]:
        """Create the `count` outputs (make(k): a fresh contiguous CPU tensor for tensor k of the layout) in
        offset order while the D2H runs, and hand each staging range's scatter to the native pool as soon as
        its copy has landed and every output it touches exists; the pool copies while this thread goes on
        creating the next outputs (their creation was otherwise serial with the scatter). Returns the outputs
        once every byte has landed in them. ADFL_HOST_PIPELINE=0: create all, then finish() (the A/B)."""
        lay = self.lay
        offs = lay.offsets
        if make is None:  # batched creation only: make(k) from it when the slow path needs one
            make = lambda k: make_batch(k, k + 1)[0][0]  # noqa: E731
        if not _PIPELINE or count != lay.ntensors or (count > 1 and (np.diff(offs) < 0).any()):
            outs = [make(k) for k in range(count)]
            hostcopy.advise_huge(outs)
            self.finish(outs)
            return outs
        es = self.host.element_size()
        base = self.host.data_ptr()
        ptrs = np.zeros(count, dtype=np.uint64)
        outs: List[torch.Tensor] = []
        pending = []
        k = 0
        try:
            for (lo, hi), ev in zip(self.ranges, self.events):
                with _ph("out.alloc"):
                    if make_batch is not None:   # the range's new outputs in one native call (adfl_torchhost)
                        k_end = int(np.searchsorted(offs, hi, side="left"))
                        if k_end > k:
                            ts, pt = make_batch(k, k_end)
                            outs.extend(ts)
                            ptrs[k:k_end] = pt.numpy().view(np.uint64)
                            for j in np.nonzero(lay.sizes[k:k_end] * es >= (4 << 20))[0].tolist():
                                hostcopy.advise_huge([ts[j]])
                            k = k_end
                    while k < count and offs[k] < hi:   # every tensor the range [lo, hi) touches starts below hi
                        t = make(k)
                        if t.is_cuda or not t.is_contiguous() or t.element_size() != es:
                            raise ValueError("staging: outputs must be contiguous CPU tensors of the bucket's "
                                             "element size")
                        if t.numel() * es >= (4 << 20):
                            hostcopy.advise_huge([t])
                        ptrs[k] = t.data_ptr()
                        outs.append(t)
                        k += 1
                with _ph("out.d2h_wait"):
                    ev.synchronize()   # usually landed already: the outputs took longer than the copy
                with _ph("out.scatter_submit"):
                    pending.append(hostcopy.submit_pieces(*_range_copies(ptrs, lay, base, es, lo, hi,
                                                                         to_bucket=False),
                                                          stream=True, keep=self.host))
            while k < count:   # tensors past the last range (none for a bucket layout; kept for safety)
                outs.append(make(k))
                k += 1
        except BaseException:
            _drain(self.stream)
            raise
        finally:
            with _ph("out.scatter_wait"):
                for pd in pending:
                    pd.wait()
        return outs

    def finish(self, outs: List[torch.Tensor], ptrs: Optional[np.ndarray] = None) -> None:
        """outs: contiguous CPU tensors owned by the caller, tensor k receiving bucket elements at offsets[k].
        ptrs: their data pointers when the caller made them (adfl_torchhost) and knows them to fit."""
        es = self.host.element_size()
        if ptrs is None:
            for t in outs:
                if t.is_cuda or not t.is_contiguous() or t.element_size() != es:
                    raise ValueError("staging: outputs must be contiguous CPU tensors of the bucket's element size")
            ptrs = _ptrs(outs)
        for (lo, hi), ev in zip(self.ranges, self.events):
            ev.synchronize()
            hostcopy.copy_pieces(*_range_copies(ptrs, self.lay, self.host.data_ptr(), es, lo, hi, to_bucket=False),
                                 stream=True)


def _stage_out(dev_buf: torch.Tensor, lay: ops.BucketLayout, st: _DeviceStaging, key: str,
               outs: List[torch.Tensor]) -> None:
    """Copy the bucket `dev_buf` (on the device) into the per-tensor CPU storages `outs` (_PendingD2H)."""
    _PendingD2H(dev_buf, lay, st, key).finish(outs)


def _hand_out(out_dev: torch.Tensor, lay: ops.BucketLayout, shapes: List[torch.Size], on_cpu: List[bool],
              st: _DeviceStaging, key: str, like: Optional[List[torch.Tensor]] = None) -> List[torch.Tensor]:
    """Decoded tensors as the reference returns them (quant.py:107-112): one new, owned, writable tensor
    per entry — pageable CPU tensors for CPU payloads, device tensors for device payloads — never views
    of a shared bucket (a strategy keeps single updates alive, Src/ADFL/Strategy/fed_buff.py:75,90, and
    pickling one must not ship the whole bucket). For an all-CPU dict the D2H is enqueued first and the
    output tensors are allocated while it runs."""
    outs: List[Optional[torch.Tensor]] = [None] * len(shapes)
    if all(on_cpu):
        pending = _PendingD2H(out_dev, lay, st, key)
        dt = out_dev.dtype
        if like is not None and dt == torch.float32:   # `like`: tensors of the outputs' shapes (the payloads)
            th = _torchhost.get()
            return pending.finish_building(None, len(shapes), make_batch=lambda a, b: th.empty_f32_like(like[a:b]))
        return pending.finish_building(lambda k: torch.empty(shapes[k], dtype=dt), len(shapes))
    if not any(on_cpu) and out_dev.device == st.device:
        # device dict: fresh owned tensors filled from the bucket by one launch (not one clone per tensor)
        th = _torchhost.get()
        if (like is not None and out_dev.dtype == torch.float32
                and th.device_ptrs(like, st.device.index, like[0].element_size())[0]):
            dev_outs, ptrs = th.empty_f32_like(like)   # one native call, on like's (= the staging's) device
            ops.bucket_scatter(out_dev, lay, dev_outs, checked=False, ptrs=ptrs)
        else:
            dev_outs = [torch.empty(s, dtype=out_dev.dtype, device=st.device) for s in shapes]
            ops.bucket_scatter(out_dev, lay, dev_outs, checked=False)
        torch.cuda.current_stream(st.device).synchronize()
        return dev_outs
    for i, (off, n, s) in enumerate(zip(lay.offsets.tolist(), lay.sizes.tolist(), shapes)):
        if on_cpu[i]:  # mixed host / device dict (rare): per-tensor copies
            outs[i] = torch.empty(s, dtype=out_dev.dtype)
            outs[i].view(-1).copy_(out_dev[off:off + n])
        else:
            outs[i] = out_dev[off:off + n].view(s).clone()
    torch.cuda.current_stream(st.device).synchronize()
    return outs


def _host_scales(amax_bits: np.ndarray, bits: int) -> np.ndarray:
    """fp32(max|x| / q_max) from the magnitude bits the staging gather reduced (quant.py:99-100: fp32 tensor
    math, correctly rounded; a NaN magnitude gives a NaN scale) — what the device encode computes."""
    return (amax_bits.view(np.float32) / np.float32((1 << (bits - 1)) - 1)).astype(np.float32)


def _qerror_sums(x_dev: torch.Tensor, d_dev: torch.Tensor, lay: ops.BucketLayout):
    """The reference's q-error sums of a bucket against its decode (qerror.reference_sums): over the
    tensors back to back, so a padded layout (int4 buckets: align 2) is compacted first."""
    sizes = lay.sizes.tolist()
    if (lay.offsets != np.concatenate([[0], np.cumsum(lay.sizes)[:-1]])).any():
        x_dev = torch.cat([x_dev[o:o + n] for o, n in zip(lay.offsets.tolist(), sizes)])
        d_dev = torch.cat([d_dev[o:o + n] for o, n in zip(lay.offsets.tolist(), sizes)])
    return qerror.reference_sums(x_dev, d_dev, sizes)


def _encode_host_dict(tensors: List[torch.Tensor], lay: ops.BucketLayout, st: _DeviceStaging, bits: int,
                      stats: Optional[list], emit, idle):
    """The all-CPU fp32 dict's encode, pipelined range by range across the host, the link and the GPU.

    The gather into the pinned bucket is queued on the native pool range by range. As each range lands (the
    thread enqueues every landed range before it builds outputs), one native call (adfl_stage_encode_range)
    enqueues its H2D and, for the tensors whose every byte is now staged, the device's absmax and quantize
    over their chunks (adfl_slq_absmax_batched_range + adfl_slq_quantize_batched_range: the two-pass encode's
    kernels, so the same payload and scales), then their payload bytes' D2H on a side stream behind an event.
    The D2H and scatter of range r overlap the H2D of range r + 1.
    The outputs are built while the copies run: the gather also reduces max|x| per tensor as it copies
    (adfl_host_copy_submit_absmax), so the host knows each scale in time to create the qint8 outputs (one
    native call per range) and emit(k, q, scale) each payload object, and the scatter into them is queued on
    the pool behind the range's event. `idle()` (the caller's other payload objects) runs in between. The
    payload bytes and scales are the device's: its scales are compared with the host's at the end and any
    output whose host scale differed is rebuilt with the device's. Returns [(q, scale)] per tensor."""
    with _ph("enc.heap"):
        _host_heap(lay)
    dev = st.device
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    lib = _lib.load()
    x_dev = st.buf("x", lay.total, torch.float32)
    host = st.buf("x_host", lay.total, torch.float32, pinned=True)
    q_dev = st.buf("q", lay.total, torch.int8)
    q_host = st.buf("q_host", lay.total, torch.int8, pinned=True)
    s_dev = st.buf("scales", lay.ntensors, torch.float32)
    part_dev = st.buf("partials", lay.nchunks, torch.int32)
    chunks_ptr = lay.device_chunks(dev).data_ptr()
    d2h = st.d2h_stream()
    cm = _chunk_meta(lay)
    amax = np.zeros(lay.ntensors, dtype=np.uint32)
    a_base = amax.ctypes.data
    th = _torchhost.get()
    ptrs = th.data_ptrs(tensors).numpy().view(np.uint64)
    ranges = _ranges(lay, 4)
    evs = st.events(2 * len(ranges))
    d2h_h = d2h.cuda_stream
    hx, dx, qd, qh = host.data_ptr(), x_dev.data_ptr(), q_dev.data_ptr(), q_host.data_ptr()
    pd, sd = part_dev.data_ptr(), s_dev.data_ptr()
    jobs = []
    with _ph("enc.gather_submit"):
        for lo, hi in ranges:
            plan = _plan(lay, lo, hi)
            b_ptr, t_ptr, nb = plan.copies(ptrs, host.data_ptr(), 4, True)
            jobs.append(hostcopy.submit_pieces(b_ptr, t_ptr, nb,
                                               absmax_ptrs=np.uint64(a_base) + plan.ku * np.uint64(4),
                                               keep=(host, amax)))
    ends = lay.offsets + lay.sizes
    outs: List[torch.Tensor] = []
    out_ptrs = np.zeros(lay.ntensors, dtype=np.uint64)
    scales = np.zeros(lay.ntensors, dtype=np.float32)
    scatters = []
    made = 0
    staged: List[Tuple[int, int, int, int, int]] = []   # ranges on the device whose outputs are not built yet
    r = 0
    try:
        while r < len(ranges) or staged:
            # every range whose gather has landed goes to the device at once (the link, not this thread, then
            # paces the H2D); the thread waits on a gather only when it has no outputs left to build
            while r < len(ranges) and (not staged or jobs[r].done()):
                lo, hi = ranges[r]
                with _ph("enc.gather_absmax_wait"):
                    jobs[r].wait()
                done = int(np.searchsorted(ends, hi, side="right"))   # tensors whose every byte is staged
                with _ph("enc.kernel_launch"):
                    # one native call: the range's H2D; the device's absmax and quantize of the tensors it
                    # completes; their payload bytes back D2H on the side stream behind an event (host_stage.hip)
                    c0 = c1 = e0 = e1 = 0
                    if done > made:
                        c0, c1 = int(cm.first[made]), int(cm.cend[done - 1])
                        e0, e1 = int(lay.offsets[made]), int(ends[done - 1])
                    check(lib.adfl_stage_encode_range(hx, dx, lo, hi, pd, chunks_ptr, c0, c1 - c0, bits, qd, sd, qh,
                                                      e0, e1, sh, d2h_h, evs[2 * r], evs[2 * r + 1]))
                if done > made:
                    staged.append((made, done, e0, e1, evs[2 * r + 1]))
                    made = done
                r += 1
            if not staged:
                continue
            t0, t1, e0, e1, ev = staged.pop(0)
            with _ph("enc.outputs"):
                scales[t0:t1] = _host_scales(amax[t0:t1], bits)
                # the range's payload tensors in one native call (adfl_torchhost): the qint8 tensors
                # torch.quantize_per_tensor(x, scale, 0, torch.qint8) would return, still to be filled
                qs, qp = th.empty_qint8_like(tensors[t0:t1], torch.from_numpy(scales[t0:t1]))
                out_ptrs[t0:t1] = qp.numpy().view(np.uint64)
                sl = scales[t0:t1].tolist()
                for j, q in enumerate(qs):
                    outs.append(q)
                    emit(t0 + j, q, sl[j])
            with _ph("enc.scatter_submit"):
                scatters.append(hostcopy.submit_pieces(
                    *_range_copies(out_ptrs, lay, q_host.data_ptr(), 1, e0, e1, to_bucket=False),
                    stream=True, event=ev, keep=q_host))
            with _ph("enc.passthrough"):
                idle()
    except BaseException:
        _drain(stream, d2h)
        raise
    finally:
        for j in jobs:
            j.wait()
        with _ph("enc.scatter_wait"):
            for j in scatters:
                j.wait()
    if stats is not None:
        stats.append(_qerror_sums(x_dev, ops.decode_batched(q_dev, s_dev, lay, out=st.buf("qe_d", lay.total, torch.float32)),
                                  lay))
    scales_host = st.buf("scales_host", lay.ntensors, torch.float32, pinned=True)
    scales_host.copy_(s_dev, non_blocking=True)
    scales_ready = torch.cuda.Event()
    scales_ready.record(stream)
    with _ph("enc.passthrough"):
        while idle():   # the caller's remaining objects
            pass
    scales_ready.synchronize()
    dev_scales = scales_host.numpy()
    bad = np.nonzero(dev_scales.view(np.uint32) != scales.view(np.uint32))[0]
    res = [(q, float(sc)) for q, sc in zip(outs, scales)]
    for k in bad.tolist():   # never seen (both reduce the same magnitude bits and divide correctly rounded):
        # the device's scale is the one the payload was quantized with
        sc = float(dev_scales[k])
        q = torch._make_per_tensor_quantized_tensor(_int8_view(outs[k]), sc, 0)
        res[k] = (q, sc)
        emit(k, q, sc)
    return res


@_serialized
def _encode_dict(params: Parameters, names: List[str], bits: int, stats: Optional[list] = None,
                 emit=None, idle=None, meta=None):
    """Encode the ndim>1 tensors `names` of `params` in one bucketed pass.

    Returns {name: (qint8 tensor on the input's device, python float scale)}. With `stats` (a list), the
    four q-error sums of the bucket against its payload are appended to it (ops.qerror_batched). For a dict
    of contiguous CPU fp32 tensors the outputs are built while the copies run (_encode_host_dict): emit(k, q,
    scale) is called for each as it is created and idle() (returning True while it has work left) between
    the copy ranges."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    # meta: (sizes, all contiguous CPU) from _quantize_params' native scan (every tensor already fp32)
    lay = st.layout(meta[0] if meta is not None else tuple(int(t.numel()) for t in tensors))
    all_host = meta[1] if meta is not None else all(not t.is_cuda and t.is_contiguous() for t in tensors)
    if _PIPELINE and all_host and (meta is not None or all(t.dtype == torch.float32 for t in tensors)):
        res = _encode_host_dict(tensors, lay, st, bits, stats, emit or (lambda k, q, sc: None),
                                idle or (lambda: False))
        return {name: r for name, r in zip(names, res)}
    x_dev = _stage_in(tensors, lay, st, "x", torch.float32)
    q_dev, s_dev = ops.encode_batched(x_dev, lay, bits, q=st.buf("q", lay.total, torch.int8),
                                      scales=st.buf("scales", lay.ntensors, torch.float32),
                                      partials=st.buf("partials", lay.nchunks, torch.int32))
    if stats is not None:
        stats.append(_qerror_sums(x_dev, ops.decode_batched(q_dev, s_dev, lay, out=st.buf("qe_d", lay.total, torch.float32)),
                                  lay))
    scales_host = st.buf("scales_host", lay.ntensors, torch.float32, pinned=True)
    scales_host.copy_(s_dev, non_blocking=True)
    on_cpu = [not t.is_cuda for t in tensors]
    if all(on_cpu):
        # every payload tensor owns its bytes (compact pickles; the staging buffer is reused by the next
        # call): the payload D2H is enqueued right behind the scales, and the qint8 tensors (which need the
        # scales) are allocated while it runs, then filled by the native scatter as its ranges land
        scales_ready = torch.cuda.Event()
        scales_ready.record(torch.cuda.current_stream(dev))
        pending = _PendingD2H(q_dev, lay, st, "q")
        scales_ready.synchronize()
        scales = scales_host.tolist()
        eaq, qint8 = torch._empty_affine_quantized, torch.qint8
        qs = pending.finish_building(
            lambda k: eaq(tensors[k].shape, scale=scales[k], zero_point=0, dtype=qint8), len(tensors))
        return {name: (qt, sc) for name, qt, sc in zip(names, qs, scales)}
    torch.cuda.current_stream(dev).synchronize()
    scales = scales_host.tolist()
    if not any(on_cpu) and all(t.device == dev for t in tensors):
        # device dict: the qint8 payloads allocated by one native call (on the tensors' device, no launch each)
        # and filled from the bucket by one launch
        qs, qp = _torchhost.get().empty_qint8_like(tensors, scales_host)
        ops.bucket_scatter(q_dev, lay, qs, checked=False, ptrs=qp)
        torch.cuda.current_stream(dev).synchronize()
        return {name: (qt, sc) for name, qt, sc in zip(names, qs, scales)}
    out = {}
    offs, sizes = lay.offsets.tolist(), lay.sizes.tolist()
    for i, (name, t) in enumerate(zip(names, tensors)):
        src = q_dev[offs[i]:offs[i] + sizes[i]].view(t.shape)
        if on_cpu[i]:
            src = src.cpu()
        # _make_per_tensor_quantized_tensor copies into a fresh qint8 storage of the source's device
        out[name] = (torch._make_per_tensor_quantized_tensor(src, scales[i], 0), scales[i])
    return out


def _int8_view(q: torch.Tensor) -> torch.Tensor:
    """The int8 bytes of a qint8 tensor without the copy `int_repr()` makes."""
    return torch.empty(0, dtype=torch.int8, device=q.device).set_(q.untyped_storage(), q.storage_offset(),
                                                                  q.shape, q.stride())


@_serialized
def _decode_dict(items: List[Tuple[str, torch.Tensor]], idle=None) -> Dict[str, torch.Tensor]:
    """Decode qint8 tensors (per-tensor affine, zero point 0) in one bucketed pass. idle(): the caller's
    other entries, run by the pipelined host path while its last copies are in flight (else not at all)."""
    st = _staging()
    dev = st.device
    qlist = [q for _, q in items]
    with _ph("dec.meta"):
        # every payload's quantizer, size, place and data pointer in one native call (adfl_torchhost)
        ok, all_host, numel, scales, ptrs = _torchhost.get().qint8_meta(qlist)
    if not ok:
        qint8, pta = torch.qint8, torch.per_tensor_affine
        for name, q in items:
            if not q.is_quantized or q.dtype != qint8 or q.qscheme() != pta or q.q_zero_point() != 0:
                raise ValueError(f"SLQChannel: '{name}' is not a per-tensor qint8 payload with zero point 0")
    lay = st.layout(tuple(numel.tolist()))
    if all_host and _PIPELINE:
        decoded = _decode_host_dict(qlist, lay, st, ptrs.numpy().view(np.uint64), scales, idle)
        return {name: t for (name, _), t in zip(items, decoded)}
    # CPU qint8 payloads are gathered byte-wise straight from their storage; device ones through int8 views
    all_dev = not all_host and all(q.is_cuda and q.device == dev and q.is_contiguous() for q in qlist)
    # host payloads are gathered byte-wise from their storages, device ones by one gather launch: neither
    # needs an int8 view object per tensor
    qs = qlist if all_host or all_dev else [_int8_view(q) for q in qlist]
    with _ph("dec.gather_h2d"):
        q_dev = _stage_in(qs, lay, st, "dq", torch.int8, host_ptrs=ptrs.numpy().view(np.uint64) if all_host else None)
    with _ph("dec.scales"):
        # q_scale() is a double; fbgemm's dequantize uses it as fp32 (quant.py:110): qint8_meta rounded it so
        s_dev = scales.to(dev, non_blocking=True)
    on_cpu = [True] * len(qlist) if all_host else [not q.is_cuda for q in qlist]
    with _ph("dec.kernel_launch"):
        out_dev = ops.decode_batched(q_dev, s_dev, lay, out=st.buf("d_out", lay.total, torch.float32))
    decoded = _hand_out(out_dev, lay, [q.shape for q in qlist] if not all_host else [None] * len(qlist), on_cpu, st,
                        "d_out", like=qlist if all_host or all_dev else None)
    return {name: t for (name, _), t in zip(items, decoded)}


def _decode_host_dict(qlist: List[torch.Tensor], lay: ops.BucketLayout, st: _DeviceStaging, ptrs: np.ndarray,
                      scales: torch.Tensor, idle=None) -> List[torch.Tensor]:
    """CPU qint8 payloads -> owned CPU fp32 tensors, pipelined range by range: the byte gather of every range
    is queued on the native pool at once; as range r lands, its H2D is enqueued, the chunks it completes are
    decoded (adfl_slq_dequantize_batched on that chunk range), their floats go back D2H behind an event, the
    outputs of the tensors they reach are created (one native call) and the scatter is queued on the pool
    behind the event — so the D2H of range r overlaps the H2D of range r + 1 and the scatters overlap the
    D2H. Bit-identical to the one-launch decode (each chunk is decoded by the same kernel)."""
    with _ph("dec.heap"):
        _host_heap(lay)
    dev = st.device
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    lib = _lib.load()
    q_dev = st.buf("dq", lay.total, torch.int8)
    q_host = st.buf("dq_host", lay.total, torch.int8, pinned=True)
    out_dev = st.buf("d_out", lay.total, torch.float32)
    out_host = st.buf("d_out_host", lay.total, torch.float32, pinned=True)
    chunks_ptr = lay.device_chunks(dev).data_ptr()
    d2h = st.d2h_stream()
    cm = _chunk_meta(lay)
    th = _torchhost.get()
    ranges = _ranges(lay, 4)
    evs = st.events(2 * len(ranges))
    d2h_h = d2h.cuda_stream
    qh, qd, od, oh = q_host.data_ptr(), q_dev.data_ptr(), out_dev.data_ptr(), out_host.data_ptr()
    with _ph("dec.gather_submit"):
        jobs = [hostcopy.submit_pieces(*_range_copies(ptrs, lay, q_host.data_ptr(), 1, lo, hi, to_bucket=True),
                                       keep=q_host) for lo, hi in ranges]
    with _ph("dec.scales"):
        s_dev = scales.to(dev, non_blocking=True)
    offs = lay.offsets
    outs: List[torch.Tensor] = []
    out_ptrs = np.zeros(lay.ntensors, dtype=np.uint64)
    scatters = []
    c_made = 0
    t_made = 0
    try:
        sd = s_dev.data_ptr()
        for r, ((lo, hi), job) in enumerate(zip(ranges, jobs)):
            with _ph("dec.gather_wait"):
                job.wait()
            with _ph("dec.kernel_launch"):
                # one native call: the range's H2D; the decode of the chunks it completes; their floats back
                # D2H on the side stream behind an event (host_stage.hip)
                c_end = int(np.searchsorted(cm.end, hi, side="right"))   # chunks whose every byte is staged
                if c_end <= c_made:
                    check(lib.adfl_stage_decode_range(qh, qd, lo, hi, chunks_ptr, 0, 0, sd, od, oh, 0, 0, sh, d2h_h,
                                                      evs[2 * r], evs[2 * r + 1]))
                    continue
                e0, e1 = int(cm.start[c_made]), int(cm.end[c_end - 1])
                check(lib.adfl_stage_decode_range(qh, qd, lo, hi, chunks_ptr, c_made, c_end - c_made, sd, od, oh, e0,
                                                  e1, sh, d2h_h, evs[2 * r], evs[2 * r + 1]))
                ev = evs[2 * r + 1]
                c_made = c_end
            with _ph("out.alloc"):
                t_end = int(np.searchsorted(offs, e1, side="left"))    # tensors starting below e1
                if t_end > t_made:
                    ts, pt = th.empty_f32_like(qlist[t_made:t_end])
                    outs.extend(ts)
                    out_ptrs[t_made:t_end] = pt.numpy().view(np.uint64)
                    for j in np.nonzero(lay.sizes[t_made:t_end] * 4 >= (4 << 20))[0].tolist():
                        hostcopy.advise_huge([ts[j]])
                    t_made = t_end
            with _ph("out.scatter_submit"):
                scatters.append(hostcopy.submit_pieces(
                    *_range_copies(out_ptrs, lay, out_host.data_ptr(), 4, e0, e1, to_bucket=False),
                    stream=True, event=ev, keep=out_host))
        if idle is not None:
            with _ph("dec.passthrough"):
                idle()
    except BaseException:
        _drain(stream, d2h)
        raise
    finally:
        for j in jobs:
            j.wait()
        with _ph("out.scatter_wait"):
            for j in scatters:
                j.wait()
    return outs


@_serialized
def _decode_add(c_params: QuantParameters, names: List[str], targets: List[Parameters]) -> None:
    """Stage the qint8 payloads of `names` into an aligned bucket and accumulate them into every target."""
    st = _staging()
    dev = st.device
    qs = [c_params.params[n].data for n in names]
    for n, q in zip(names, qs):
        if q.qscheme() != torch.per_tensor_affine or q.dtype != torch.qint8 or q.q_zero_point() != 0:
            raise ValueError(f"SLQChannel: '{n}' is not a per-tensor qint8 payload with zero point 0")
    lay = st.layout(tuple(int(q.numel()) for q in qs), align=ops.ALIGN_ELEMS)
    q_dev = _stage_in([_int8_view(q) for q in qs], lay, st, "aq", torch.int8)
    s_dev = torch.tensor([q.q_scale() for q in qs], dtype=torch.float32).to(dev, non_blocking=True)
    with torch.no_grad():
        ops.dequantize_add_batched(q_dev, s_dev, lay, [[t[n] for n in names] for t in targets])
    # the next call's host gather rewrites the pinned staging this call's H2D reads from
    torch.cuda.current_stream(dev).synchronize()


def _stage_rows(clients: List[List[torch.Tensor]], lay: ops.BucketLayout, st: _DeviceStaging,
                key: str) -> torch.Tensor:
    """K clients' payload tensors of one byte per element (int8 / uint8 / qint8; client k's tensor j at
    lay.offsets[j]) -> device rows [K, pad16(lay.total)] uint8. All on the CPU: one native gather per
    client into its pinned row, that row's H2D enqueued as soon as it is staged (the copy engine overlaps
    the next client's gather)."""
    k = len(clients)
    row = (lay.total + 15) // 16 * 16
    dev = st.buf(key, k * row, torch.uint8).view(k, row)
    if all(not t.is_cuda and t.is_contiguous() and t.element_size() == 1 for c in clients for t in c):
        # byte copies from the tensors' storages: qint8 payloads need no int8 view object here
        host = st.buf(key + "_host", k * row, torch.uint8, pinned=True).view(k, row)
        for r, c in enumerate(clients):
            hostcopy.copy_pieces(*_range_copies(_ptrs(c), lay, host[r].data_ptr(), 1, 0, lay.total, to_bucket=True))
            dev[r].copy_(host[r], non_blocking=True)
    elif all(t.device == st.device and t.is_contiguous() and t.element_size() == 1 and t.numel() == n
             for c in clients for t, n in zip(c, lay.sizes.tolist())):
        for r, c in enumerate(clients):   # device payloads: one gather launch per client row
            ops.bucket_gather(c, lay, dev[r], checked=False)
    else:  # mixed payloads: per-tensor copies into the device rows
        for r, c in enumerate(clients):
            for t, off, n in zip(c, lay.offsets.tolist(), lay.sizes.tolist()):
                dev[r, off:off + n].copy_(_byte_view(t).reshape(-1).to(st.device))
    return dev


def _byte_view(t: torch.Tensor) -> torch.Tensor:
    """The bytes of an int8 / uint8 / qint8 tensor as a uint8 tensor over the same storage."""
    if t.is_quantized:
        t = _int8_view(t)
    return t if t.dtype == torch.uint8 else t.view(torch.uint8)


@_serialized
def _decode_mean(clients: List[List[torch.Tensor]], scales: List[List[float]], shapes: List[torch.Size],
                 packed: bool) -> List[torch.Tensor]:
    """The fp32 mean over K clients of their decoded tensors, tensor by tensor, in torch's CPU summation
    order for simple_aggregate (csrc/torch_sum_order.h), in ONE launch (ops.dequantize_mean_batched): clients[k][j] is client k's payload for tensor j (a qint8 tensor,
    or ceil(n/2) packed int8 bytes with packed=True), scales[k][j] its scale. Returns one
    owned tensor per entry (CPU when every client's payload is on the CPU)."""
    st = _staging()
    dev = st.device
    sizes = tuple(int(torch.Size(s).numel()) for s in shapes)
    if packed:   # element layout with even offsets; its bytes: every slot exactly ceil(n/2), back to back
        lay = st.layout(sizes, align=2)
        b_lay = st.layout(tuple((n + 1) // 2 for n in sizes), align=1)
    else:
        lay = b_lay = st.layout(sizes, align=1)
    rows = _stage_rows(clients, b_lay, st, "mq")
    s_dev = torch.tensor(scales, dtype=torch.float32).to(dev, non_blocking=True)
    out_dev = ops.dequantize_mean_batched(rows if packed else rows.view(torch.int8), s_dev, lay,
                                          out=st.buf("m_out", lay.total, torch.float32), packed=packed)
    on_cpu = [not any(c[j].is_cuda for c in clients) for j in range(len(sizes))]
    return _hand_out(out_dev, lay, [torch.Size(s) for s in shapes], on_cpu, st, "m_out")


@_serialized
def _decode_mean_host(st: _DeviceStaging, like: List[torch.Tensor], numel: torch.Tensor, ptrs: List[np.ndarray],
                      scales: torch.Tensor) -> List[torch.Tensor]:
    """_decode_mean for K CPU qint8 payload lists already checked (SLQChannel._mean_host_updates): each client's
    bytes gathered straight from the storages into its pinned row (one native gather per client, that row's
    H2D enqueued as soon as it is staged), one decode-mean launch, and the fp32 means handed back as owned CPU
    tensors shaped like `like`, created by one native call per staging range while the D2H runs."""
    dev = st.device
    lay = st.layout(tuple(numel.tolist()), align=1)
    _host_heap(lay)
    k = len(ptrs)
    row = (lay.total + 15) // 16 * 16
    rows = st.buf("mq", k * row, torch.uint8).view(k, row)
    host = st.buf("mq_host", k * row, torch.uint8, pinned=True).view(k, row)
    for r in range(k):
        hostcopy.copy_pieces(*_range_copies(ptrs[r], lay, host[r].data_ptr(), 1, 0, lay.total, to_bucket=True))
        rows[r].copy_(host[r], non_blocking=True)
    s_dev = scales.to(dev, non_blocking=True)
    out_dev = ops.dequantize_mean_batched(rows.view(torch.int8), s_dev, lay,
                                          out=st.buf("m_out", lay.total, torch.float32))
    return _hand_out(out_dev, lay, [None] * len(like), [True] * len(like), st, "m_out", like=like)


def _simple_aggregate(values: List[torch.Tensor]) -> torch.Tensor:
    """One entry of simple_aggregate (Src/ADFL/model.py:221-234), as the reference computes it."""
    with torch.no_grad():
        return torch.sum(torch.stack(values, dim=0), dim=0) / len(values)


def device_mean_order_ok() -> bool:
    """The device mean kernels follow torch's CPU sum(dim=0) order as ATen's AVX2 kernel takes it
    (csrc/torch_sum_order.h). If this process's torch sums in another order (sum_order.self_check fails:
    another torch build or CPU kernel), receive_mean decodes and aggregates every entry on the host the
    reference's way instead, so the device and host halves of one aggregate never disagree; warned once."""
    ok = sum_order.self_check()
    if not ok and not _ORDER_WARNED[0]:
        _ORDER_WARNED[0] = True
        import warnings
        warnings.warn("adfl_amd: this torch's CPU sum order differs from the one the device mean kernels "
                      "restate; receive_mean aggregates on the host (bit-identical, slower)", RuntimeWarning)
    return ok


_ORDER_WARNED = [False]


def _aggregate_entries(names: List[str], parts: List[Parameters]) -> Dict[str, torch.Tensor]:
    """simple_aggregate over the entries `names` of the K dicts `parts` (host tensors: biases, running
    statistics, counters), with the per-entry call's values but not its per-entry dispatch cost (256
    biases: about 3 ms of stack / sum / div). Entries of one dtype are concatenated into K rows and summed
    together: int64 with K elementwise adds (integer sums are exact in any order), fp32 in torch's own CPU
    summation order (adfl_amd.sum_order: each entry's columns in the order its own
    torch.sum(torch.stack(...), 0) takes, bit for bit; checked against torch once per process,
    sum_order.self_check). Then one division and a split into owned tensors. One-element fp32 entries at
    K >= 8 (torch's inner-sum kernel) and everything else go through simple_aggregate per entry."""
    k = len(parts)
    res: Dict[str, torch.Tensor] = {}
    f32_ok = sum_order.self_check()
    lists = [[p[n] for n in names] for p in parts]
    if names and all(isinstance(v, torch.Tensor) for row in lists for v in row):
        # the classification, the K rows and the owned results in native calls (adfl_torchhost)
        th = _torchhost.get()
        uni, code, numel = (a.numpy() for a in th.entry_meta_k(lists))
        f32 = uni & (code == 0) & f32_ok & (numel > 0) & ~((numel == 1) & (k >= 8))
        with torch.no_grad():
            for sel, is_f32 in ((f32, True), (uni & (code == 1), False)):
                idx = np.nonzero(sel)[0]
                if idx.size < 2:
                    continue
                rows = th.concat_rows(lists, torch.from_numpy(idx))
                if is_f32:
                    acc = sum_order.sum_rows(rows, numel[idx].tolist())
                else:   # int64: K elementwise adds from zero (exact in any order)
                    acc = torch.zeros_like(rows[0])
                    for r in rows.unbind(0):
                        acc = acc + r
                agg = acc / k
                for i, t in zip(idx.tolist(), th.split_owned(agg, [lists[0][i] for i in idx.tolist()])):
                    res[names[i]] = t
        for n in names:
            if n not in res:
                res[n] = _simple_aggregate([p[n] for p in parts])
        return res
    groups: Dict[torch.dtype, List[str]] = {}
    for n in names:
        vals = [p[n] for p in parts]
        t0 = vals[0]
        if not all(isinstance(v, torch.Tensor) and not v.is_cuda and v.is_contiguous() and v.dtype == t0.dtype
                   and v.shape == t0.shape for v in vals):
            continue
        if t0.dtype == torch.int64 or (t0.dtype == torch.float32 and f32_ok and t0.numel() > 0
                                       and not (t0.numel() == 1 and k >= 8)):
            groups.setdefault(t0.dtype, []).append(n)
    with torch.no_grad():
        for dt, ns in groups.items():
            if len(ns) < 2:
                continue
            sizes = [parts[0][n].numel() for n in ns]
            if dt == torch.int64:
                rows = [torch.cat([p[n].reshape(-1) for n in ns]) for p in parts]
                acc = torch.zeros_like(rows[0])
                for r in rows:
                    acc = acc + r
            else:
                stacked = torch.stack([torch.cat([p[n].reshape(-1) for n in ns]) for p in parts])
                acc = sum_order.sum_rows(stacked, sizes)
            agg = acc / k
            for n, piece in zip(ns, torch.split(agg, sizes)):
                shape = parts[0][n].shape
                res[n] = (piece if piece.shape == shape else piece.view(shape)).clone()
    for n in names:
        if n not in res:
            res[n] = _simple_aggregate([p[n] for p in parts])
    return res


@_serialized
def _encode_dict_packed(params: Parameters, names: List[str], bits: int, stats: Optional[list] = None):
    """Packed int4 variant of _encode_dict: {name: (int8 tensor of ceil(n/2) packed bytes, scale)}; with
    `stats`, the bucket's four q-error sums against its packed payload are appended."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    th = _torchhost.get()
    host_ok, numel, hptrs = th.host_bytes(tensors, 4)   # sizes, and contiguous CPU fp32 storages, in one call
    lay = st.layout(tuple(numel.tolist()), align=2)
    x_dev = _stage_in(tensors, lay, st, "x", torch.float32, host_ptrs=hptrs.numpy().view(np.uint64) if host_ok else None)
    p_dev, s_dev = ops.encode_batched_int4(x_dev, lay, bits, packed=st.buf("p", lay.total // 2, torch.uint8),
                                           scales=st.buf("scales", lay.ntensors, torch.float32),
                                           partials=st.buf("partials", lay.nchunks, torch.int32))
    if stats is not None:
        stats.append(_qerror_sums(x_dev, ops.decode_batched_int4(p_dev, s_dev, lay,
                                                                 out=st.buf("qe_d", lay.total, torch.float32)), lay))
    scales_host = st.buf("scales_host", lay.ntensors, torch.float32, pinned=True)
    scales_host.copy_(s_dev, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    scales = scales_host.tolist()
    # packed-byte layout: with align=2 tensor k's ceil(n/2) bytes sit at offsets[k] / 2
    p_lay = st.layout(tuple(int(n) // 2 for n in lay.padded.tolist()), align=1)
    if host_ok:   # the owned int8 payloads created by one native call per staging range while the D2H runs
        p_numel = (numel + 1) // 2
        parts = _PendingD2H(p_dev.view(torch.int8), p_lay, st, "p").finish_building(
            None, len(tensors), make_batch=lambda a, b: th.empty_1d(p_numel[a:b], 1))
        return {name: (pt, sc) for name, pt, sc in zip(names, parts, scales)}
    on_cpu = [not t.is_cuda for t in tensors]
    shapes = [torch.Size([(int(t.numel()) + 1) // 2]) for t in tensors]
    # int8, as compression.py:pack_4bit returns; each tensor owns its bytes (the staging is reused)
    parts = _hand_out(p_dev.view(torch.int8), p_lay, shapes, on_cpu, st, "p")
    return {name: (pt, sc) for name, pt, sc in zip(names, parts, scales)}


@_serialized
def _decode_dict_packed(items: List[Tuple[str, torch.Tensor, torch.Size, float]]) -> Dict[str, torch.Tensor]:
    """Decode packed int4 payloads (name, packed int8 [ceil(n/2)], original shape, scale)."""
    st = _staging()
    dev = st.device
    sizes = tuple(int(torch.Size(shape).numel()) for _, _, shape, _ in items)
    lay = st.layout(sizes, align=2)
    for (name, p, _, _), n in zip(items, sizes):
        if p.numel() != (n + 1) // 2:
            raise ValueError(f"PackedSLQChannel: '{name}' holds {p.numel()} packed bytes, expected {(n + 1) // 2}")
    # with align=2 every tensor's slot is exactly ceil(n/2) packed bytes: the gather is one concatenation
    p_lay = st.layout(tuple((n + 1) // 2 for n in sizes), align=1)
    p_dev = _stage_in([p.view(torch.uint8) for _, p, _, _ in items], p_lay, st, "dp", torch.uint8)
    s_dev = torch.tensor([s for _, _, _, s in items], dtype=torch.float32).to(dev, non_blocking=True)
    on_cpu = [not p.is_cuda for _, p, _, _ in items]
    out_dev = ops.decode_batched_int4(p_dev, s_dev, lay, out=st.buf("d_out", lay.total, torch.float32))
    decoded = _hand_out(out_dev, lay, [torch.Size(shape) for _, _, shape, _ in items], on_cpu, st, "d_out")
    return {name: t for (name, _, _, _), t in zip(items, decoded)}


class SLQChannel(Channel):
    """Bi-directional symmetric linear quantization (quant.py:15-112) on the MI355X HIP codec."""

    def __init__(self, bits: int) -> None:
        self.bits = bits

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
        """self.bits for weights, 32 bits for biases, 32 bits per scale (quant.py:47-58)."""
        p_info = get_parameter_info(params)
        num_bytes = p_info.num_non_bias_w * self.bits / 8
        num_bytes += p_info.num_bias_w * 4
        num_bytes += p_info.num_non_bias_t * 4
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
        datas = [p.data for p in c_params.params.values()]
        th = _torchhost.get()
        kinds = th.payload_kinds(datas).numpy()   # _dequantize_tensor's cases for every entry in one call
        qi = np.nonzero(kinds == 1)[0].tolist()
        vals: List[Optional[torch.Tensor]] = [None] * len(names)
        rest_done = []

        def rest():   # every entry but the decoded ones; the host decode runs it while its copies land
            if rest_done:
                return
            rest_done.append(True)
            pi = np.nonzero(kinds == 0)[0].tolist()
            for i, t in zip(pi, th.variable_data([datas[i] for i in pi])):
                vals[i] = t  # passthrough: q_param.data.data (quant.py:111-112)
            for i in np.nonzero(kinds == 2)[0].tolist():
                vals[i] = datas[i].data.dequantize()  # non-quantized ndim > 1 payload: what quant.py:110 does

        decoded = _decode_dict([(names[i], datas[i]) for i in qi], idle=rest) if qi else {}
        for i in qi:
            vals[i] = decoded[names[i]]
        rest()
        return dict(zip(names, vals)), time.perf_counter() - s_time

    def receive_add_(self, c_params: CompressedParameters, targets: List[Parameters]) -> float:
        """``on_client_receive(c_params)`` followed by ``add_parameters_inpace(t, decoded, 1, 1, False)`` for
        every ``t`` in ``targets`` — the client pool's ``add_to_model`` / ``add_to_model_all``
        (Src/ADFL/Client/pool.py:62-75) and QAFeL's hidden-state update (Src/ADFL/Server/qafel.py:176-179),
        bit-identical to them. Returns the seconds spent.

        Quantized tensors whose targets all live on the GPU are decoded once and accumulated into every
        model by one launch (ops.dequantize_add_batched: the payload is read once, each model read and
        written once, no decoded tensor is materialised). Everything else takes the reference's route:
        decode, then ``mul_(1).add_(decoded, alpha=1)``."""
        assert isinstance(c_params, QuantParameters)
        for t in targets:
            assert set(t.keys()) == set(c_params.params.keys())  # add_parameters_inpace, model.py:340
        s_time = time.perf_counter()
        fused = [n for n, p in c_params.params.items()
                 if p.data.ndim > 1 and p.data.is_quantized and p.data.numel() > 0
                 and all(t[n].is_cuda and t[n].dtype == torch.float32 and t[n].is_contiguous()
                         and t[n].data_ptr() % 16 == 0 for t in targets)]
        if fused:
            _decode_add(c_params, fused, targets)
        rest = QuantParameters({n: p for n, p in c_params.params.items() if n not in fused}, 0)
        if rest.params:
            decoded, _ = self.on_client_receive(rest)
            with torch.no_grad():
                for t in targets:
                    for n, d in decoded.items():
                        t[n].mul_(1).add_(d.to(t[n].device), alpha=1)
        return time.perf_counter() - s_time

    def receive_mean(self, all_c_params: List[CompressedParameters]) -> Tuple[Parameters, float]:
        """``simple_aggregate([self.on_server_receive(c)[0] for c in all_c_params])`` — a synchronous
        server decoding K client updates and averaging them (Src/ADFL/Strategy/simple.py:83-89 over
        Src/ADFL/model.py:221-234; the peer mean of Examples/ray_ad.py:188). Returns (aggregate, seconds).

        Tensors quantized in every update are decoded and averaged on the device in one launch: the K
        payloads are read once and no decoded copy is materialised (ops.dequantize_mean_batched). Their
        mean is summed in torch's CPU order for ``torch.sum(torch.stack(...), dim=0)`` (csrc/torch_sum_order.h:
        per tensor, a 16-row cascade over the SEQ columns, four interleaved partials over each tensor's last
        n % 32 elements), then / K correctly rounded: bit-identical to simple_aggregate on CPU tensors (as
        the reference runs it, model.py:195-197) for every K (tests/golden/aggregate.npz: the reference
        executed at K = 1 .. 64). Everything else (biases, running statistics, non-quantized payloads) is
        decoded and aggregated as the reference does, on the host, in the same order."""
        if not all_c_params:
            raise AssertionError("receive_mean: no updates")   # simple_aggregate asserts len > 0
        for c in all_c_params:
            assert isinstance(c, QuantParameters)
        s_time = time.perf_counter()
        names = list(all_c_params[0].params.keys())
        order_ok = device_mean_order_ok()
        out: Parameters = {}
        fast = self._mean_host_updates(all_c_params, names) if order_ok else None
        plain = None
        if fast is not None:   # every update a CPU dict of the same entries: classified in native calls
            fused, decoded, plain = fast
            out.update(zip(fused, decoded))
        else:
            fused = [n for n in names if all(n in c.params and self._fusable(c.params[n]) for c in all_c_params)
                     and len({tuple(c.params[n].shape) for c in all_c_params}) == 1] if order_ok else []
            if fused:
                decoded = self._mean_payloads(all_c_params, fused)
                out.update(zip(fused, decoded))
        rest = [n for n in names if n not in out]
        if rest:
            # passthrough entries decode to their own payload tensor (quant.py:111-112): used as they are
            # (the values _receive hands back, without its per-entry work); the rest through _receive
            if plain is None:
                plain = [n for n in rest if all(self._passthrough(c.params[n]) for c in all_c_params)]
            other = [n for n in rest if n not in set(plain)]
            parts = []
            for c in all_c_params:
                part = {n: c.params[n].data for n in plain}
                if other:
                    part.update(self._receive(QuantParameters({n: c.params[n] for n in other}, 0))[0])
                parts.append(part)
            out.update(_aggregate_entries(rest, parts))
        return {n: out[n] for n in names}, time.perf_counter() - s_time

    @staticmethod
    def _mean_host_updates(all_c_params: List[QuantParameters], names: List[str]):
        """receive_mean's common case in a few native calls: K updates of one model whose entries come in the
        same order, every ndim > 1 payload a non-empty per-tensor qint8 CPU tensor with zero point 0 of the same
        shape in every update. Returns (fused names, their means) — the means from one decode-mean launch
        over rows staged straight from the payloads' storages, the outputs created by one native call per
        staging range — or None when the updates are anything else (receive_mean then classifies entry by
        entry)."""
        if any(list(c.params.keys()) != names for c in all_c_params):
            return None
        th = _torchhost.get()
        datas = [[p.data for p in c.params.values()] for c in all_c_params]
        kinds = np.stack([th.payload_kinds(d).numpy() for d in datas])
        if (kinds == 2).any() or (kinds != kinds[0]).any():
            return None
        idx = np.nonzero(kinds[0] == 1)[0].tolist()
        plain = [names[i] for i in np.nonzero(kinds[0] == 0)[0].tolist()]   # ndim <= 1 in every update
        if not idx:
            return [], [], plain
        qs = [[d[i] for i in idx] for d in datas]
        metas = [th.qint8_meta(q) for q in qs]   # (ok, all contiguous CPU, numel, fp32 scales, data pointers)
        numel = metas[0][2]
        if not all(m[0] and m[1] and torch.equal(m[2], numel) for m in metas) or int(numel.min()) == 0:
            return None
        if not th.shapes_equal(qs):
            return None
        fused = [names[i] for i in idx]
        st = _staging()
        return fused, _decode_mean_host(st, qs[0], numel, [m[4].numpy().view(np.uint64) for m in metas],
                                        torch.stack([m[3] for m in metas])), plain

    @staticmethod
    def _passthrough(p: QuantParameter) -> bool:
        """_receive hands this entry back as its own payload tensor (quant.py:111-112)."""
        return isinstance(p.data, torch.Tensor) and p.data.ndim <= 1

    @staticmethod
    def _fusable(p: QuantParameter) -> bool:
        d = p.data
        return (d.dtype == torch.qint8 and d.ndim > 1 and d.numel() > 0
                and d.qscheme() == torch.per_tensor_affine and d.q_zero_point() == 0)

    def _mean_payloads(self, all_c_params: List[QuantParameters], names: List[str]) -> List[torch.Tensor]:
        qs = [[c.params[n].data for n in names] for c in all_c_params]
        # q_scale() is a double; fbgemm's dequantize uses it as fp32 (quant.py:110)
        return _decode_mean(qs, [[q.q_scale() for q in c] for c in qs], [q.shape for q in qs[0]], packed=False)

    def send_with_q_error(self, params: Parameters) -> Tuple[CompressedParameters, float, float, float]:
        """`on_client_send` fused with the worker's quantization-error metrics.

        Returns (c_params, c_time, q_error_mse, q_error_cos): the values
        Src/ADFL/Client/worker.py:176,186-189 gets from on_client_send, an extra on_server_receive and
        parameter_relative_mse / parameter_cosine_similarity(exclude_bias=True)
        (Src/ADFL/model.py:256-323), bit for bit: the decode stays on the device (no extra transfer) and
        the fp32 sums run in torch's CPU order with this process's torch.get_num_threads() (qerror.py).
        c_time covers the encode only, as on_client_send's does."""
        s_time = time.perf_counter()
        stats: list = []
        q_params = self._quantize_params(params, self.bits, stats)
        c_time = time.perf_counter() - s_time
        if not stats:  # nothing quantized: parameter_relative_mse returns 0.0; cosine of empty vectors raises
            raise RuntimeError("send_with_q_error: no ndim > 1 tensors to measure (torch.cat of an empty list)")
        e, s, c = stats[0]
        count = sum(int(p.numel()) for p in params.values() if p.ndim > 1)
        rel_mse, cos = qerror.metrics(e, s, c, count)
        return q_params, c_time, rel_mse, cos

    def _quantize_params(self, params: Parameters, bits: int, stats: Optional[list] = None) -> QuantParameters:
        """Biases and running metrics (ndim <= 1) are not quantized (quant.py:74-94)."""
        items = list(params.items())
        # every entry's ndim / numel / dtype / placement in one native call (adfl_torchhost.tensor_meta)
        ndim, numel, f32, host = (a.numpy() for a in _torchhost.get().tensor_meta([p for _, p in items]))
        qi = np.nonzero(ndim > 1)[0]
        names = [items[i][0] for i in qi.tolist()]
        bad = qi[(numel[qi] == 0) | ~f32[qi]]
        if bad.size:
            ops.require_quantizable(items[int(bad[0])][1])   # raises the reference's error for that tensor
        sizes = numel[qi].tolist()
        meta = (tuple(sizes), bool(host[qi].all()))
        signs = torch.zeros(1, dtype=torch.uint8)  # the unused field (quant.py:91), one object per call
        qp = QuantParameter
        made: Dict[str, QuantParameter] = {}
        size = [0]
        # positional: QuantParameter(data, bits, scale, signs, shape, dtype, q_dtype) (model.py:21-31)

        f32t, qint8 = torch.float32, torch.qint8

        def emit(k, q, scale):   # a quantized entry, built as soon as its output exists
            n = names[k]
            if n not in made:
                size[0] += sizes[k]           # a qint8 payload: one byte per element
            made[n] = qp(q, bits, scale, signs, q.shape, f32t, qint8)
        rest = iter([items[i] for i in np.nonzero(ndim <= 1)[0].tolist()])

        def idle(batch=32):      # passthrough entries (quant.py:80-81), a batch per copy range
            for _ in range(batch):
                e = next(rest, None)
                if e is None:
                    return False
                t = e[1]
                made[e[0]] = qp(t, bits, 1, signs, t.shape, t.dtype, t.dtype)
                size[0] += t.nbytes
            return True
        encoded = _encode_dict(params, names, bits, stats, emit=emit, idle=idle, meta=meta) if names else {}
        for k, n in enumerate(names):
            if n not in made:    # device dicts and the other staging paths: built here
                emit(k, *encoded[n])
        while idle():
            pass
        return QuantParameters({name: made[name] for name in params}, size[0])


class USLQChannel(SLQChannel):
    """Uni-directional SLQ (quant.py:115-137): only client -> server is quantized."""

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return IdentityChannel(no_compute_time=True).on_server_send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return IdentityChannel(no_compute_time=True).on_client_receive(c_params)

    def to_json(self) -> Dict:
        return {"name": self.__class__.__name__, "bits": self.bits}


class PackedSLQChannel(SLQChannel):
    """SLQ with the 4-bit payload actually packed two values per byte — the end-to-end int4 path the
    reference meant to provide but cannot run (Src/ADFL/compression.py:91-94 passes a qint8 tensor to
    pack_4bit and raises; its dequantize_tensor never unpacks, :71-74).

    Encode = SLQ quantize (bit-exact with SLQChannel(bits)) + pack_4bit's nibble layout
    (compression.py:35-48); decode = unpack_4bit (:51-66) + dequantize. Payload entries:
    QuantParameter(data = int8 tensor of ceil(n/2) packed bytes, bits, scale, shape = original shape,
    dtype = float32, q_dtype = int8) — what compression.quantize_params builds for bits == 4 (:86-110).
    bits must be <= 4 (larger codes do not fit a nibble). Values 127 from an all-zero / NaN tensor alias
    exactly as pack_4bit makes them alias (nibbles 7, -1); they dequantize to +-0.0 / NaN."""

    def __init__(self, bits: int) -> None:
        if not 1 <= bits <= 4:
            raise ValueError(f"PackedSLQChannel: bits must be in [1, 4], got {bits}")
        super().__init__(bits)

    @staticmethod
    def _is_packed(p: QuantParameter) -> bool:
        return p.dtype == torch.float32 and p.q_dtype == torch.int8 and len(p.shape) > 1 and p.data.ndim == 1

    def _receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        assert isinstance(c_params, QuantParameters)
        s_time = time.perf_counter()
        packed = [(name, p.data, p.shape, p.scale) for name, p in c_params.params.items() if self._is_packed(p)]
        decoded = _decode_dict_packed(packed) if packed else {}
        params = {name: decoded[name] if name in decoded else p.data.data for name, p in c_params.params.items()}
        return params, time.perf_counter() - s_time

    def _fusable(self, p: QuantParameter) -> bool:
        return self._is_packed(p) and p.data.numel() == (torch.Size(p.shape).numel() + 1) // 2

    def _passthrough(self, p: QuantParameter) -> bool:
        return isinstance(p.data, torch.Tensor) and p.data.ndim <= 1 and not self._is_packed(p)

    @staticmethod
    def _mean_host_updates(all_c_params: List[QuantParameters], names: List[str]):
        """Packed payloads are 1-D byte buffers whose shape lives in the payload object: the native
        classification of SLQChannel's qint8 updates does not apply (receive_mean classifies entry by entry)."""
        return None

    def _mean_payloads(self, all_c_params: List[QuantParameters], names: List[str]) -> List[torch.Tensor]:
        return _decode_mean([[c.params[n].data for n in names] for c in all_c_params],
                            [[c.params[n].scale for n in names] for c in all_c_params],
                            [torch.Size(all_c_params[0].params[n].shape) for n in names], packed=True)

    def _quantize_params(self, params: Parameters, bits: int, stats: Optional[list] = None) -> QuantParameters:
        items = list(params.items())
        # every entry's ndim / numel / dtype in one native call (adfl_torchhost.tensor_meta)
        ndim, numel, f32, _ = (a.numpy() for a in _torchhost.get().tensor_meta([p for _, p in items]))
        qi = np.nonzero(ndim > 1)[0]
        names = [items[i][0] for i in qi.tolist()]
        bad = qi[(numel[qi] == 0) | ~f32[qi]]
        if bad.size:
            ops.require_quantizable(items[int(bad[0])][1])   # raises the reference's error for that tensor
        encoded = _encode_dict_packed(params, names, bits, stats) if names else {}
        signs = torch.zeros(1, dtype=torch.uint8)  # the unused field (compression.py:102), one object per call
        qp = QuantParameter
        out: Dict[str, QuantParameter] = {}
        size = 0
        for name, param in items:
            q_param, scale = encoded[name] if name in encoded else (param, 1)
            # positional: QuantParameter(data, bits, scale, signs, shape, dtype, q_dtype) (model.py:21-31)
            out[name] = qp(q_param, bits, scale, signs, param.shape, param.dtype, q_param.dtype)
            size += q_param.nbytes
        return QuantParameters(out, size)


HipSLQChannel = SLQChannel
HipUSLQChannel = USLQChannel

# The stochastic channels live beside the reference's in quant.py's namespace (quant.py:140-570).
from .stoch import (CNATChannel, QSGDChannel, RQSGDChannel, UCNATChannel, UQSGDChannel,  # noqa: E402,F401
                    URQSGDChannel)
