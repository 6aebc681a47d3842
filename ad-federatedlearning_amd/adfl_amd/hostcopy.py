"""Parallel host staging copies over the native pool (include/adfl_host.h, csrc/host_copy.cpp).

gather(): pieces of a CPU state dict -> one (pinned) host bucket; scatter(): a host bucket -> per-tensor
storages. ctypes releases the GIL for the call, so the copy runs on the pool's threads plus the caller's.
"""

import ctypes
import os
from typing import Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check

_host = None


def _host_lib():
    """The library exporting adfl_host_copy: libadfl_slq.so, or — for CPU sanitizer runs only
    (tools/sanitize/run.sh) — a separately built host-copy object named by ADFL_HOST_LIB."""
    global _host
    if _host is None:
        path = os.environ.get("ADFL_HOST_LIB")
        if path:
            lib = ctypes.CDLL(path)
            for name in ("adfl_host_copy", "adfl_host_copy_ex", "adfl_host_threads", "adfl_host_copy_submit",
                         "adfl_host_copy_wait", "adfl_host_copy_done", "adfl_host_copy_submit_absmax",
                         "adfl_host_bind"):
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = _lib.SIGNATURES[name]
            _host = lib
        else:
            _host = _lib.load()
    return _host


STREAM = 1  # ADFL_HOST_COPY_STREAM


def copy_pieces(dst_ptrs: Sequence[int], src_ptrs: Sequence[int], nbytes: Sequence[int], threads: int = 0,
                stream: bool = False) -> None:
    """stream=True: streaming (non-temporal) stores for large pieces — for fresh destinations nothing reads
    soon (the scatter into per-tensor outputs); the gather into a pinned bucket keeps plain memcpy."""
    d = np.asarray(dst_ptrs, dtype=np.uint64)
    s = np.asarray(src_ptrs, dtype=np.uint64)
    b = np.asarray(nbytes, dtype=np.int64)
    if not (len(d) == len(s) == len(b)):
        raise ValueError("copy_pieces: pointer and size lists differ in length")
    check(_host_lib().adfl_host_copy_ex(d.ctypes.data, s.ctypes.data, b.ctypes.data, len(b), threads,
                                        STREAM if stream else 0))


class Pending:
    """An asynchronous copy job (adfl_host_copy_submit): the pool's workers run it — after `event` has
    completed, when one is given — while the caller's thread goes on; wait() blocks (GIL released) until every
    byte is copied. The arrays and tensors named by the job are kept alive here until then."""

    __slots__ = ("ticket", "_keep")

    def __init__(self, ticket: int, keep):
        self.ticket = ticket
        self._keep = keep

    def wait(self) -> None:
        if self.ticket:
            t, self.ticket = self.ticket, 0
            try:
                check(_host_lib().adfl_host_copy_wait(t))
            finally:
                self._keep = None   # only now: the workers may still read the buffers / wait on the event

    def done(self) -> bool:
        """True once every byte is copied (wait() then returns at once); never blocks."""
        if not self.ticket:
            return True
        r = _host_lib().adfl_host_copy_done(self.ticket)
        if r < 0:
            check(int(r))
        return r == 1

    def __del__(self):   # a job is always waited for: its buffers must outlive the copy
        try:
            self.wait()
        except Exception:  # noqa: BLE001
            pass


_event_wait = None


def _event_wait_fn() -> int:
    """Address of adfl_event_synchronize (the HIP library's own export) for the pool's wait callback."""
    global _event_wait
    if _event_wait is None:
        _event_wait = ctypes.cast(_lib.load().adfl_event_synchronize, ctypes.c_void_p).value
    return _event_wait


def submit_pieces(dst_ptrs: Sequence[int], src_ptrs: Sequence[int], nbytes: Sequence[int], *, stream: bool = False,
                  event: "torch.cuda.Event | int | None" = None, keep=None, threads: int = 0,
                  absmax_ptrs: "np.ndarray | None" = None) -> Pending:
    """copy_pieces on the pool's workers, asynchronously; with `event` (a recorded torch.cuda.Event, or the
    hipEvent_t handle of one the staging owns, adfl_stage_events_create) every part first waits for it
    (hipEventSynchronize), so the copy starts the moment the D2H that fills its source lands. `keep`: objects the copy reads or writes, held until wait(). `absmax_ptrs` (uint64 per
    piece, 0 = none): fp32 pieces whose max |bits| is max'ed into the uint32 at that address
    (adfl_host_copy_submit_absmax)."""
    d = np.ascontiguousarray(dst_ptrs, dtype=np.uint64)
    s = np.ascontiguousarray(src_ptrs, dtype=np.uint64)
    b = np.ascontiguousarray(nbytes, dtype=np.int64)
    if not (len(d) == len(s) == len(b)):
        raise ValueError("submit_pieces: pointer and size lists differ in length")
    fn, arg = (None, None) if event is None else (_event_wait_fn(), event if isinstance(event, int) else event.cuda_event)
    if absmax_ptrs is not None:
        a = np.ascontiguousarray(absmax_ptrs, dtype=np.uint64)
        if len(a) != len(b):
            raise ValueError("submit_pieces: one absmax slot per piece")
        t = _host_lib().adfl_host_copy_submit_absmax(d.ctypes.data, s.ctypes.data, b.ctypes.data, len(b), threads,
                                                     STREAM if stream else 0, fn, arg, a.ctypes.data)
        if t <= 0:
            check(int(t))
        return Pending(int(t), (keep, event, a))
    t = _host_lib().adfl_host_copy_submit(d.ctypes.data, s.ctypes.data, b.ctypes.data, len(b), threads,
                                          STREAM if stream else 0, fn, arg)
    if t <= 0:
        check(int(t))
    return Pending(int(t), (keep, event))


def gather(srcs: Sequence[torch.Tensor], dst: torch.Tensor, offsets: Sequence[int]) -> None:
    """dst.view(-1)[offsets[k] : offsets[k] + srcs[k].numel()] = srcs[k] for contiguous CPU tensors of
    dst's element size (byte copies; dtypes of equal size are reinterpreted)."""
    es = dst.element_size()
    base = dst.data_ptr()
    for t in srcs:
        if t.is_cuda or not t.is_contiguous() or t.element_size() != es:
            raise ValueError("hostcopy.gather: sources must be contiguous CPU tensors of the bucket's element size")
    copy_pieces([base + int(o) * es for o in offsets], [t.data_ptr() for t in srcs], [t.numel() * es for t in srcs])


def scatter(src: torch.Tensor, dsts: Sequence[torch.Tensor], offsets: Sequence[int]) -> None:
    """dsts[k] = src.view(-1)[offsets[k] : offsets[k] + dsts[k].numel()] (byte copies)."""
    es = src.element_size()
    base = src.data_ptr()
    for t in dsts:
        if t.is_cuda or not t.is_contiguous() or t.element_size() != es:
            raise ValueError("hostcopy.scatter: destinations must be contiguous CPU tensors of the bucket's element size")
    copy_pieces([t.data_ptr() for t in dsts], [base + int(o) * es for o in offsets], [t.numel() * es for t in dsts],
                stream=True)


_HUGE = 2 << 20        # x86-64 transparent huge page
_MADV_HUGEPAGE = 14
_libc = None


def advise_huge(tensors: Sequence[torch.Tensor], min_bytes: int = 4 << 20) -> None:
    """madvise(MADV_HUGEPAGE) over the 2 MiB-aligned interior of every fresh CPU tensor of at least
    `min_bytes`, before anything touches it. Large outputs are fresh anonymous mmaps (glibc) whose first
    touch faults in every 4 KiB page; with the advice (THP mode "madvise", the common default) the scatter
    faults 2 MiB pages instead: a first copy into a fresh 1 GiB tensor measured 143 -> 60 ms on 8 threads
    (tools/channel_breakdown.py). Advice only: a kernel without THP ignores it, and the bytes are the same."""
    global _libc
    if _libc is None:
        try:
            _libc = ctypes.CDLL("libc.so.6", use_errno=True)
            _libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            _libc.madvise.restype = ctypes.c_int
        except OSError:
            _libc = False
    if not _libc:
        return
    for t in tensors:
        nb = t.numel() * t.element_size()
        if t.is_cuda or nb < min_bytes:
            continue
        p = t.data_ptr()
        a = (p + _HUGE - 1) // _HUGE * _HUGE
        e = (p + nb) // _HUGE * _HUGE
        if e > a:
            _libc.madvise(a, e - a, _MADV_HUGEPAGE)  # failure is harmless: the advice is simply not taken


_M_TRIM_THRESHOLD, _M_MMAP_THRESHOLD = -1, -3   # glibc mallopt parameters (malloc.h)
_GLIBC_MMAP_MIN = 128 << 10    # glibc's default mmap threshold
_MMAP_CAP = 32 << 20
_TRIM_CAP = 1 << 30
_heap = {"enabled": None, "mmap": 0, "trim": 0}
_libc_mallopt = None


def _mallopt(param: int, value: int) -> bool:
    global _libc_mallopt
    if _libc_mallopt is None:
        try:
            libc = ctypes.CDLL("libc.so.6")
            libc.mallopt.argtypes = [ctypes.c_int, ctypes.c_int]
            libc.mallopt.restype = ctypes.c_int
            _libc_mallopt = libc.mallopt
        except (OSError, AttributeError):
            _libc_mallopt = False
    return bool(_libc_mallopt) and bool(_libc_mallopt(param, value))


def keep_host_heap(working_set: int = 0, largest: int = 0) -> bool:
    """Keep the channel's freed host outputs in the process heap, sized from its working set.

    The channel's per-tensor outputs (ResNet-18's are about 180 KiB each, above glibc's 128 KiB mmap
    threshold) would each be a fresh mmap: first-touch page faults in the scatter, an munmap on free, and
    mmap_lock contention with the copying pool. This sets, PROCESS-WIDE (glibc mallopt; it also turns off
    glibc's dynamic thresholds):
      M_MMAP_THRESHOLD = `largest` (the biggest output, bytes) rounded up to a power of two, between 128 KiB
                         and 32 MiB — so those outputs come from the heap;
      M_TRIM_THRESHOLD = 2 x `working_set` (one call's output bytes), at most 1 GiB — so at most that much
                         freed heap stays resident between rounds.
    Both are only ever raised, as the largest layout seen grows (no setting before the first host-resident
    call). A round's outputs then reuse the previous round's pages. ADFL_KEEP_HOST_HEAP=0 in the environment
    leaves the allocator untouched. Returns whether the settings are in force."""
    if _heap["enabled"] is None:
        _heap["enabled"] = os.environ.get("ADFL_KEEP_HOST_HEAP", "1") != "0"
    if not _heap["enabled"] or working_set <= 0:
        return bool(_heap["mmap"])
    mmap = _GLIBC_MMAP_MIN
    while mmap < min(int(largest), _MMAP_CAP):
        mmap <<= 1
    trim = min(2 * int(working_set), _TRIM_CAP)
    if mmap > _heap["mmap"] and _mallopt(_M_MMAP_THRESHOLD, mmap):
        _heap["mmap"] = mmap
    if trim > _heap["trim"] and _mallopt(_M_TRIM_THRESHOLD, trim):
        _heap["trim"] = trim
    return bool(_heap["mmap"])


def heap_settings() -> dict:
    """The (mmap, trim) thresholds keep_host_heap has set in this process (0: untouched)."""
    return {"mmap": _heap["mmap"], "trim": _heap["trim"]}


def _cpulist(text: str):
    cpus = []
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.extend(range(int(a), int(b or a) + 1))
    return cpus


def device_cpus(device: "torch.device") -> "list[int]":
    """The CPUs of the NUMA node the GPU hangs off (sysfs local_cpulist of its PCI function), within this
    process's affinity mask; [] when unknown."""
    try:
        p = torch.cuda.get_device_properties(device)
        path = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(os.path.join(path, "local_cpulist")) as f:
            cpus = _cpulist(f.read())
    except (OSError, ValueError, AttributeError, RuntimeError):
        return []
    allowed = os.sched_getaffinity(0)
    return [c for c in cpus if c in allowed] if len(cpus) < os.cpu_count() else []


_bound = {}          # device -> the CPUs of its NUMA node (what on_cpus uses for its pinned buffers)
_pool_cpus = None    # what the one process-wide copy pool is pinned to


def bind_to_device(device: "torch.device") -> "list[int]":
    """Pin the copy pool's workers to the GPU's NUMA node (ADFL_HOST_BIND=0: never). The pool is one per
    process: with one device it runs on that device's node; once a process stages for devices on different
    nodes it is re-pinned to the union of their nodes (not to whichever device came last), so no device's
    staging is left on a far node alone. The pinned staging buckets are allocated from a thread on each
    device's own node (on_cpus). Returns the CPUs of this device's node."""
    global _pool_cpus
    key = (device.type, device.index)
    if key not in _bound:
        cpus = device_cpus(device) if os.environ.get("ADFL_HOST_BIND", "1") != "0" else []
        _bound[key] = cpus
        want = sorted(set().union(*[set(c) for c in _bound.values() if c]))
        if want and want != _pool_cpus:
            arr = np.asarray(want, dtype=np.int32)
            if _host_lib().adfl_host_bind(arr.ctypes.data, len(arr)) == 0:
                _pool_cpus = want
    return _bound[key]


def pool_cpus() -> "list[int] | None":
    """The CPUs the copy pool is pinned to (None: not pinned)."""
    return _pool_cpus


class on_cpus:
    """Run a block with this thread's affinity set to `cpus` (restored after): a pinned host buffer allocated
    inside gets its pages on their NUMA node. No-op for an empty list."""

    def __init__(self, cpus):
        self.cpus = cpus
        self.old = None

    def __enter__(self):
        if self.cpus:
            self.old = os.sched_getaffinity(0)
            os.sched_setaffinity(0, self.cpus)
        return self

    def __exit__(self, *exc):
        if self.old is not None:
            os.sched_setaffinity(0, self.old)
        return False


def threads() -> int:
    return int(_host_lib().adfl_host_threads())
