"""The reference's quantization-error metrics, bit for bit, on the device.

Src/ADFL/Client/worker.py:186-189 decodes every update it sends and reports
``parameter_relative_mse(x, d, exclude_bias=True)`` and ``parameter_cosine_similarity(x, d, exclude_bias=True)``
(Src/ADFL/model.py:256-323): per ndim > 1 tensor an fp32 ``torch.sum((x - d) ** 2)`` and
``torch.sum((x - 0) ** 2)`` turned into Python doubles and summed in dict order, and
``F.cosine_similarity`` of the fp32 concatenations. csrc/qerror_ref.hip computes every fp32 sum in torch
2.10's CPU order (include/adfl_qerror.h), the norms come from the reference-order norm
(csrc/torch_norm.hip), and the doubles are formed here exactly as model.py forms them.
"""

import collections
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib, ops, stoch
from ._lib import check

_PLANS: "collections.OrderedDict" = collections.OrderedDict()
_PLAN_CACHE_MAX = 16


def _plan(sizes: Tuple[int, ...], threads: int, dev: torch.device):
    key = (sizes, threads, dev)
    hit = _PLANS.get(key)
    if hit is not None:
        _PLANS.move_to_end(key)
        return hit
    L = _lib.load()
    arr = np.asarray(sizes, dtype=np.int64)
    need = L.adfl_qerror_ref_plan(arr.ctypes.data, len(sizes), threads, None, 0)
    check(int(need) if need < 0 else 0)
    host = np.zeros(int(need) // 8, dtype=np.int64)
    got = L.adfl_qerror_ref_plan(arr.ctypes.data, len(sizes), threads, host.ctypes.data, int(need))
    if got != need:
        check(int(got) if got < 0 else -1)
    scratch = int(L.adfl_qerror_ref_scratch_bytes(host.ctypes.data))
    check(scratch if scratch < 0 else 0)
    hit = (host, torch.from_numpy(host).to(dev), scratch,
           ops.BucketLayout([int(sum(sizes))], align=1))
    _PLANS[key] = hit
    if len(_PLANS) > _PLAN_CACHE_MAX:
        _PLANS.popitem(last=False)
    return hit


def reference_sums(x: torch.Tensor, d: torch.Tensor, sizes: Sequence[int], *, threads: Optional[int] = None):
    """fp32 e[t] = sum((x_t - d_t)^2), s[t] = sum((x_t - 0)^2) per tensor and the cosine's fp32 sum c, for
    tensors of `sizes` back to back at the start of the device fp32 buffers x (an update) and d (its decode).
    threads: the torch.get_num_threads() whose two-pass split is reproduced (default: this process's, what
    the reference's own call uses). Synchronises; returns (e, s, c) as numpy float32 arrays and a float."""
    sizes = tuple(int(n) for n in sizes)
    if not sizes or min(sizes) < 1:
        raise ValueError("adfl_amd.qerror: every tensor needs at least one element")
    total = sum(sizes)
    for t, what in ((x, "x"), (d, "d")):
        if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous() or t.numel() < total:
            raise ValueError(f"adfl_amd.qerror: {what} must be a contiguous fp32 device tensor of >= {total} elements")
    dev = x.device
    threads = torch.get_num_threads() if threads is None else int(threads)
    host, dplan, scratch_bytes, cat = _plan(sizes, threads, dev)
    norms = torch.empty(2, dtype=torch.float32, device=dev)
    stoch.reference_norms(x, cat, out32=norms[0:1], threads=threads)
    stoch.reference_norms(d, cat, out32=norms[1:2], threads=threads)
    scratch = torch.empty(max(scratch_bytes, 256), dtype=torch.uint8, device=dev)
    out = torch.empty(2 * len(sizes) + 1, dtype=torch.float32, device=dev)
    check(_lib.load().adfl_qerror_ref(x.data_ptr(), d.data_ptr(), host.ctypes.data, dplan.data_ptr(), norms.data_ptr(),
                                      scratch.data_ptr(), scratch_bytes, out.data_ptr(), ops._stream(dev)))
    o = out.cpu().numpy()
    n = len(sizes)
    return o[:n].copy(), o[n:2 * n].copy(), float(o[2 * n])


def metrics(e: np.ndarray, s: np.ndarray, c: float, count: int) -> Tuple[float, float]:
    """(parameter_relative_mse, parameter_cosine_similarity) from the fp32 sums, as model.py:256-323 forms
    them: each parameter_mse is sum(float(.item())) in dict order / count; their ratio, 0.0 when the
    denominator is not > 0; the cosine is the fp32 sum itself."""
    num = 0.0
    for v in e.tolist():
        num += v
    den = 0.0
    for v in s.tolist():
        den += v
    num = num / count if count > 0 else 0.0
    den = den / count if count > 0 else 0.0
    return (num / den if den > 0 else 0.0), float(c)
