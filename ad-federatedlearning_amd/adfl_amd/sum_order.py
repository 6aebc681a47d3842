"""torch 2.10's CPU summation order for ``torch.sum(torch.stack(rows), dim=0)``, on the host, for many
entries at once.

The mean kernels follow this order on the device (``csrc/torch_sum_order.h`` states it and cites
``aten/src/ATen/native/cpu/SumKernel.cpp``); this module applies the same order with elementwise torch adds
to a [K, total] stack of concatenated host entries, so that ``receive_mean`` can aggregate every passthrough
entry (biases, running statistics — ``simple_aggregate``, ``Src/ADFL/model.py:221-234``) of a state dict in
a few vector operations instead of a stack / sum / div per entry, with each entry's result bit-identical to
its own ``torch.sum(torch.stack(...), dim=0)``:

* SEQ columns (entry index j < seq_end(n)): rows added in order from +0 into level 0; every 16th row level 0
  is added into level 1 (every 256th level 1 into 2, every 4096th 2 into 3); then ((l0 + l1) + l2) + l3;
* ILP4 columns (an entry's last n % 32 elements; n % 4 for n < 8): partial p sums rows 4g + p with the same
  cascade over g, leftover rows go into partial 0, then ((p0 + p1) + p2) + p3;
* one-element entries with K >= 8 (vectorized_inner_sum) are left to torch per entry (rare).

``self_check()`` compares this against torch itself once per process (a handful of sizes at K = 1 .. 20
and 64); ``_aggregate_entries`` aggregates per entry through torch when it fails, so the host values stay
the reference's even on a torch build whose order differs."""

from typing import List, Optional

import numpy as np
import torch

_CHECKED: Optional[bool] = None


def seq_end(n: int) -> int:
    if n == 1:
        return 0
    return n & ~31 if n >= 8 else n & ~3


def _cascade(rows: List[torch.Tensor]) -> torch.Tensor:
    """multi_row_sum over the rows (each a 1-D tensor of the same length), elementwise."""
    z = torch.zeros_like(rows[0])
    a0 = z
    a1 = a2 = a3 = None
    for i, r in enumerate(rows, 1):
        a0 = a0 + r
        if i % 16 == 0:
            a1 = a0 if a1 is None else a1 + a0   # first fold: +0 + a0 == a0 (a0 is never -0)
            a0 = z
            if i % 256 == 0:
                a2 = a1 if a2 is None else a2 + a1
                a1 = None
                if i % 4096 == 0:
                    a3 = a2 if a3 is None else a3 + a2
                    a2 = None
    for lv in (a1, a2, a3):
        if lv is not None:
            a0 = a0 + lv
    return a0


def _ilp4(rows: List[torch.Tensor]) -> torch.Tensor:
    g = len(rows) // 4
    if g:
        p = [_cascade(rows[q:4 * g:4]) for q in range(4)]
    else:
        p = [torch.zeros_like(rows[0]) for _ in range(4)]
    p0 = p[0]
    for r in rows[4 * g:]:
        p0 = p0 + r
    return ((p0 + p[1]) + p[2]) + p[3]


def sum_rows(stacked: torch.Tensor, sizes: List[int]) -> torch.Tensor:
    """torch.sum(torch.stack(...), dim=0) of every entry: `stacked` is [K, total] (row k = client k's
    entries concatenated, entry e of `sizes[e]` elements); returns [total]. One-element entries need K < 8
    (torch's inner-sum kernel handles them otherwise; the caller routes those per entry)."""
    rows = list(stacked.unbind(0))
    seq = _cascade(rows)
    n = np.asarray(sizes, dtype=np.int64)
    e = np.where(n == 1, 0, np.where(n >= 8, n & ~31, n & ~3))   # seq_end of every entry
    off = np.concatenate([[0], np.cumsum(n)[:-1]])
    tail = e < n
    if not tail.any():
        return seq
    edge = np.zeros(int(n.sum()) + 1, dtype=np.int64)   # +1 where an entry's tail starts, -1 where it ends
    np.add.at(edge, (off + e)[tail], 1)
    np.add.at(edge, (off + n)[tail], -1)
    idx = torch.from_numpy(np.nonzero(np.cumsum(edge[:-1]) > 0)[0])
    tail = _ilp4([r.index_select(0, idx) for r in rows])
    seq[idx] = tail
    return seq


def self_check() -> bool:
    """One-time comparison of sum_rows with torch's own per-entry sums (sizes covering every branch)."""
    global _CHECKED
    if _CHECKED is None:
        g = torch.Generator().manual_seed(1234)
        sizes = [1, 2, 3, 6, 7, 9, 33, 64, 70, 100]
        ok = True
        for k in (1, 4, 5, 7, 16, 17, 20, 64):
            ents = [torch.randn(k, n, generator=g) * torch.exp(torch.randn(k, n, generator=g) * 4) for n in sizes]
            use = [i for i, n in enumerate(sizes) if not (n == 1 and k >= 8)]
            got = sum_rows(torch.cat([ents[i] for i in use], dim=1), [sizes[i] for i in use])
            want = torch.cat([torch.sum(torch.stack(list(ents[i].unbind(0))), dim=0) for i in use])
            if not torch.equal(got.view(torch.int32), want.view(torch.int32)):
                ok = False
                break
        _CHECKED = ok
    return _CHECKED
