"""CPU: the native parallel host copy (include/adfl_host.h) — gathers and scatters of ragged piece lists
equal numpy's, from one and from several Python threads at once."""

import threading

import numpy as np
import pytest
import torch

from adfl_amd import _lib, hostcopy


@pytest.mark.parametrize("sizes", [[1], [0, 5, 0], [3, 1 << 20, 7, 65537, (1 << 18) + 3], [64] * 1000,
                                   [12_345_678]])
def test_gather_scatter_roundtrip(sizes):
    rng = np.random.default_rng(len(sizes))
    srcs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)) for n in sizes]
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64) + 3  # unaligned start
    bucket = torch.full((int(sum(sizes)) + 5,), -1.0)
    hostcopy.gather(srcs, bucket, offsets)
    want = np.concatenate([[-1.0] * 3, *[s.numpy() for s in srcs], [-1.0] * 2]).astype(np.float32)
    assert np.array_equal(bucket.numpy(), want)
    outs = [torch.empty(n) for n in sizes]
    hostcopy.scatter(bucket, outs, offsets)
    for a, b in zip(outs, srcs):
        assert torch.equal(a, b)


def test_int8_and_thread_counts():
    src = torch.randint(-128, 127, (3_000_001,), dtype=torch.int8)
    for threads in (1, 2, 7, 0):
        dst = torch.zeros_like(src)
        hostcopy.copy_pieces([dst.data_ptr()], [src.data_ptr()], [src.numel()], threads)
        assert torch.equal(dst, src)
    assert 1 <= hostcopy.threads() <= 16


def test_concurrent_callers():
    """Several Python threads (the GIL is released in the call) share the pool; every copy completes."""
    srcs = [torch.randn(2_000_000 + i) for i in range(8)]
    dsts = [torch.empty_like(s) for s in srcs]
    errs = []

    def work(i):
        try:
            for _ in range(5):
                hostcopy.copy_pieces([dsts[i].data_ptr()], [srcs[i].data_ptr()], [srcs[i].numel() * 4])
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errs
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)


def test_argument_errors():
    lib = _lib.load()
    assert lib.adfl_host_copy(None, None, None, 1, 0) == -1
    assert lib.adfl_host_copy(None, None, None, 0, 0) == 0
    with pytest.raises(ValueError):
        hostcopy.gather([torch.zeros(4, dtype=torch.float64)], torch.zeros(8), [0])
