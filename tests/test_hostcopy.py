"""CPU: the native parallel host copy (include/adfl_host.h) — gathers and scatters of ragged piece lists
equal numpy's, from one and from several Python threads at once."""

import threading
import time

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


@pytest.mark.parametrize("align", [1, 64])
@pytest.mark.parametrize("sizes,piece", [([5, 3_000_000, 17, 65_536, 1], 1 << 20), ([1 << 22], 1 << 20),
                                         ([64] * 500 + [999_999], 1 << 16)])
def test_channel_staging_ranges_cut_through_tensors(sizes, piece, align, monkeypatch):
    """The Channel's host staging (Channel/quant.py _ranges / _range_copies): element ranges that cut through
    tensors gather into the bucket and scatter back exactly, pads untouched, every element once."""
    from adfl_amd import ops
    from adfl_amd.Channel import quant
    monkeypatch.setattr(quant, "_PIECE_BYTES", piece)
    lay = ops.BucketLayout(sizes, align=align)
    rng = np.random.default_rng(7)
    srcs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)) for n in sizes]
    bucket = torch.full((lay.total,), -7.0)
    ranges = quant._ranges(lay, 4)
    assert ranges[0][0] == 0 and ranges[-1][1] == lay.total
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    ptrs = quant._ptrs(srcs)
    for lo, hi in ranges:
        hostcopy.copy_pieces(*quant._range_copies(ptrs, lay, bucket.data_ptr(), 4, lo, hi, to_bucket=True))
    want = np.full(lay.total, -7.0, np.float32)
    for s, o in zip(srcs, lay.offsets):
        want[o:o + s.numel()] = s.numpy()
    assert np.array_equal(bucket.numpy(), want)
    outs = [torch.empty(n) for n in sizes]
    optr = quant._ptrs(outs)
    for lo, hi in reversed(ranges):
        hostcopy.copy_pieces(*quant._range_copies(optr, lay, bucket.data_ptr(), 4, lo, hi, to_bucket=False))
    for a, b in zip(outs, srcs):
        assert torch.equal(a, b)


def test_advise_huge_is_advice_only():
    """hostcopy.advise_huge never changes bytes or raises (small, large, unaligned, device-less tensors)."""
    ts = [torch.arange(10, dtype=torch.float32), torch.zeros(3 << 20), torch.empty(5 << 20, dtype=torch.int8)[1:]]
    hostcopy.advise_huge(ts)
    ts[2].fill_(3)
    assert torch.equal(ts[0], torch.arange(10, dtype=torch.float32)) and int(ts[1].abs().sum()) == 0
    assert int(ts[2].sum()) == 3 * ((5 << 20) - 1)


def test_async_submit_and_wait():
    """hostcopy.submit_pieces (adfl_host_copy_submit): jobs queued behind each other run on the pool's workers
    while the caller goes on; wait() returns when every byte is in place (the channel's pipelined scatter)."""
    rng = np.random.default_rng(5)
    srcs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)) for n in (1, 70_001, 3_000_000, 0, 513)]
    dsts = [torch.full_like(s, -7.0) for s in srcs]
    jobs = [hostcopy.submit_pieces([d.data_ptr()], [s.data_ptr()], [s.numel() * 4], stream=bool(i % 2), keep=(s, d))
            for i, (s, d) in enumerate(zip(srcs, dsts))]
    for j in reversed(jobs):
        j.wait()
        j.wait()   # idempotent
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)
    lib = _lib.load()
    assert lib.adfl_host_copy_wait(0) == -1
    assert lib.adfl_host_copy_done(0) == -1
    with pytest.raises(ValueError):
        hostcopy.submit_pieces([1, 2], [3], [4])


def test_async_done_polls_without_consuming():
    """Pending.done() (adfl_host_copy_done): never blocks, turns True once the copy has finished, and leaves
    the ticket to wait() (the encode enqueues every landed range before building outputs)."""
    s = torch.randn(4_000_000)
    d = torch.zeros_like(s)
    job = hostcopy.submit_pieces([d.data_ptr()], [s.data_ptr()], [s.numel() * 4], keep=(s, d))
    deadline = time.monotonic() + 30
    while not job.done():
        assert time.monotonic() < deadline
        time.sleep(1e-4)
    assert job.ticket != 0   # done() did not consume it
    job.wait()
    assert job.done() and torch.equal(s, d)


def test_async_gather_reduces_absmax_bits():
    """adfl_host_copy_submit_absmax: the staging gather of the host-resident SLQ encode reduces max|x| per
    tensor as it copies — the magnitude bits' unsigned max (NaN wins, -0 is 0, denormals kept), the value
    torch.max(torch.abs(t)) gives (quant.py:100) — whatever the piece split across threads."""
    rng = np.random.default_rng(9)
    sizes = [1, 3, 1_000_003, 70_000, 4, 2_000_000, 17]
    xs = [rng.standard_normal(n).astype(np.float32) * np.float32(10.0 ** (i - 3)) for i, n in enumerate(sizes)]
    xs[1][:] = [-0.0, 1e-40, -3e-45]                  # denormals only
    xs[2][123_457] = np.float32(np.inf) * -1          # -inf
    xs[4][2] = np.nan                                  # NaN wins
    xs[6][:] = 0.0
    srcs = [torch.from_numpy(x) for x in xs]
    bucket = torch.empty(sum(sizes))
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    amax = np.zeros(len(sizes), np.uint32)
    job = hostcopy.submit_pieces([bucket.data_ptr() + 4 * int(o) for o in offs], [s.data_ptr() for s in srcs],
                                 [4 * n for n in sizes], absmax_ptrs=np.uint64(amax.ctypes.data) +
                                 np.arange(len(sizes), dtype=np.uint64) * np.uint64(4), keep=(srcs, bucket, amax))
    job.wait()
    assert np.array_equal(bucket.numpy().view(np.uint32), np.concatenate(xs).view(np.uint32))
    for k, x in enumerate(xs):
        want = torch.max(torch.abs(torch.from_numpy(x))).numpy()
        got = amax[k:k + 1].view(np.float32)[0]
        assert (np.isnan(got) and np.isnan(want)) or got.view(np.uint32) == want.view(np.uint32), k
    with pytest.raises(Exception):   # pieces that are not whole fp32 words
        hostcopy.submit_pieces([bucket.data_ptr()], [srcs[2].data_ptr()], [6], absmax_ptrs=[amax.ctypes.data])
