"""GPU: the event-gated submit path of the native host-copy pool (adfl_host_copy_submit with
adfl_event_synchronize as the wait callback; hostcopy.submit_pieces(event=...)).

The pool's workers must not read a pinned source before the D2H that fills it has landed: a copy submitted
behind a HIP event recorded after a long kernel and that D2H must deliver the D2H's bytes, not the stale
ones the pinned buffer held at submit time — while the submitting thread is free (submit returns at once).
"""

import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from adfl_amd import hostcopy  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("pieces", [1, 7])
def test_copy_waits_for_the_event(pieces):
    n = 1 << 26                                 # a 256 MiB D2H: milliseconds on the link, so it is still running
    pinned = torch.full((n,), -1.0).pin_memory()
    dst = torch.zeros(n)
    src_dev = torch.arange(n, dtype=torch.float32, device=DEV)
    stream = torch.cuda.current_stream(DEV)
    scratch = torch.empty(n).pin_memory()
    cuts = np.linspace(0, n, pieces + 1).astype(np.int64)
    es = 4
    d = [dst.data_ptr() + int(a) * es for a in cuts[:-1]]
    s = [pinned.data_ptr() + int(a) * es for a in cuts[:-1]]
    b = [int(c - a) * es for a, c in zip(cuts[:-1], cuts[1:])]
    # ~40 ms of D2H queued in front of the one the copy waits for; on a loaded host this thread can be
    # descheduled for longer than that, so the gate grows until the event is still pending at submit
    for gate in (8, 32, 128):
        torch.cuda.synchronize()
        for _ in range(gate):
            scratch.copy_(src_dev, non_blocking=True)
        pinned.copy_(src_dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        t0 = time.perf_counter()
        job = hostcopy.submit_pieces(d, s, b, event=ev, keep=(pinned, dst))
        submit_s = time.perf_counter() - t0
        if not ev.query():                      # the D2H is still behind the others: the copy must wait
            break
        job.wait()
        pinned.fill_(-1.0)
        dst.zero_()
    else:
        pytest.skip("every gate's D2H had landed before submit returned (host descheduled): not exercised")
    job.wait()
    assert ev.query()
    assert torch.equal(dst, src_dev.cpu()), "copied before the event completed"
    assert submit_s < 0.05                      # submit does not block on the event


def test_many_jobs_behind_one_event_keep_order():
    """Several jobs behind one event, each into its own destination; every one sees the landed bytes."""
    n = 1 << 20
    pinned = torch.zeros(n).pin_memory()
    src_dev = torch.randn(n, device=DEV)
    torch.cuda.synchronize()
    torch.cuda._sleep(50_000_000)
    pinned.copy_(src_dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(DEV))
    outs = [torch.empty(n) for _ in range(4)]
    jobs = [hostcopy.submit_pieces([o.data_ptr()], [pinned.data_ptr()], [4 * n], event=ev, keep=(pinned, o))
            for o in outs]
    for j in jobs:
        j.wait()
    want = src_dev.cpu()
    for o in outs:
        assert torch.equal(o, want)


def test_job_keeps_its_event_and_buffers_alive():
    """The job, not the caller, keeps the event (and the buffers it names) alive until every part has run: a
    caller that drops its own references right after submitting must not leave the workers waiting on a
    destroyed event (the range-pipelined host paths record a fresh event per range)."""
    import gc
    n = 1 << 21
    src_dev = torch.randn(n, device=DEV)
    pinned = torch.zeros(n).pin_memory()
    dst = torch.zeros(n)
    torch.cuda.synchronize()
    torch.cuda._sleep(20_000_000)
    pinned.copy_(src_dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(DEV))
    job = hostcopy.submit_pieces([dst.data_ptr()], [pinned.data_ptr()], [4 * n], event=ev, keep=pinned)
    want = None
    del ev, pinned
    gc.collect()
    job.wait()
    want = src_dev.cpu()
    assert torch.equal(dst, want)
