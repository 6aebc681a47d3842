"""Probe (GPU): tests/test_gpu_hostcopy_event.py::test_copy_waits_for_the_event's sequence, repeated, with
the event's query before and after the pool submit, the time the event completes and whether the pool's
copy read the landed D2H (dst equal to the device data) — to tell a misreported query from an early copy."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "ad-federatedlearning_amd")
from adfl_amd import hostcopy  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 24
for rep in range(8):
    pieces = 1 if rep % 2 == 0 else 7
    pinned = torch.full((n,), -1.0).pin_memory()
    dst = torch.zeros(n)
    src_dev = torch.arange(n, dtype=torch.float32, device=dev) + rep
    stream = torch.cuda.current_stream(dev)
    cuts = np.linspace(0, n, pieces + 1).astype(np.int64)
    d = [dst.data_ptr() + int(a) * 4 for a in cuts[:-1]]
    s = [pinned.data_ptr() + int(a) * 4 for a in cuts[:-1]]
    b = [int(c - a) * 4 for a, c in zip(cuts[:-1], cuts[1:])]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(100_000_000)
    pinned.copy_(src_dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(stream)
    t_enq = time.perf_counter() - t0
    q_before = ev.query()
    job = hostcopy.submit_pieces(d, s, b, event=ev, keep=(pinned, dst))
    t_sub = time.perf_counter() - t0
    q_after = ev.query()
    t_q = time.perf_counter() - t0
    job.wait()
    t_job = time.perf_counter() - t0
    q_end = ev.query()
    ok = torch.equal(dst, src_dev.cpu())
    print(f"rep {rep} pieces {pieces}: enqueue {t_enq*1e3:.2f} ms, query before submit {q_before}, submit done "
          f"{t_sub*1e3:.2f} ms, query after {q_after} ({t_q*1e3:.2f} ms), job done {t_job*1e3:.2f} ms, query at end "
          f"{q_end}, dst == device data {ok}", flush=True)
