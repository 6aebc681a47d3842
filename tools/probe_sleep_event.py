"""Probe (GPU): whether a non_blocking D2H into pinned memory, enqueued behind torch.cuda._sleep and a fill
on the same stream, waits for them — fresh vs reused pinned buffers, null vs side stream — with the event
recorded after it, its query right after record, its completion time and the copied data checked
(tests/test_gpu_hostcopy_event.py::test_copy_waits_for_the_event failed once: event landed within 1.8 ms)."""
import time

import torch

dev = torch.device("cuda", 0)
n = 1 << 24
src = torch.zeros(n, dtype=torch.float32, device=dev)
reused = torch.full((n,), -1.0).pin_memory()
side = torch.cuda.Stream(dev)
torch.cuda.synchronize()
for k in range(12):
    fresh = k % 3 == 0
    use_side = k % 2 == 1
    s = side if use_side else torch.cuda.current_stream(dev)
    dst = torch.full((n,), -1.0).pin_memory() if fresh else reused
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        t0 = time.perf_counter()
        torch.cuda._sleep(100_000_000)
        src.fill_(float(k + 1))
        t_a = time.perf_counter() - t0
        dst.copy_(src, non_blocking=True)
        t_b = time.perf_counter() - t0
        ev = torch.cuda.Event()
        ev.record(s)
    q0 = ev.query()
    t_q = time.perf_counter() - t0
    while not ev.query():
        time.sleep(0.0002)
    t_done = time.perf_counter() - t0
    ok = bool((dst == float(k + 1)).all())
    print(f"rep {k:2d} fresh={fresh} side={use_side}: sleep+fill enqueue {t_a*1e3:6.2f} ms, copy enqueue "
          f"{(t_b - t_a)*1e3:6.2f} ms, pending after record {not q0} ({t_q*1e3:.2f} ms), event done at "
          f"{t_done*1e3:6.2f} ms, data ok {ok}", flush=True)
