"""Headline benchmark: device-resident SLQ quantize+dequantize of a 1 GiB fp32 gradient per GPU.

Metric (BASELINE.json): "GiB/s device-resident quantize+dequantize, 1 GiB fp32 grads, 1/2/4/8 GPU".
One step = one round trip of the hot path over one 1 GiB fp32 buffer already resident in HBM
(BASELINE.json configs[1], shape [262144, 1024], randn * 1e-3): encode (absmax pass + quantize pass,
quant.py:97-104) then decode (quant.py:107-112), 3 HIP launches. With N GPUs (torchrun, one process per
GPU) every rank round-trips its own 1 GiB client update concurrently (weak scaling, no collective in the
data path); value = N GiB / max-over-ranks time per step.

Also reported on the same line:
* roofline — the dominant kernel's algorithmic bytes / its average launch time, measured with HIP
  events on the launch stream inside the timed region, against the 8.0 TB/s HBM3E peak; `traffic` is
  that kernel's HBM bytes per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over the same
  workload, run as child processes after the timed region (N=1; `--pmc off` or a failed pass falls back
  to the committed profiles/pmc_traffic.json while its kernel-source hash matches);
* cpu_baseline — the reference's ATen op sequence (quant.py:100-103,110) timed on this host's cores
  (rank 0, N=1), over a bounded sample of the same workload;
* exchange (N > 1, or --exchange on) — BASELINE configs[3] (C4) on the same buffers after the timed
  headline: encode + RCCL all-gather of the int8 payloads over xGMI + fused decode-mean, with the
  all-gather's bus bandwidth. Never part of `value`.

    python bench.py [--gpus N] [--steps K] [--warmup W]

`--gpus N` with N > 1 outside torchrun starts N rank processes of this script itself (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set per child, one free 127.0.0.1 port) before anything touches the GPU, and exits
with their status; under torchrun WORLD_SIZE must equal --gpus.
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))

GIB = 1 << 30
N_ELEMS = 1 << 28                 # 1 GiB of fp32
SHAPE = (262144, 1024)
HBM_PEAK_GBS = 8000.0             # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes per fp32 element, per kernel
KERNEL_BYTES = {"absmax": 4, "quantize": 5, "dequantize": 5}
KERNEL_SYMBOLS = {"absmax": "k_absmax_flat", "quantize": "k_quantize_flat", "dequantize": "k_dequantize_flat"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--bits", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget for the CPU baseline sample")
    p.add_argument("--exchange", choices=("auto", "on", "off"), default="auto",
                   help="C4 peer-exchange leg (encode + RCCL all-gather + decode-mean); auto = only when N > 1")
    p.add_argument("--pmc", choices=("auto", "off"), default="auto",
                   help="roofline.traffic from live rocprofv3 PMC passes (auto: N=1 only, after the timed region)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--plumbing-check", action="store_true",
                   help="CPU-only check of the rank launcher / barrier / max-over-ranks (gloo); no GPU, no bench")
    return p.parse_args()


_JSON_FD = None


def reserve_stdout() -> None:
    """The driver reads ONE JSON line from stdout, but RCCL prints its banner (version, host, library path)
    to fd 1 when a process group starts. Keep the real stdout for the JSON line only and send everything
    else written to fd 1 — by this process, torch or RCCL — to stderr."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj) -> None:
    data = (json.dumps(obj) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(data.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, data)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n_gpus: int, script: str, argv) -> int:
    """Run `script argv` as `n_gpus` rank processes, one per GPU (the torchrun contract: RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT). The caller must not have touched the GPU. If a rank
    fails, the others are terminated (they would otherwise wait at a barrier). Returns the exit status:
    0, or the first failing rank's."""
    port = free_port()
    procs = []
    for r in range(n_gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_gpus),
                   LOCAL_WORLD_SIZE=str(n_gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    status = 0
    try:
        while procs:
            for p in list(procs):
                rc = p.poll()
                if rc is None:
                    continue
                procs.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    for q in procs:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for q in procs:
            q.kill()
    return status


def maybe_launch(n_gpus: int, script: str, argv) -> "int | None":
    """Multi-GPU entry: None when this process is the (only) rank to run — N=1, or a rank already started by
    torchrun / launch_ranks — otherwise the exit status of the N ranks it started."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != n_gpus:
            raise SystemExit(f"bench: --gpus {n_gpus} disagrees with WORLD_SIZE={env_world}; "
                             f"launch with torchrun --nproc-per-node {n_gpus} or without torchrun")
        return None
    if n_gpus < 1:
        raise SystemExit(f"bench: --gpus must be >= 1, got {n_gpus}")
    if n_gpus == 1:
        return None
    return launch_ranks(n_gpus, script, argv)


def dist_setup(args, backend: str = "nccl"):
    """One process per GPU (torchrun env: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*). `backend` is
    "nccl" (= RCCL) for the bench; tests drive the same code with "gloo" on CPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        import datetime
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        # a stuck collective fails in minutes rather than torch's default 10
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=180), **kw)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(v: float, world: int) -> float:
    """The slowest rank's value (the step time the whole job sees)."""
    if world == 1:
        return v
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_child(args):
    """--pmc-child: the bench workload alone (no timing, no baseline), the program rocprofv3 --pmc runs."""
    from adfl_amd import ops
    from adfl_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(SHAPE, device=dev, generator=g) * 1e-3).contiguous()
    q = torch.empty(SHAPE, dtype=torch.int8, device=dev)
    scale = torch.empty(1, dtype=torch.float32, device=dev)
    ws = ops.new_workspace(dev)
    out = torch.empty(SHAPE, dtype=torch.float32, device=dev)
    n = x.numel()
    for _ in range(args.steps):
        _lib.check(lib.adfl_slq_absmax(x.data_ptr(), n, ws.data_ptr(), ws.numel(), sh))
        _lib.check(lib.adfl_slq_quantize(x.data_ptr(), n, args.bits, ws.data_ptr(), q.data_ptr(), scale.data_ptr(), sh))
        _lib.check(lib.adfl_slq_dequantize(q.data_ptr(), n, scale.data_ptr(), out.data_ptr(), sh))
    torch.cuda.synchronize()


def pmc_live(bits: int, steps: int = 4, timeout_s: float = 120.0):
    """HBM bytes per launch of every bench kernel, measured in this run: two rocprofv3 passes (FETCH_SIZE and
    WRITE_SIZE cannot share one: TCC slots) over `bench.py --pmc-child`, started as child processes after the
    timed region. gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of a 16-B
    per lane streaming read, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) KiB. Returns ({kernel: bytes}, note);
    bytes is None if rocprofv3 is missing or a pass fails (the bench line never fails on it)."""
    import csv
    import glob
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    vals = {}
    with tempfile.TemporaryDirectory(prefix="adfl_pmc_", dir="/tmp") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", str(steps), "--bits", str(bits)]
            env = dict(os.environ, TMPDIR="/tmp")
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
                env.pop(k, None)
            try:
                r = subprocess.run(cmd, cwd="/tmp", env=env, timeout=timeout_s, stdout=subprocess.DEVNULL,
                                   stderr=subprocess.PIPE)
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 --pmc {counter} timed out"
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} exited {r.returncode}: {r.stderr.decode()[-300:]}"
            acc = {}
            for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(path) as f:
                    for row in csv.DictReader(f):
                        if row.get("Counter_Name") != counter:
                            continue
                        for sym in KERNEL_SYMBOLS.values():
                            if sym in row.get("Kernel_Name", ""):
                                acc.setdefault(sym, []).append(float(row["Counter_Value"]))
            vals[counter] = {k: sum(v) / len(v) for k, v in acc.items()}
    out = {}
    for sym in KERNEL_SYMBOLS.values():
        f, w = vals["FETCH_SIZE"].get(sym), vals["WRITE_SIZE"].get(sym)
        out[sym] = None if f is None or w is None else int((2 * f + w) * 1024)
    return out, f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over {steps} child steps, this run"


def pmc_traffic(kernel: str):
    """Fallback when the live passes are off or fail: HBM bytes per launch from the committed PMC summary
    (profiles/pmc_traffic.json), only while the kernel source it was measured on is the one built now (its
    SHA-256 is recorded by tools/pmc_summary.py); a stale or missing summary gives None."""
    import hashlib
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    src = os.path.join(REPO, "ad-federatedlearning_amd", "csrc", "slq_codec.hip")
    try:
        with open(path) as f:
            d = json.load(f)
        with open(src, "rb") as f:
            if d.get("kernel_source_sha256") != hashlib.sha256(f.read()).hexdigest():
                return None
        return d["kernels"][KERNEL_SYMBOLS[kernel]]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(x_dev: torch.Tensor, bits: int, budget_s: float, q_dev: torch.Tensor, s_dev: torch.Tensor):
    """The reference's own op sequence (quant.py:100-103,110) on host cores, timed on the full 1 GiB workload
    at three thread counts — ATen's default (the job's share of cores, OMP_NUM_THREADS), 1, and
    os.cpu_count() — best of >= 3 round trips each (fewer only if one round trip exceeds the budget).
    `value`/`cores` report the fastest of the three."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import slq_oracle as oracle  # test infrastructure: the checker / baseline leg only

    default_threads = torch.get_num_threads()
    x = x_dev.cpu()
    parity = None
    per_threads = {}
    counts = []
    for t in (default_threads, 1, os.cpu_count() or default_threads):
        if t not in counts:
            counts.append(t)
    share = budget_s / len(counts)
    for threads in counts:
        torch.set_num_threads(threads)
        times = []
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            q, scale = oracle.aten_encode(x, bits)
            d = oracle.aten_decode(q)
            times.append(time.perf_counter() - t0)
            if parity is None:  # the GPU result on this very workload must equal the reference's
                parity = bool(torch.equal(q.int_repr(), q_dev.cpu())) and float(s_dev.item()) == scale
            del q, d
            if len(times) >= 5 or (len(times) >= 3 and time.perf_counter() - t_start + min(times) > share) \
                    or time.perf_counter() - t_start > 2 * share:
                break
        per_threads[threads] = (min(times), len(times))
    torch.set_num_threads(default_threads)
    gib = x.numel() * 4 / GIB
    best_threads = min(per_threads, key=lambda k: per_threads[k][0])
    best = per_threads[best_threads][0]
    cpu = {"value": round(gib / best, 3), "unit": "GiB/s", "cores": best_threads, "kind": "port",
           "sample": f"full 1 GiB round trip (torch.abs/max/quantize_per_tensor/dequantize, quant.py:100-110), "
                     f"best of >= 3 per thread count, thread counts {counts}; {os.cpu_count()} CPUs visible, "
                     f"{len(os.sched_getaffinity(0))} in this process's affinity mask",
           "cpu_model": cpu_model(), "ms_per_round_trip": round(best * 1e3, 1),
           "by_threads": {str(t): {"GiB_per_s": round(gib / v[0], 3), "ms_per_round_trip": round(v[0] * 1e3, 1),
                                   "runs": v[1]} for t, v in per_threads.items()}}
    return cpu, parity


def cold_decode_ms(lib, qp, n, sp, op, stream, reps: int = 10) -> float:
    """Decode with the Infinity Cache holding none of the payload: a 512 MiB read between the encode and the
    decode evicts it (a READ, so no dirty lines drain into the timed decode). The timed headline decodes
    right after the encode, and decode starts on the payload bytes the encode wrote last;
    a receiving peer decodes a payload that arrived from elsewhere — this number."""
    from adfl_amd import _lib
    junk = torch.ones(128 << 20, dtype=torch.float32, device=stream.device)
    sh = stream.cuda_stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        junk.amax()
        e0.record(stream)
        _lib.check(lib.adfl_slq_dequantize(qp, n, sp, op, sh))
        e1.record(stream)
    torch.cuda.synchronize()
    del junk
    return sorted(e0.elapsed_time(e1) for e0, e1 in evs)[reps // 2]


def copy_ceiling_GBs(x: torch.Tensor, out: torch.Tensor, stream, reps: int = 10) -> float:
    """The device-to-device copy ceiling of this GPU (SURVEY.md §8d asks for it beside the roofline): torch's
    own 1 GiB fp32 copy (read 1 GiB + write 1 GiB), median of `reps` HIP-event timings on the launch stream.
    Reported only; the roofline fraction stays against the 8.0 TB/s spec peak."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    with torch.cuda.stream(stream):
        out.copy_(x)
        for e0, e1 in evs:
            e0.record(stream)
            out.copy_(x)
            e1.record(stream)
    torch.cuda.synchronize()
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)[reps // 2]
    return 2 * x.numel() * x.element_size() / (ms * 1e-3) / 1e9


def exchange_leg(x: torch.Tensor, out: torch.Tensor, bits: int, world: int, steps: int, warmup: int):
    """BASELINE configs[3] (C4) on the same buffers: every rank is one simulated client that encodes its
    1 GiB update, all-gathers the int8 payloads (+ scale trailers) over RCCL and decodes the K payloads
    into their fp32 mean in one fused launch (adfl_amd.exchange; Examples/ray_ad.py:164-190). Reported
    beside the headline, never as `value`. Segments are HIP events on the compute stream: the stream
    waits on the all-gather, so [encode end, wait] is the collective as the codec sees it."""
    import torch.distributed as dist
    from adfl_amd.exchange import PeerExchange

    n = x.numel()
    ex = PeerExchange(n, bits=bits, device=x.device)
    flat, flat_out = x.reshape(-1), out.reshape(-1)
    stream = torch.cuda.current_stream(x.device)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        works = ex.encode_and_gather(flat)
        if ev is not None:
            ev[1].record(stream)
        for w in works:
            w.wait()
        if ev is not None:
            ev[2].record(stream)
        ex.mean([None] * len(works), flat_out)
        if ev is not None:
            ev[3].record(stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(evs[k])
    torch.cuda.synchronize()
    barrier(world)
    t = max_over_ranks(time.perf_counter() - t0, world) / steps
    seg = [max_over_ranks(sum(e[i].elapsed_time(e[i + 1]) for e in evs) / steps, world) for i in range(3)]
    recv = ex.bytes_per_rank * (world - 1)          # bytes each rank receives (rccl-tests: busbw)
    return {"workload": f"C4: {world} simulated clients x 1 GiB fp32, SLQ bits={bits} encode + RCCL "
                        f"all_gather_into_tensor + fused decode-mean", "steps": steps,
            "ms_per_step": round(t * 1e3, 4), "GiB_per_s": round(world * n * 4 / GIB / t, 2),
            "encode_ms": round(seg[0], 4), "allgather_wait_ms": round(seg[1], 4), "mean_ms": round(seg[2], 4),
            "bytes_per_rank_on_wire": ex.bytes_per_rank,
            "allgather_busbw_GBs": round(recv / (seg[1] * 1e-3) / 1e9, 1) if world > 1 and seg[1] > 0 else None,
            "backend": dist.get_backend()}


def plumbing_check(args):
    """--plumbing-check: the N-rank path of this script without a GPU (gloo): every rank joins, reports
    itself, spins for (rank + 1) * 50 ms between the two barriers, and rank 0 prints the max over ranks."""
    world, rank, _ = dist_setup(args, backend="gloo")
    import torch.distributed as dist
    if os.environ.get("ADFL_PLUMBING_FAIL_RANK") == str(rank):   # tests: a rank that dies before the barrier
        sys.exit(3)
    barrier(world)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.05 * (rank + 1):
        pass
    barrier(world)
    slowest = max_over_ranks(time.perf_counter() - t0, world)
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, (rank, int(os.environ.get("LOCAL_RANK", "0"))))
    else:
        ranks = [(0, 0)]
    if rank == 0:
        emit({"plumbing_check": True, "n_gpus": world, "ranks": ranks, "max_over_ranks_s": round(slowest, 4)})
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    args = parse()
    rc = maybe_launch(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    reserve_stdout()
    if args.plumbing_check:
        return plumbing_check(args)
    if args.pmc_child:
        return pmc_child(args)
    world, rank, local = dist_setup(args)
    assert world == args.gpus, (world, args.gpus)
    from adfl_amd import ops
    from adfl_amd import _lib

    lib = _lib.load()
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    g = torch.Generator(device=dev).manual_seed(rank)
    x = (torch.randn(SHAPE, device=dev, generator=g) * 1e-3).contiguous()
    n = x.numel()
    q = torch.empty(SHAPE, dtype=torch.int8, device=dev)
    scale = torch.empty(1, dtype=torch.float32, device=dev)
    ws = ops.new_workspace(dev)
    out = torch.empty(SHAPE, dtype=torch.float32, device=dev)
    xp, qp, sp, wp, op = x.data_ptr(), q.data_ptr(), scale.data_ptr(), ws.data_ptr(), out.data_ptr()
    wsb = ws.numel()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        _lib.check(lib.adfl_slq_absmax(xp, n, wp, wsb, sh))
        if ev is not None:
            ev[1].record(stream)
        _lib.check(lib.adfl_slq_quantize(xp, n, args.bits, wp, qp, sp, sh))
        if ev is not None:
            ev[2].record(stream)
        _lib.check(lib.adfl_slq_dequantize(qp, n, sp, op, sh))
        if ev is not None:
            ev[3].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, world)

    decode_cold = cold_decode_ms(lib, qp, n, sp, op, stream)
    copy_ceiling = copy_ceiling_GBs(x, out, stream)

    exchange = None
    if args.exchange == "on" or (args.exchange == "auto" and world > 1):
        if world == 1:
            import torch.distributed as dist
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                                    device_id=dev)
        try:  # never at the cost of the headline line: a failure is reported in the `exchange` object
            exchange = exchange_leg(x, out, args.bits, world, min(args.steps, 20), min(args.warmup, 3))
        except Exception as e:  # noqa: BLE001
            exchange = {"error": f"{type(e).__name__}: {e}"[:400]}

    per_kernel = {name: sum(e[i].elapsed_time(e[i + 1]) for e in events) / args.steps
                  for i, name in enumerate(("absmax", "quantize", "dequantize"))}
    ms_per_step = elapsed / args.steps * 1e3
    gib_per_rank = n * 4 / GIB
    value = world * gib_per_rank / (elapsed / args.steps)

    if rank != 0:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return
    dominant = max(per_kernel, key=per_kernel.get)
    alg_bytes = KERNEL_BYTES[dominant] * n
    achieved = alg_bytes / (per_kernel[dominant] * 1e-3) / 1e9
    kernels_ms = sum(per_kernel.values())
    line = {
        "metric": "GiB/s device-resident quantize+dequantize, 1 GiB fp32 grads, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (torch.randn * 1e-3 on device, seed = rank)",
        "config": {"workload": "C2: 1 GiB fp32 flat gradient [262144,1024] per GPU, SLQ bits=8 encode+decode",
                   "bits": args.bits, "elements_per_gpu": n, "parallelism": f"independent clients x{world}"},
        "roofline": {"bound": "hbm", "kernel": KERNEL_SYMBOLS[dominant], "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic(dominant), "traffic_source": "profiles/pmc_traffic.json",
                     "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(per_kernel[dominant], 4)},
        "kernels_ms": {k: round(v, 4) for k, v in per_kernel.items()},
        "decode_cold_ms": round(decode_cold, 4),
        "copy_ceiling_GBs": round(copy_ceiling, 1),
        "round_trip_roofline": {"alg_bytes": 14 * n, "kernel_ms": round(kernels_ms, 4),
                                "achieved_GBs": round(14 * n / (kernels_ms * 1e-3) / 1e9, 1),
                                "frac": round(14 * n / (kernels_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "wall_frac": round(14 * n / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "cpu_baseline": None,
    }
    if exchange is not None:
        line["exchange"] = exchange
    if world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(x, args.bits, args.cpu_seconds, q, scale)
        line["cpu_baseline"] = cpu
        line["parity_vs_reference_ops"] = parity
    under_profiler = any(k.startswith("ROCPROF") for k in os.environ)   # rocprofv3 configures its tool via env
    if world == 1 and args.pmc == "auto" and not under_profiler:
        live, note = pmc_live(args.bits)
        if live is not None and live.get(KERNEL_SYMBOLS[dominant]) is not None:
            line["roofline"]["traffic"] = live[KERNEL_SYMBOLS[dominant]]
            line["roofline"]["traffic_source"] = note
            line["traffic_by_kernel"] = {k: {"hbm_bytes": v, "over_alg": round(v / (KERNEL_BYTES[name] * n), 4)}
                                         for name, k in KERNEL_SYMBOLS.items() if (v := live.get(k)) is not None}
        else:
            line["roofline"]["traffic_live_error"] = note
    emit(line)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
