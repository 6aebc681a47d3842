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
  all-gather's bus bandwidth; and `exchange_c3`, a ResNet-18-sized state dict per client exchanged as one
  bucket with per-tensor scales. Both check the gathered rows and the mean across ranks. Never part of
  `value`.

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

_T_START = time.perf_counter()  # bench_wall_s: process start to the line (the driver's run includes interpreter start)

import numpy as np
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
    p.add_argument("--extras", choices=("auto", "on", "off"), default="auto",
                   help="C3 / C5 int4 / host-inclusive (pcie) objects after the timed headline; auto = N=1 only")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--cpu-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--cpu-input", help=argparse.SUPPRESS)
    p.add_argument("--cpu-list", help=argparse.SUPPRESS)
    p.add_argument("--share-gpu", action="store_true", help=argparse.SUPPRESS)   # N ranks on cuda:0 over gloo (tests)
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


def dist_setup(args, backend: str = "nccl", share_gpu: bool = False):
    """One process per GPU (torchrun env: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*). `backend` is
    "nccl" (= RCCL) for the bench; tests drive the same code with "gloo" on CPU. share_gpu (the hidden
    --share-gpu): every rank on cuda:0 over gloo — the reference's two-clients-per-GPU packing
    (Examples/ray_ad.py:29), which RCCL cannot form — so the N-rank path runs on a one-GPU box.
    Returns (world, rank, device index)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl" or share_gpu:
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


def cpu_round_trips(x: torch.Tensor, bits: int, budget_s: float, first=None):
    """Best-of round-trip seconds of the reference's op sequence (quant.py:100-103,110) on host tensor x:
    >= 3 round trips (fewer only when one exceeds the budget), at most 5. `first(q, scale)` sees the first
    result. Returns (best seconds, runs)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import slq_oracle as oracle  # test infrastructure: the checker / baseline leg only
    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        q, scale = oracle.aten_encode(x, bits)
        d = oracle.aten_decode(q)
        times.append(time.perf_counter() - t0)
        if first is not None and len(times) == 1:
            first(q, scale)
        del q, d
        if len(times) >= 5 or (len(times) >= 3 and time.perf_counter() - t_start + min(times) > budget_s) \
                or time.perf_counter() - t_start > 2 * budget_s:
            break
    return min(times), len(times)


def cpu_child(args):
    """--cpu-child: one point of the CPU baseline sweep in a fresh process (never touches the GPU). Its
    OMP_NUM_THREADS comes from the parent; the affinity mask is set here, before the first parallel region
    creates ATen's thread pool, so every pool thread inherits it. Reads the bench's own 1 GiB input from
    --cpu-input and prints {"best_s", "runs", "threads", "affinity"}."""
    import numpy as np
    os.sched_setaffinity(0, [int(c) for c in args.cpu_list.split(",")])
    x = torch.from_numpy(np.fromfile(args.cpu_input, dtype=np.float32))
    x = x.reshape(SHAPE) if x.numel() == N_ELEMS else x.reshape(1, -1)
    best, runs = cpu_round_trips(x, args.bits, args.cpu_seconds)
    emit({"best_s": best, "runs": runs, "threads": torch.get_num_threads(),
          "affinity": len(os.sched_getaffinity(0))})


def cpu_sweep_points():
    """(label, cpus or None, threads) for the CPU baseline sweep: ATen's default (the job's share,
    OMP_NUM_THREADS, no pinning), 1 thread, every physical core of one socket, every physical core of both
    sockets (one hardware thread per core, pinned), and every CPU in the affinity mask (SMT included). The
    topology is sysfs's, restricted to this process's affinity mask."""
    allowed = sorted(os.sched_getaffinity(0))
    cores = {}
    for cpu in allowed:
        base = f"/sys/devices/system/cpu/cpu{cpu}/topology"
        try:
            with open(base + "/physical_package_id") as f:
                pkg = int(f.read())
            with open(base + "/core_id") as f:
                core = int(f.read())
        except (OSError, ValueError):
            pkg, core = 0, cpu
        cores.setdefault((pkg, core), []).append(cpu)
    first_thread = {k: min(v) for k, v in cores.items()}
    packages = sorted({p for p, _ in cores})
    pts = [("default", None, torch.get_num_threads()), ("1 thread", [allowed[0]], 1)]
    one = sorted(c for (p, _), c in first_thread.items() if p == packages[0])
    pts.append((f"socket {packages[0]} physical cores", one, len(one)))
    if len(packages) > 1:
        both = sorted(first_thread.values())
        pts.append((f"{len(packages)} sockets physical cores", both, len(both)))
    if len(allowed) > len(first_thread):
        pts.append(("all CPUs (SMT)", allowed, len(allowed)))
    return pts


def cpu_baseline(x_dev: torch.Tensor, bits: int, budget_s: float, q_dev: torch.Tensor, s_dev: torch.Tensor):
    """The reference's own op sequence (quant.py:100-103,110) on host cores, timed on the bench's own 1 GiB
    input over the sweep of cpu_sweep_points(). The default point runs in this process (and checks the GPU
    payload and scale against the reference ops on this very workload); every other point runs in a child
    process pinned to its CPUs before torch starts. `value`/`cores` report the fastest point."""
    import tempfile
    x = x_dev.cpu()
    parity = []
    points = cpu_sweep_points()
    share = budget_s / len(points)

    def check(q, scale):  # the GPU result on this very workload must equal the reference's
        parity.append(bool(torch.equal(q.int_repr(), q_dev.cpu())) and float(s_dev.item()) == scale)

    results = {}
    with tempfile.TemporaryDirectory(prefix="adfl_cpu_", dir="/tmp") as tmp:
        path = os.path.join(tmp, "x.f32")
        x.numpy().tofile(path)
        for label, cpus, threads in points:
            if cpus is None:
                best, runs = cpu_round_trips(x, bits, share, first=check)
                results[label] = {"threads": threads, "best_s": best, "runs": runs}
                continue
            env = {k: v for k, v in os.environ.items()
                   if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                "MASTER_PORT")}
            env.update(OMP_NUM_THREADS=str(threads), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
            cmd = [sys.executable, os.path.abspath(__file__), "--cpu-child", "--cpu-input", path,
                   "--cpu-list", ",".join(map(str, cpus)), "--bits", str(bits), "--cpu-seconds", str(share)]
            try:
                r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=60 + 4 * share)
                res = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None
            except (subprocess.TimeoutExpired, ValueError, IndexError):
                res = None
            results[label] = ({"threads": threads, "pinned_cpus": len(cpus), "best_s": res["best_s"],
                               "runs": res["runs"]} if res else {"threads": threads, "error": "child failed"})
    gib = x.numel() * 4 / GIB
    ok = {k: v for k, v in results.items() if "best_s" in v}
    best_label = min(ok, key=lambda k: ok[k]["best_s"])
    best = ok[best_label]["best_s"]
    cpu = {"value": round(gib / best, 3), "unit": "GiB/s", "cores": ok[best_label]["threads"], "kind": "port",
           "best_point": best_label,
           "sample": f"full 1 GiB round trip (torch.abs/max/quantize_per_tensor/dequantize, quant.py:100-110), "
                     f"best of >= 3 per point; points: " + ", ".join(f"{k} ({v['threads']} thr)"
                                                                      for k, v in results.items())
                     + f"; {os.cpu_count()} CPUs visible, {len(os.sched_getaffinity(0))} in the affinity mask",
           "cpu_model": cpu_model(), "ms_per_round_trip": round(best * 1e3, 1),
           "by_point": {k: ({"threads": v["threads"], "GiB_per_s": round(gib / v["best_s"], 3),
                             "ms_per_round_trip": round(v["best_s"] * 1e3, 1), "runs": v["runs"]}
                            if "best_s" in v else v) for k, v in results.items()}}
    return cpu, (all(parity) if parity else None)


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


RESNET18_PARAMS = 11_689_512          # C3: ResNet-18's parameter count in 256 tensors
C5_ELEMS = 1 << 30                    # C5: 4 GiB of fp32 per client


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def _ref_encode(t: torch.Tensor, bits: int):
    """The reference's own op sequence on a host tensor (Src/ADFL/Channel/quant.py:99-104): scale =
    max|t| / q_max in fp32 tensor math, then quantize_per_tensor with float(scale)."""
    scale = torch.max(torch.abs(t)) / (2 ** (bits - 1) - 1)
    return torch.quantize_per_tensor(t, float(scale), 0, torch.qint8), float(scale)


def extra_c3(dev, lib, steps: int) -> dict:
    """BASELINE configs[2] (C3) beside the headline: ResNet-18's 11,689,512 fp32 parameters in 256 equal tensors,
    one bucket with per-tensor scales (quant.py:74-94), device-resident, the Infinity Cache flushed by a 512 MiB
    READ before every step. Encode = ONE launch (k_encode_resident: a block per tensor, x read once), decode
    one launch. Fractions: on the bytes the two kernels move (encode 5 B + decode 5 B per element; the PMC
    passes count 1.004-1.008x that) and at the survey's 14 B/element round-trip count. parity: the
    payload, the 256 scales and the decoded floats against the reference's ATen ops per tensor."""
    from adfl_amd import _lib, ops
    base, rem = divmod(RESNET18_PARAMS, 256)
    sizes = [base + (1 if i < rem else 0) for i in range(256)]
    lay = ops.BucketLayout(sizes)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(lay.total, device=dev, generator=g) * 1e-3
    q = torch.empty(lay.total, dtype=torch.int8, device=dev)
    scales = torch.empty(lay.ntensors, device=dev)
    partials = torch.empty(lay.nchunks, dtype=torch.int32, device=dev)
    out = torch.zeros(lay.total, device=dev)
    chunks, work = lay.device_chunks(dev), lay.device_work(dev)
    junk = torch.ones(128 << 20, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def enc():
        _lib.check(lib.adfl_slq_encode_batched_work(x.data_ptr(), chunks.data_ptr(), lay.nchunks, work.data_ptr(),
                                                    lay.nwork, 8, q.data_ptr(), scales.data_ptr(),
                                                    partials.data_ptr(), sh))

    def dec():
        _lib.check(lib.adfl_slq_dequantize_batched(q.data_ptr(), chunks.data_ptr(), lay.nchunks, scales.data_ptr(),
                                                   out.data_ptr(), sh))
    for _ in range(3):
        junk.amax()
        enc()
        dec()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    rt = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
    for e in evs:           # encode and decode apart
        junk.amax()
        e[0].record(stream)
        enc()
        e[1].record(stream)
        dec()
        e[2].record(stream)
    for e in rt:            # the round trip as one span (no event between the launches)
        junk.amax()
        e[0].record(stream)
        enc()
        dec()
        e[1].record(stream)
    torch.cuda.synchronize()
    e_ms = _median([e[0].elapsed_time(e[1]) for e in evs])
    d_ms = _median([e[1].elapsed_time(e[2]) for e in evs])
    r_ms = _median([e[0].elapsed_time(e[1]) for e in rt])
    n = RESNET18_PARAMS
    frac = lambda b, ms: round(b * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)  # noqa: E731
    # parity against the reference's ATen ops, tensor by tensor (quant.py:97-112)
    xc, qc, sc, oc = x.cpu(), q.cpu(), scales.cpu(), out.cpu()
    ok = True
    for t, (o, m) in enumerate(zip(lay.offsets.tolist(), sizes)):
        qr, s = _ref_encode(xc[o:o + m].view(1, m), 8)
        ok = ok and float(sc[t]) == s and torch.equal(qr.int_repr().view(-1), qc[o:o + m]) \
            and torch.equal(qr.dequantize().view(-1), oc[o:o + m])
    return {"workload": "C3: 11,689,512 fp32 in 256 tensors (ResNet-18 size, equal layout), per-tensor scales, "
                        "bits=8, device-resident, Infinity Cache flushed by a 512 MiB read before each step",
            "steps": steps, "encode_launches": 1 if lay.nwork else 2, "encode_ms": round(e_ms, 4),
            "decode_ms": round(d_ms, 4), "round_trip_ms": round(r_ms, 4),
            "GiB_per_s": round(n * 4 / GIB / (r_ms * 1e-3), 1),
            "frac_moved": frac(10, r_ms), "encode_frac_moved": frac(5, e_ms), "decode_frac_moved": frac(5, d_ms),
            "frac_14B": frac(14, r_ms), "parity": bool(ok)}


def extra_c5(dev, lib, steps: int) -> dict:
    """BASELINE configs[4]'s codec (C5) beside the headline: 2^30 fp32 (4 GiB) per client, SLQ bits=4 packed
    two codes per byte (pack_4bit's layout, compression.py:35-48): absmax, fused quantize+pack, fused
    unpack+dequantize, HIP events per kernel. Bytes per element: absmax 4, quantize+pack 4.5, unpack+dequantize
    4.5 (13 per round trip). parity: the scale against max|x| / 7 (quant.py:99-100), every code against the
    reference's quantize_per_tensor on the host copy (the nibbles unpacked with torch ops), and the decoded
    floats against fp32(scale * code) (quant.py:110)."""
    from adfl_amd import _lib, ops
    n = C5_ELEMS
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    packed = torch.empty(n // 2, dtype=torch.uint8, device=dev)
    scale = torch.empty(1, device=dev)
    ws = ops.new_workspace(dev)
    out = torch.empty(n, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(e=None):
        if e is not None:
            e[0].record(stream)
        _lib.check(lib.adfl_slq_absmax(x.data_ptr(), n, ws.data_ptr(), ws.numel(), sh))
        if e is not None:
            e[1].record(stream)
        _lib.check(lib.adfl_slq_quantize_int4(x.data_ptr(), n, 4, ws.data_ptr(), packed.data_ptr(), scale.data_ptr(),
                                              sh))
        if e is not None:
            e[2].record(stream)
        _lib.check(lib.adfl_slq_dequantize_int4(packed.data_ptr(), n, scale.data_ptr(), out.data_ptr(), sh))
        if e is not None:
            e[3].record(stream)
    for _ in range(2):
        step()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    names = ("absmax", "quantize_pack", "unpack_dequantize")
    ms = {k: _median([e[i].elapsed_time(e[i + 1]) for e in evs]) for i, k in enumerate(names)}
    per = dict(zip(names, (4.0, 4.5, 4.5)))
    rt = sum(ms.values())
    xc = x.cpu()
    qr, s = _ref_encode(xc, 4)
    del xc
    ok = float(scale.item()) == s
    qd = qr.int_repr().to(dev)
    del qr
    hi = (packed >> 4).to(torch.int16) - 8
    lo = (packed & 15).to(torch.int16) - 8
    ok = ok and torch.equal(hi, qd[0::2].to(torch.int16)) and torch.equal(lo, qd[1::2].to(torch.int16))
    ok = ok and torch.equal(out.view(torch.int32), (qd.to(torch.float32) * scale).view(torch.int32))
    return {"workload": "C5: 2^30 fp32 (4 GiB) per client, SLQ bits=4, pack_4bit layout, device-resident",
            "steps": steps, "kernels_ms": {k: round(v, 4) for k, v in ms.items()},
            "kernels_frac": {k: round(per[k] * n / (ms[k] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for k in names},
            "round_trip_ms": round(rt, 4), "GiB_per_s": round(n * 4 / GIB / (rt * 1e-3), 1),
            "frac_13B": round(13 * n / (rt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "parity": bool(ok)}


def extra_pcie(dev, lib, steps: int) -> dict:
    """The rate that includes the host hops (north_star: the path starts and ends in host memory, ADFL's Ray
    loopback): (1) the 1 GiB C2 round trip from and to pinned host memory — H2D of x (4N), encode, the payload
    D2H and back H2D (2N), decode, D2H of the output (4N); (2) ADFL's own call pattern: a CPU ResNet-18-sized
    state dict (256 weights + 256 biases) through SLQChannel.on_client_send then on_server_receive, host to
    host, as Src/ADFL/Client/worker.py:176 and Src/ADFL/Server/async_sc.py:209 call it. parity: both against
    the reference's ATen ops on the same host tensors (quant.py:97-112)."""
    from adfl_amd import _lib, ops
    from adfl_amd.Channel import SLQChannel
    n = N_ELEMS
    x_h = (torch.randn(n, generator=torch.Generator().manual_seed(7)) * 1e-3).pin_memory()
    q_h = torch.empty(n, dtype=torch.int8).pin_memory()
    out_h = torch.empty(n).pin_memory()
    x = torch.empty(n, device=dev)
    q = torch.empty(n, dtype=torch.int8, device=dev)
    q2 = torch.empty(n, dtype=torch.int8, device=dev)
    s = torch.empty(1, device=dev)
    out = torch.empty(n, device=dev)
    ws = ops.new_workspace(dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(e=None):
        rec = (lambda i: e[i].record(stream)) if e is not None else (lambda i: None)
        rec(0)
        x.copy_(x_h, non_blocking=True)
        rec(1)
        _lib.check(lib.adfl_slq_encode(x.data_ptr(), n, 8, q.data_ptr(), s.data_ptr(), ws.data_ptr(), ws.numel(), sh))
        rec(2)
        q_h.copy_(q, non_blocking=True)
        q2.copy_(q_h, non_blocking=True)   # the payload crosses the host "wire" and comes back
        rec(3)
        _lib.check(lib.adfl_slq_dequantize(q2.data_ptr(), n, s.data_ptr(), out.data_ptr(), sh))
        rec(4)
        out_h.copy_(out, non_blocking=True)
        rec(5)
    step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(steps)]
    t0 = time.perf_counter()
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    segs = {k: round(_median([e[i].elapsed_time(e[i + 1]) for e in evs]), 4)
            for i, k in enumerate(("h2d_x", "encode", "payload_d2h_h2d", "decode", "d2h_out"))}
    pcie_ms = segs["h2d_x"] + segs["payload_d2h_h2d"] + segs["d2h_out"]
    qr, sr = _ref_encode(x_h, 8)
    pinned_ok = float(s.item()) == sr and torch.equal(qr.int_repr(), q_h) and torch.equal(qr.dequantize(), out_h)
    del qr, x, q, q2, out, x_h, q_h, out_h

    dict_leg = channel_c3_dict(steps)
    return {"pinned_1GiB": {"workload": "C2's 1 GiB fp32 from and to pinned host memory (10N bytes over PCIe)",
                            "steps": steps, "ms_per_round_trip": round(wall * 1e3, 3),
                            "GiB_per_s": round(n * 4 / GIB / wall, 2), "segments_ms": segs,
                            "pcie_GBs": round(10 * n / (pcie_ms * 1e-3) / 1e9, 1), "parity": bool(pinned_ok)},
            "channel_c3_dict": dict_leg}


def channel_c3_dict(steps: int) -> dict:
    """ADFL's own host call pattern on C3: SLQChannel(8).on_client_send then on_server_receive of a CPU
    state dict of 256 weights (11,689,512 fp32) + 256 biases (Src/ADFL/Client/worker.py:176,
    Src/ADFL/Server/async_sc.py:209), medians of the calls, with the calling thread's wall time per internal
    phase (quant.phase_clock: gather + absmax, H2D enqueue, output allocation, D2H wait, scatter, ...;
    "other" is the rest of the call)."""
    from adfl_amd.Channel import SLQChannel, quant
    base, rem = divmod(RESNET18_PARAMS, 256)
    g = torch.Generator().manual_seed(11)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
    ch = SLQChannel(8)
    enc_t, dec_t, enc_ph, dec_ph = [], [], [], []
    qp = dp = None
    for k in range(3 + max(steps, 10)):
        dp = None  # the previous round's results are released outside the timed calls
        qp = None
        with quant.phase_clock() as ce:
            t1 = time.perf_counter()
            qp, _ = ch.on_client_send(params)
            t2 = time.perf_counter()
        with quant.phase_clock() as cd:
            t3 = time.perf_counter()
            dp, _ = ch.on_server_receive(qp)
            t4 = time.perf_counter()
        if k >= 3:
            enc_t.append(t2 - t1)
            dec_t.append(t4 - t3)
            ce.ms["other"] = (t2 - t1) * 1e3 - sum(ce.ms.values())
            cd.ms["other"] = (t4 - t3) * 1e3 - sum(cd.ms.values())
            enc_ph.append(ce.ms)
            dec_ph.append(cd.ms)
    dict_ok = True
    for name, t in params.items():
        if t.ndim > 1:
            qr, _ = _ref_encode(t, 8)
            dict_ok = dict_ok and torch.equal(qp.params[name].data.int_repr(), qr.int_repr()) \
                and qp.params[name].data.q_scale() == qr.q_scale() and torch.equal(dp[name], qr.dequantize())
        else:
            dict_ok = dict_ok and torch.equal(dp[name], t)

    def phases(rows):
        keys = sorted({k for r in rows for k in r})
        return {k: round(_median([r.get(k, 0.0) for r in rows]), 3) for k in keys}
    e_ms, d_ms = _median(enc_t) * 1e3, _median(dec_t) * 1e3
    gib_dict = sum(t.numel() for t in params.values()) * 4 / GIB
    return {"workload": "SLQChannel(8).on_client_send + on_server_receive on a CPU state dict "
                        "of 256 weights (11,689,512 fp32) + 256 biases, host to host",
            "rounds": len(enc_t), "encode_ms": round(e_ms, 3), "decode_ms": round(d_ms, 3),
            "round_trip_ms": round(e_ms + d_ms, 3),
            "GiB_per_s": round(gib_dict / ((e_ms + d_ms) * 1e-3), 2),
            "phases_ms": {"encode": phases(enc_ph), "decode": phases(dec_ph)},
            "statistic": "median of the calls (phases: median per phase); the previous round's results are "
                         "freed before each timed call", "parity": bool(dict_ok)}


def c3_sizes(layout: str) -> list:
    """C3's 256 tensor sizes (tests/golden/recipes.bucket_sizes): "equal" (11,689,512 / 256) or
    "loguniform" (seed-0 log-uniform draws in [64, 2.4 M] scaled to the same total)."""
    if layout == "equal":
        base, rem = divmod(RESNET18_PARAMS, 256)
        return [base + (1 if i < rem else 0) for i in range(256)]
    import math
    rng = np.random.default_rng(0)
    raw = np.exp(rng.uniform(math.log(64), math.log(2_400_000), size=256))
    sizes = np.maximum(64, np.floor(raw / raw.sum() * RESNET18_PARAMS)).astype(np.int64)
    sizes[int(np.argmax(sizes))] += RESNET18_PARAMS - int(sizes.sum())
    return [int(v) for v in sizes]


def _stoch_want(name: str, scale: float, data: torch.Tensor, signs: torch.Tensor, levels: int) -> torch.Tensor:
    """The reference's _dequantize_tensor arithmetic on a payload (quant.py:251-252 QSGD, :545 CNAT), in fp32."""
    if name == "qsgd":
        return (scale * data.float() / levels) * signs.float()
    return scale * signs.float() * (2 ** data.float())


def _stoch_layout_leg(dev, sizes, seed: int, steps: int) -> dict:
    """One C3 layout through the stochastic channels the reference's experiments run (QSGDChannel(8) beside
    SLQChannel(8), Src/main.py:229,488), with the reference's own L2 norm (torch's CPU vector_norm order,
    csrc/torch_norm.hip; quant.py:226,512): (1) host to host, QSGDChannel(8) / CNATChannel(8) built with the
    reference's constructor, on_client_send then on_server_receive of a CPU state dict (the weights + 256 biases),
    medians of the calls, with the calling thread's per-phase medians (quant.phase_clock); (2) device-resident, the
    bucket's encode (norm + levels + signs, Philox uniforms) and decode, each timed by HIP events behind an
    Infinity-Cache flush. parity: every weight's scale equals torch.linalg.vector_norm of the tensor (the
    reference's scale) and every decoded tensor equals the reference's _dequantize_tensor arithmetic on the payload;
    on the device, the norms equal torch's and the decode equals that arithmetic (torch's own ops on the device).
    (The levels follow the Philox stream, not torch's mt19937 draws: compared with a reference run only
    statistically — tests/.)"""
    from adfl_amd import ops, stoch
    from adfl_amd.Channel import CNATChannel, QSGDChannel, quant
    g = torch.Generator().manual_seed(seed)
    params = {}
    for i, m in enumerate(sizes):
        params[f"layer{i}.weight"] = torch.randn(1, m, generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
    ref_norms = {k: torch.linalg.vector_norm(t).item() for k, t in params.items() if t.ndim > 1}
    out = {}

    def phases(rows):
        keys = sorted({k for r in rows for k in r})
        return {k: round(_median([r.get(k, 0.0) for r in rows]), 3) for k in keys}
    for name, cls in (("qsgd", QSGDChannel), ("cnat", CNATChannel)):
        ch = cls(8)
        enc_t, dec_t, enc_ph, dec_ph = [], [], [], []
        qp = dp = None
        for k in range(3 + max(steps, 5)):
            dp = qp = None
            with quant.phase_clock() as ce:
                t1 = time.perf_counter()
                qp, _ = ch.on_client_send(params)
                t2 = time.perf_counter()
            with quant.phase_clock() as cd:
                t3 = time.perf_counter()
                dp, _ = ch.on_server_receive(qp)
                t4 = time.perf_counter()
            if k >= 3:
                enc_t.append(t2 - t1)
                dec_t.append(t4 - t3)
                ce.ms["other"] = (t2 - t1) * 1e3 - sum(ce.ms.values())
                cd.ms["other"] = (t4 - t3) * 1e3 - sum(cd.ms.values())
                enc_ph.append(ce.ms)
                dec_ph.append(cd.ms)
        ok = True
        for k, t in params.items():
            p = qp.params[k]
            if t.ndim <= 1:
                ok = ok and torch.equal(dp[k], t)
                continue
            ok = ok and p.scale == ref_norms[k]
            want = _stoch_want(name, p.scale, p.data, p.signs, ch.levels)
            ok = ok and torch.equal(dp[k].view(torch.int32), want.view(torch.int32))
        e_ms, d_ms = _median(enc_t) * 1e3, _median(dec_t) * 1e3
        out[f"{name}_host"] = {"encode_ms": round(e_ms, 3), "decode_ms": round(d_ms, 3),
                               "round_trip_ms": round(e_ms + d_ms, 3), "rounds": len(enc_t),
                               "phases_ms": {"encode": phases(enc_ph), "decode": phases(dec_ph)}, "parity": bool(ok)}
    # device-resident encode + decode of the same bucket (norm in torch's order + levels + signs; decode)
    lay = ops.BucketLayout(sizes, align=1)
    x = torch.cat([params[f"layer{i}.weight"].view(-1) for i in range(len(sizes))]).to(dev)
    want_n = torch.tensor([ref_norms[f"layer{i}.weight"] for i in range(len(sizes))], dtype=torch.float32)
    out.update(_stoch_device_legs(dev, x, lay, want_n, steps))
    return out


def _stoch_device_legs(dev, x: torch.Tensor, lay, want_norms: torch.Tensor, steps: int) -> dict:
    """QSGD / CNAT (bits 8) device encode with the reference's norm, then decode, of the bucket x: median HIP-event
    ms of each behind an Infinity-Cache flush, the reference-order norm's own share, and parity (norms equal
    want_norms — torch.linalg.vector_norm on the host — and the decode equals the reference's arithmetic computed
    by torch on the device)."""
    from adfl_amd import stoch
    lv = torch.empty(lay.total, dtype=torch.uint8, device=dev)
    sg = torch.empty(lay.total, dtype=torch.int8, device=dev)
    nrm = torch.empty(lay.ntensors, device=dev)
    dq = torch.empty(lay.total, device=dev)
    ws = stoch.workspace(lay, dev)
    junk = torch.ones(128 << 20, device=dev)
    stream = torch.cuda.current_stream(dev)
    reps = max(steps, 10)
    levels = (1 << 8) - 1
    out = {}

    def timed(fn):
        fn()
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(reps)]
        for e in evs:
            junk.amax()
            e[0].record(stream)
            fn()
            e[1].record(stream)
        torch.cuda.synchronize()
        return _median([e[0].elapsed_time(e[1]) for e in evs])
    norm_ms = timed(lambda: stoch.reference_norms(x, lay, out32=nrm))
    gib = lay.total * 4 / GIB
    for name in ("qsgd", "cnat"):
        if name == "qsgd":
            enc = lambda: stoch.qsgd_encode_batched(x, lay, 8, seed=1, levels=lv, signs=sg, norms=nrm, ws=ws,  # noqa: E731
                                                    torch_norm=True)
            dec = lambda: stoch.qsgd_decode_batched(lv, sg, nrm, lay, 8, out=dq)  # noqa: E731
        else:
            enc = lambda: stoch.cnat_encode_batched(x, lay, 8, seed=1, exps=lv.view(torch.int8), signs=sg,  # noqa: E731
                                                    norms=nrm, ws=ws, torch_norm=True)
            dec = lambda: stoch.cnat_decode_batched(lv.view(torch.int8), sg, nrm, lay, out=dq)  # noqa: E731
        e_ms = timed(enc)
        d_ms = timed(dec)
        ok = torch.equal(nrm.cpu().view(torch.int32), want_norms.view(torch.int32))
        if lay.total == int(lay.sizes.sum()):   # compact: element e belongs to tensor searchsorted(ends, e)
            # the decode against the reference's arithmetic on the host (torch's device division is not
            # correctly rounded, the reference's CPU one is): every element up to 2^24, else 2^22 seeded positions
            idx = (torch.arange(lay.total, device=dev) if lay.total <= (1 << 24) else
                   torch.randint(0, lay.total, (1 << 22,), device=dev, generator=torch.Generator(device=dev).manual_seed(5)))
            ends = torch.as_tensor(np.cumsum(lay.sizes), device=dev)
            nr = nrm[torch.searchsorted(ends, idx, right=True)].cpu()
            data = (lv if name == "qsgd" else lv.view(torch.int8))[idx].cpu()
            sgc = sg[idx].cpu().float()
            want = (nr * data.float() / levels) * sgc if name == "qsgd" else nr * sgc * (2 ** data.float())
            ok = ok and torch.equal(dq[idx].cpu().view(torch.int32), want.view(torch.int32))
        out[f"{name}_device"] = {"encode_ms": round(e_ms, 4), "decode_ms": round(d_ms, 4),
                                 "round_trip_GiB_per_s": round(gib / ((e_ms + d_ms) * 1e-3), 1),
                                 "parity": bool(ok)}
    out["reference_norm_ms"] = round(norm_ms, 4)
    return out


def extra_stoch_c3(dev, lib, steps: int) -> dict:
    """The stochastic channels with the reference's norm on both C3 layouts (_stoch_layout_leg)."""
    out = {"workload": "C3: a CPU state dict of 256 weights (11,689,512 fp32) + 256 biases, bits=8, the reference's "
                       "L2 norm; 'equal' and 'loguniform' layouts (SURVEY.md §8d)"}
    for layout, seed in (("equal", 13), ("loguniform", 14)):
        out[layout] = _stoch_layout_leg(dev, c3_sizes(layout), seed, steps)
    return out


def extra_stoch_c2(dev, lib, steps: int) -> dict:
    """C2's 1 GiB flat fp32 gradient through QSGD / CNAT bits 8 on the device with the reference's norm (the
    default of QSGDChannel(8) / CNATChannel(8)): encode and decode (_stoch_device_legs), parity against
    torch.linalg.vector_norm of the same tensor on the host."""
    from adfl_amd import ops
    g = torch.Generator().manual_seed(17)
    xc = torch.randn(1 << 28, generator=g) * 1e-3
    want = torch.linalg.vector_norm(xc).reshape(1).to(torch.float32)
    x = xc.to(dev)
    del xc
    lay = ops.BucketLayout([1 << 28], align=1)
    out = {"workload": "C2: one 2^28-element fp32 tensor, QSGD / CNAT bits=8, the reference's L2 norm"}
    out.update(_stoch_device_legs(dev, x, lay, want, steps))
    return out


_FP_MUL = -7046029254386353131        # 0x9E3779B97F4A7C15 as int64 (golden-ratio multiplier)


def fingerprint(t: torch.Tensor) -> int:
    """A 64-bit, position-sensitive fingerprint of t's bytes, computed where t lives (wrapping int64
    arithmetic): sum over 8-byte words w_i of mix(w_i * M + i), mix(y) = y ^ (y >> 29). Equal bytes give
    equal fingerprints; a flipped, lost or misplaced word changes it except with negligible probability."""
    b = t.detach().reshape(-1).view(torch.uint8)
    if b.numel() % 8:
        b = torch.cat([b, b.new_zeros(8 - b.numel() % 8)])
    w = b.view(torch.int64)
    y = w * _FP_MUL + torch.arange(w.numel(), device=w.device, dtype=torch.int64)
    y = y ^ (y >> 29)
    return int(y.sum().item())


def exchange_verify(ex, flat: torch.Tensor, world: int) -> dict:
    """Checks the exchange leg's last all-gather and mean on every rank (run after the timed steps):
    * rows:  every rank all-gathers the fingerprint of each of its own message rows; every received row,
             on every rank and chunk, must match its sender's fingerprint, and row `rank` must equal the
             local row byte for byte — the RCCL/xGMI transport delivered exactly what was sent;
    * mean:  one exact_self=False mean (all K decoded payloads in rank order) must be bit-identical on every
             rank (fingerprints all-gathered).
    The verdict is agreed over ranks (MIN all-reduce), so every rank reports the same `parity`."""
    import torch.distributed as dist
    works = ex.encode_and_gather(flat)
    for w in works:
        if w is not None:
            w.wait()
    own_ok = all(torch.equal(g[ex.rank], loc) for g, loc in zip(ex.gathered, ex.local))
    sent = [None] * world
    dist.all_gather_object(sent, [fingerprint(loc) for loc in ex.local])
    bad_rows = [(r, c) for c, g in enumerate(ex.gathered) for r in range(world) if fingerprint(g[r]) != sent[r][c]]
    saved = ex.exact_self
    ex.exact_self = False
    try:
        m = ex.mean([None] * len(works))
    finally:
        ex.exact_self = saved
    means = [None] * world
    dist.all_gather_object(means, fingerprint(m))
    mean_ok = len(set(means)) == 1
    ok = own_ok and not bad_rows and mean_ok
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                        device=flat.device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return {"parity": bool(flag.item()), "own_row_equal": own_ok, "rows_checked": world * len(ex.gathered),
            "rows_mismatched": bad_rows[:8], "mean_identical_on_all_ranks": mean_ok,
            "mean_fingerprint": f"{means[0] & 0xFFFFFFFFFFFFFFFF:016x}"}


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
    check = exchange_verify(ex, flat, world)        # after the timed steps: never inside them
    return {"workload": f"C4: {world} simulated clients x 1 GiB fp32, SLQ bits={bits} encode + RCCL "
                        f"all_gather_into_tensor + fused decode-mean", "steps": steps,
            "parity": check.pop("parity"), "check": check,
            "ms_per_step": round(t * 1e3, 4), "GiB_per_s": round(world * n * 4 / GIB / t, 2),
            "encode_ms": round(seg[0], 4), "allgather_wait_ms": round(seg[1], 4), "mean_ms": round(seg[2], 4),
            "bytes_per_rank_on_wire": ex.bytes_per_rank,
            "allgather_busbw_GBs": round(recv / (seg[1] * 1e-3) / 1e9, 1) if world > 1 and seg[1] > 0 else None,
            # rccl-tests convention: algbw = gathered bytes / time; busbw = algbw * (n - 1) / n
            "allgather_algbw_GBs": (round(world * ex.bytes_per_rank / (seg[1] * 1e-3) / 1e9, 1)
                                    if world > 1 and seg[1] > 0 else None),
            "backend": dist.get_backend()}


def exchange_bucket_leg(dev, bits: int, world: int, steps: int, warmup: int):
    """BASELINE configs[2] exchanged as configs[3] does: every rank's ResNet-18-sized state dict
    (11,689,512 fp32 in 256 equal tensors, one bucket, SLQChannel's per-tensor scales) encoded, all-gathered
    over RCCL as one row (payload + 256 scales) and averaged per tensor in one launch (adfl_amd.exchange
    with a BucketLayout; Examples/ray_ad.py:164-190). Checked like the C4 leg. Never part of `value`."""
    import torch.distributed as dist
    from adfl_amd import ops
    from adfl_amd.exchange import PeerExchange

    base, rem = divmod(11_689_512, 256)
    lay = ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)])
    rank = dist.get_rank()
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    flat = torch.zeros(lay.total, device=dev)
    for o, n in zip(lay.offsets.tolist(), lay.sizes.tolist()):
        flat[o:o + n] = torch.randn(n, device=dev, generator=g) * 1e-3
    out = torch.empty(lay.total, device=dev)
    ex = PeerExchange(lay.total, bits=bits, device=dev, layout=lay)
    for _ in range(warmup):
        ex.exchange_mean(flat, out)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ex.exchange_mean(flat, out)
    torch.cuda.synchronize()
    barrier(world)
    t = max_over_ranks(time.perf_counter() - t0, world) / steps
    check = exchange_verify(ex, flat, world)
    return {"workload": f"C3 state dict per client: {world} clients x 11,689,512 fp32 in 256 tensors, SLQ bits={bits} "
                        f"per-tensor scales, RCCL all_gather_into_tensor of one bucket row + per-tensor fused mean",
            "steps": steps, "parity": check.pop("parity"), "check": check, "ms_per_step": round(t * 1e3, 4),
            "bytes_per_rank_on_wire": ex.bytes_per_rank,
            "GiB_per_s": round(world * int(lay.sizes.sum()) * 4 / GIB / t, 2)}


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
    if args.cpu_child:
        return cpu_child(args)
    world, rank, local = dist_setup(args, "gloo" if args.share_gpu else "nccl", args.share_gpu)
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
        try:
            exchange_c3 = exchange_bucket_leg(dev, args.bits, world, min(args.steps, 20), min(args.warmup, 3))
        except Exception as e:  # noqa: BLE001
            exchange_c3 = {"error": f"{type(e).__name__}: {e}"[:400]}

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
    cold_ms = per_kernel["absmax"] + per_kernel["quantize"] + decode_cold
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
        # the receiver-side round trip: a peer decodes a payload that did not just leave its own encode
        "cold_round_trip": {"kernel_ms": round(cold_ms, 4), "GiB_per_s": round(gib_per_rank / (cold_ms * 1e-3), 2),
                            "achieved_GBs": round(14 * n / (cold_ms * 1e-3) / 1e9, 1),
                            "frac": round(14 * n / (cold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "copy_ceiling_GBs": round(copy_ceiling, 1),
        "round_trip_roofline": {"alg_bytes": 14 * n, "kernel_ms": round(kernels_ms, 4),
                                "achieved_GBs": round(14 * n / (kernels_ms * 1e-3) / 1e9, 1),
                                "frac": round(14 * n / (kernels_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "wall_frac": round(14 * n / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "cpu_baseline": None,
    }
    if exchange is not None:
        line["exchange"] = exchange
        line["exchange_c3"] = exchange_c3
    if args.extras == "on" or (args.extras == "auto" and world == 1):
        # BASELINE's other single-GPU configs and the host-inclusive rate, after the timed headline (never in
        # `value`); each carries its own parity against the reference's ATen ops
        for key, fn, st in (("c3", extra_c3, 20), ("c5_int4", extra_c5, 10), ("pcie", extra_pcie, 5),
                            ("stoch_c3", extra_stoch_c3, 5), ("stoch_c2", extra_stoch_c2, 5)):
            try:
                line[key] = fn(dev, lib, st)
            except Exception as e:  # noqa: BLE001
                line[key] = {"error": f"{type(e).__name__}: {e}"[:400]}
            torch.cuda.empty_cache()
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
    line["bench_wall_s"] = round(time.perf_counter() - _T_START, 1)
    emit(line)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
