"""CPU, world_size 2 (gloo): bench.py's multi-rank plumbing — torchrun-style env setup, barrier and the
max-over-ranks step time the whole-job value is computed from."""

import os
import socket
import sys

import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    try:
        os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, repo)
        import bench
        import torch.distributed as dist
        w, r, local = bench.dist_setup(None, backend="gloo")
        assert (w, r, local) == (world, rank, rank)
        bench.barrier(w)
        slowest = bench.max_over_ranks(0.5 + rank, w)     # rank 1 is the slow one
        value = w * 1.0 / slowest                          # bench.py: world * GiB / max step time
        q.put((rank, slowest, value))
        dist.destroy_process_group()
    except Exception as e:  # surfaced in the parent
        q.put((rank, "error", repr(e)))


def test_bench_max_over_ranks_gloo():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] != "error" for r in res), res
    assert sorted(res) == [(0, 1.5, 2 / 1.5), (1, 1.5, 2 / 1.5)]


def _run_bench(argv, env_extra=None, timeout=180):
    import json
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + argv, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, [json.loads(ln) for ln in lines]


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` outside torchrun starts two rank processes itself (the driver's scaling run),
    and the line it prints is rank 0's, with n_gpus == 2 and the slowest rank's time."""
    r, lines = _run_bench(["--gpus", "2", "--plumbing-check"])
    assert r.returncode == 0, r.stderr
    assert len(lines) == 1, r.stdout                     # one JSON line, from rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2
    assert sorted(tuple(x) for x in line["ranks"]) == [(0, 0), (1, 1)]
    assert line["max_over_ranks_s"] >= 0.1               # rank 1 spins 2 x 50 ms: its time is the max


def test_bench_gpus1_runs_in_process():
    r, lines = _run_bench(["--gpus", "1", "--plumbing-check"])
    assert r.returncode == 0, r.stderr
    assert lines[0]["n_gpus"] == 1 and lines[0]["ranks"] == [[0, 0]]


def test_bench_refuses_gpus_world_size_mismatch():
    r, lines = _run_bench(["--gpus", "2", "--plumbing-check"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and not lines
    assert "disagrees with WORLD_SIZE" in r.stderr


def test_bench_failing_rank_fails_launch():
    """A rank that dies makes the launcher exit non-zero instead of hanging at the barrier."""
    r, lines = _run_bench(["--gpus", "3", "--plumbing-check"], {"ADFL_PLUMBING_FAIL_RANK": "1"})
    assert r.returncode == 3 and not lines


def test_cpu_sweep_points_cover_the_physical_core_counts():
    """The CPU baseline sweep (bench.cpu_sweep_points): the default point unpinned, then 1 thread and the
    physical cores of one socket (and of every socket when there are several), pinned, each CPU list inside
    this process's affinity mask and one hardware thread per core."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import bench
    pts = bench.cpu_sweep_points()
    labels = [p[0] for p in pts]
    assert labels[0] == "default" and pts[0][1] is None
    assert labels[1] == "1 thread" and pts[1][2] == 1
    assert any("physical cores" in lbl for lbl in labels)
    allowed = os.sched_getaffinity(0)
    for label, cpus, threads in pts[1:]:
        assert set(cpus) <= allowed and len(cpus) == threads, label


def test_cpu_child_times_the_reference_ops_pinned(tmp_path):
    """One sweep point in its own process: pinned to the given CPUs, reads the input file, prints its
    best-of round trip as the one JSON line."""
    import numpy as np
    path = tmp_path / "x.f32"
    (np.random.default_rng(0).standard_normal(1 << 16, dtype=np.float32) * np.float32(1e-3)).tofile(path)
    cpu = sorted(os.sched_getaffinity(0))[0]
    r, lines = _run_bench(["--cpu-child", "--cpu-input", str(path), "--cpu-list", str(cpu), "--cpu-seconds", "0.05"],
                          {"OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, r.stderr
    assert len(lines) == 1 and lines[0]["affinity"] == 1 and lines[0]["threads"] == 1
    assert lines[0]["runs"] >= 3 and lines[0]["best_s"] > 0
