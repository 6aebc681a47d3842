"""bench.py's output contract on the GPU (the line the driver parses): exactly one JSON line on stdout with the
headline keys, n_gpus = 1, a roofline object for the dominant kernel, and value consistent with ms_per_step.
A short run: 3 timed steps, no CPU baseline, no PMC passes, no exchange leg (each is covered elsewhere)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_emits_one_contract_line():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--pmc", "off", "--exchange", "off"],
                       cwd=REPO, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["unit"] == "GiB/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["workload"].startswith("C2") and d["config"]["elements_per_gpu"] == 1 << 28
    # value = 1 GiB per step / step time
    assert abs(d["value"] - 1.0 / (d["ms_per_step"] * 1e-3)) / d["value"] < 0.01
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert 0.0 < rf["frac"] < 1.0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["alg_bytes_per_launch"] > 0 and rf["avg_launch_ms"] > 0
    assert d["cpu_baseline"] is None  # --no-cpu-baseline
    # the receiver-side round trip: absmax + quantize + a decode whose payload is not in the Infinity Cache
    cr = d["cold_round_trip"]
    assert abs(cr["kernel_ms"] - (d["kernels_ms"]["absmax"] + d["kernels_ms"]["quantize"] + d["decode_cold_ms"])) < 2.5e-4  # four 4-decimal roundings
    assert 0.0 < cr["frac"] < 1.0 and cr["GiB_per_s"] > 0


def test_bench_exchange_leg_checks_itself():
    """The C4 exchange leg at world 1 over RCCL (--exchange on): after its timed steps it verifies the
    gathered rows against the sent rows and the exact_self=False mean across ranks, and says so."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--pmc", "off", "--exchange", "on"],
                       cwd=REPO, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    ex = d["exchange"]
    assert "error" not in ex, ex
    assert ex["parity"] is True, ex
    assert ex["check"]["own_row_equal"] and ex["check"]["rows_checked"] == 1 and ex["backend"] == "nccl"
    c3 = d["exchange_c3"]   # the ResNet-18-sized state dict exchanged as one bucket
    assert "error" not in c3, c3
    assert c3["parity"] is True and c3["check"]["rows_checked"] == 1, c3
    assert c3["bytes_per_rank_on_wire"] > 11_689_512 and c3["GiB_per_s"] > 0


def test_bench_two_ranks_share_one_gpu():
    """bench.py --gpus 2 end to end on a one-GPU box (hidden --share-gpu: both ranks on cuda:0, gloo): the
    launcher, both ranks' timed round trips, the max over ranks, rank 0's single line with n_gpus 2 and
    value = 2 GiB per step, and the exchange leg (host-staged all-gather) verifying itself across ranks."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--pmc", "off", "--share-gpu"],
                       cwd=REPO, capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "independent clients x2"
    assert abs(d["value"] - 2.0 / (d["ms_per_step"] * 1e-3)) / d["value"] < 0.01
    ex = d["exchange"]
    assert "error" not in ex, ex
    assert ex["parity"] is True and ex["backend"] == "gloo", ex
    assert ex["check"]["rows_checked"] == 2 and ex["check"]["mean_identical_on_all_ranks"]
    c3 = d["exchange_c3"]
    assert "error" not in c3, c3
    assert c3["parity"] is True and c3["check"]["rows_checked"] == 2 and c3["check"]["mean_identical_on_all_ranks"]
