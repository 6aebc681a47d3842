"""bench.py's output contract on the GPU (the line the driver parses): exactly one JSON line on stdout with the
headline keys, n_gpus = 1, a roofline object for the dominant kernel, and value consistent with ms_per_step.
A short run: 3 timed steps, no CPU baseline, no PMC passes, no exchange leg, no extras (each is covered
elsewhere)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_emits_one_contract_line():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--pmc", "off", "--exchange", "off", "--extras", "off"],
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
                        "--no-cpu-baseline", "--pmc", "off", "--exchange", "on", "--extras", "off"],
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


@pytest.mark.timeout(240)
def test_bench_eight_ranks_share_one_gpu():
    """The driver's 8-GPU command shape, rehearsed on one GPU: bench.py --gpus 8 starts
    eight rank processes itself, each a simulated client on cuda:0 (hidden --share-gpu: gloo, host-staged
    rows), runs its timed round trips, then both exchange legs at K = 8 — the C4 1 GiB update and the
    ResNet-18-sized bucket (Examples/ray_ad.py:175,183-188) — and exchange_verify over 8 row sets: every
    received row's fingerprint equals its sender's, and the exact_self=False mean is identical on all ranks."""
    import time
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--pmc", "off", "--share-gpu"],
                       cwd=REPO, capture_output=True, text=True, timeout=230)
    wall = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "independent clients x8"
    assert abs(d["value"] - 8.0 / (d["ms_per_step"] * 1e-3)) / d["value"] < 0.01
    for leg in ("exchange", "exchange_c3"):
        ex = d[leg]
        assert "error" not in ex, (leg, ex)
        assert ex["parity"] is True, (leg, ex)
        assert ex["check"]["rows_checked"] == 8 and ex["check"]["mean_identical_on_all_ranks"], (leg, ex)
    assert d["exchange"]["backend"] == "gloo"
    print(f"8-rank share-gpu bench: {wall:.1f} s wall; exchange {d['exchange']['ms_per_step']} ms/step, "
          f"C3 bucket exchange {d['exchange_c3']['ms_per_step']} ms/step")
    assert wall < 150, wall


def test_bench_extras_c3_c5_pcie():
    """The objects bench.py adds after the timed headline at N = 1: C3 (ResNet-18-sized
    bucket, flushed), C5 (4 GiB int4 round trip) and the host-inclusive rates (pinned 1 GiB round trip, the C3
    CPU dict through SLQChannel), each with its parity against the reference's ATen ops true."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--pmc", "off", "--exchange", "off", "--extras", "on"],
                       cwd=REPO, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    c3, c5, pc = d["c3"], d["c5_int4"], d["pcie"]
    for o in (c3, c5, pc):
        assert "error" not in o, o
    assert c3["parity"] is True and c3["encode_launches"] == 1 and 0 < c3["frac_14B"] < 1, c3
    assert abs(c3["frac_14B"] / c3["frac_moved"] - 1.4) < 1e-2
    assert c5["parity"] is True and set(c5["kernels_ms"]) == {"absmax", "quantize_pack", "unpack_dequantize"}, c5
    assert 0 < c5["frac_13B"] < 1
    assert pc["pinned_1GiB"]["parity"] is True and pc["channel_c3_dict"]["parity"] is True, pc
    assert pc["pinned_1GiB"]["pcie_GBs"] > 1 and pc["channel_c3_dict"]["round_trip_ms"] > 0
