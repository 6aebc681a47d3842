"""CPU: the restatement of torch 2.10's fp32 full-reduction order (oracle/slq_oracle.c oracle_torch_sum_f32)
and of the reference's q-error metrics (oracle_qerror_ref, slq_oracle.qerror_metrics), pinned three ways:

* oracle_torch_sum_f32 == torch.sum itself, run here, at sizes across every branch (n < 8, the 8-lane
  vectors, the 32-value ILP groups, the cascade's level steps 16 / 32, the 32,768 grain and the two-pass
  split) and thread counts 1 .. 16;
* the metrics == the reference's own doubles for every client of tests/golden/aggregate_manifest.json
  (Src/ADFL/model.py:256-323 executed in place, small dicts) — bit for bit;
* the metrics == tests/golden/qerror_manifest.json (the reference executed on a ResNet-18-sized dict and on
  tensors around the grain, at 1 / 3 / 8 / 16 threads: tests/golden/make_golden_qerror.py).

Also the host side of csrc/qerror_ref.hip: adfl_qerror_ref_plan's split equals at::parallel_for's.
"""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

import slq_oracle as so

from make_golden_aggregate import client_arrays  # noqa: E402
import make_golden_qerror as mgq  # noqa: E402
import recipes  # noqa: E402


def _bits(v: float) -> int:
    return int(np.float32(v).view(np.uint32))


SIZES = [1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 129, 511, 512, 513, 1000, 4095, 4096,
         8191, 8192, 8193, 16385, 32767, 32768, 32769, 65535, 65536, 65537, 100003, 262147, 524289, 1 << 20]


@pytest.mark.parametrize("threads", [1, 2, 3, 5, 8, 16])
def test_sum_order_equals_torch(threads):
    rng = np.random.default_rng(threads)
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        for n in SIZES:
            x = (rng.standard_normal(n) * np.exp2(rng.integers(-12, 12, n))).astype(np.float32)
            want = torch.sum(torch.from_numpy(x)).item()
            got = so.torch_sum_f32(x, threads)
            assert _bits(got) == _bits(want), (threads, n, got, want)
    finally:
        torch.set_num_threads(old)


@pytest.mark.parametrize("n,threads", [((1 << 24) + 17, 1), ((1 << 24) + 17, 3), (20_000_001, 16)])
def test_sum_order_equals_torch_large(n, threads):
    """Level step 32 (more than 2^19 groups in one range) and long two-pass ranges."""
    x = np.random.default_rng(n).standard_normal(n).astype(np.float32)
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        want = torch.sum(torch.from_numpy(x)).item()
    finally:
        torch.set_num_threads(old)
    assert _bits(so.torch_sum_f32(x, threads)) == _bits(want)


def test_squared_difference_sums_equal_torch():
    """torch.sum((a - b) ** 2): the elementwise square rounds once per op, then the same order."""
    rng = np.random.default_rng(5)
    for threads in (1, 4, 8):
        old = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            for n in (7, 1000, 40_000, 300_001):
                a = rng.standard_normal(n).astype(np.float32)
                b = (a + rng.standard_normal(n).astype(np.float32) * np.float32(1e-3)).astype(np.float32)
                want = torch.sum((torch.from_numpy(a) - torch.from_numpy(b)) ** 2).item()
                df = (a - b).astype(np.float32)
                assert _bits(so.torch_sum_f32((df * df).astype(np.float32), threads)) == _bits(want)
        finally:
            torch.set_num_threads(old)


def _decode(xs, bits):
    L = so.lib()
    ds = []
    for x in xs:
        xf = np.ascontiguousarray(x.reshape(-1), dtype=np.float32)
        q = np.zeros(xf.size, np.int8)
        sc = L.oracle_slq_encode(so._ptr(xf), xf.size, bits, so._ptr(q))
        d = np.zeros(xf.size, np.float32)
        L.oracle_slq_dequantize(so._ptr(q), xf.size, sc, so._ptr(d))
        ds.append(d)
    return ds


def _same(a, b):
    return (np.isnan(a) and np.isnan(b)) or a == b


@pytest.mark.parametrize("bits", [8, 4])
def test_metrics_equal_reference_small_dicts(bits):
    m = json.load(open(os.path.join(GOLDEN, "aggregate_manifest.json")))
    for c in range(len(m["clients"])):
        arr = client_arrays(c)
        xs = [arr[n] for n in arr if arr[n].ndim > 1]
        mse, cos = so.qerror_metrics(xs, _decode(xs, bits), 8)
        ref = m["q_error"][f"slq{bits}_c{c}"]
        assert _same(mse, float(ref["mse"])) and _same(cos, float(ref["cos"])), (bits, c, mse, ref)


def _manifest_dict(name):
    m = json.load(open(os.path.join(GOLDEN, "qerror_manifest.json")))
    e = m["dicts"][name]
    spec = mgq.dicts()[name]
    xs = [recipes.randn(s, e["seed0"] + i, mult) for i, (_, s, mult) in enumerate(spec)]
    for (n, _, _), x in zip(spec, xs):
        assert recipes.sha256(x) == e["sha256"][n]
    return e, [x for x in xs if x.ndim > 1]


@pytest.mark.parametrize("name", ["edges", "resnet18"])
def test_metrics_equal_reference_model_sizes(name):
    e, xs = _manifest_dict(name)
    for bits in mgq.BITS:
        ds = _decode(xs, bits)
        for t in mgq.THREADS:
            mse, cos = so.qerror_metrics(xs, ds, t)
            ref = e["metrics"][f"slq{bits}_t{t}"]
            assert mse == float(ref["mse"]) and cos == float(ref["cos"]), (name, bits, t, mse, cos, ref)


def test_plan_split_equals_parallel_for():
    """adfl_qerror_ref_plan (host code): one site per tensor plus the cosine's over the concatenation; a
    site of n >= 32768 elements with T > 1 threads splits into min(T, ceil(n / 32768)) ranges of ceil(n / nt)."""
    from adfl_amd import _lib
    L = _lib.load()
    sizes = np.array([5, 32767, 32768, 100003, 7], dtype=np.int64)
    for threads in (1, 3, 8):
        need = L.adfl_qerror_ref_plan(sizes.ctypes.data, len(sizes), threads, None, 0)
        assert need > 0
        plan = np.zeros(need // 8, dtype=np.int64)
        assert L.adfl_qerror_ref_plan(sizes.ctypes.data, len(sizes), threads, plan.ctypes.data, need) == need
        assert L.adfl_qerror_ref_scratch_bytes(plan.ctypes.data) > 0
        nsites, nsegs, off_sites, off_segs = plan[1], plan[2], plan[6], plan[7]
        assert nsites == len(sizes) + 1
        total = int(sizes.sum())
        seen = 0
        for si, n in enumerate(list(sizes) + [total]):
            site = plan[off_sites + 8 * si: off_sites + 8 * si + 8]
            nt = 1
            if n >= 32768 and threads > 1:
                nt = min(threads, -(-n // 32768))
            cs = -(-n // nt)
            assert site[4] == nt and site[7] == (1 if n >= 32768 and threads > 1 else 0)
            for t in range(nt):
                seg = plan[off_segs + 8 * (site[3] + t): off_segs + 8 * (site[3] + t) + 8]
                assert seg[1] == min(cs, n - t * cs) and seg[0] == site[0] + t * cs
            seen += nt
        assert seen == nsegs
    assert L.adfl_qerror_ref_plan(sizes.ctypes.data, 0, 8, None, 0) < 0
    assert L.adfl_qerror_ref_plan(sizes.ctypes.data, len(sizes), 0, None, 0) < 0
