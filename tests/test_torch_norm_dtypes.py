"""CPU: the reference-order L2 norm restatements for fp16 / bf16 / fp64 (oracle/slq_oracle.c
oracle_torch_l2_norm_{f16,bf16,f64}, wrapped by stoch_dt_oracle.torch_l2_norm) pinned two ways:

* to the reference's own norms: every QSGD / CNAT case of tests/golden/stoch_dt.npz (the reference channels
  executed in place, Src/ADFL/Channel/quant.py:226,512, on fp16 / bf16 / fp64 tensors) — bit for bit;
* to torch.linalg.vector_norm itself, run here, on data that exercises the orders: the n % 16 (bf16) and
  n % 4 (fp64) tails, fp16's at::parallel_for split around 32768 elements at 1 / 2 / 3 / 5 / 8 threads,
  ties, subnormal / overflowing squares, NaN and inf.

The GPU kernels (csrc/torch_norm.hip) are compared with torch.linalg.vector_norm directly on the GPU box
(tests/test_gpu_torch_norm_dt.py).
"""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

import stoch_dt_oracle as do
import stoch_oracle as so

DT = {"float16": do.DT_F16, "bfloat16": do.DT_BF16, "float64": do.DT_F64}
MANIFEST = json.load(open(os.path.join(GOLDEN, "stoch_dt_manifest.json")))
ARR = np.load(os.path.join(GOLDEN, "stoch_dt.npz"))
L2_CASES = [c for c in MANIFEST["cases"] if c["codec"] in ("qsgd", "cnat")]


def _same(a: float, b: float) -> bool:
    return (np.isnan(a) and np.isnan(b)) or np.float64(a).view(np.uint64) == np.float64(b).view(np.uint64)


def _scale(rec) -> float:
    if "int" in rec:
        return float(rec["int"])
    if rec.get("tensor"):
        return float(rec["value"])
    return float(np.array([rec["f64_bits"]], np.uint64).view(np.float64)[0])


@pytest.mark.parametrize("c", L2_CASES, ids=[c["name"] for c in L2_CASES])
def test_restatement_equals_reference_norm(c):
    """The norm the reference computed (its QuantParameter.scale) equals the restatement bit for bit."""
    x = ARR[f"{c['name']}__x"]
    want = _scale(c["scale"])
    got = do.torch_l2_norm(x, DT[c["dtype"]], threads=8)
    assert _same(got, want), (c["name"], got, want)


def _torch_tensor(raw: np.ndarray, dt) -> torch.Tensor:
    if dt == do.DT_F64:
        return torch.from_numpy(raw.astype(np.float64))
    t = torch.from_numpy(raw.view(np.int16).copy())
    return t.view(torch.float16 if dt == do.DT_F16 else torch.bfloat16)


def _make(kind, n, rng, dt) -> np.ndarray:
    if kind == "randn":
        x = rng.standard_normal(n) * 1e-3
    elif kind == "ties":
        x = np.round(rng.standard_normal(n) * 16) / 64
    elif kind == "wide":
        x = rng.standard_normal(n) * np.exp2(rng.integers(-7 if dt == do.DT_F16 else -60,
                                                          7 if dt == do.DT_F16 else 60, n))
    elif kind == "special":
        x = rng.standard_normal(n)
        x[rng.integers(0, n)] = np.inf
        if n > 5:
            x[rng.integers(0, n)] = np.nan
    else:
        raise ValueError(kind)
    t = torch.from_numpy(x)
    if dt == do.DT_F64:
        return t.numpy()
    return t.to(torch.float16 if dt == do.DT_F16 else torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


@pytest.mark.parametrize("kind", ["randn", "ties", "wide", "special"])
@pytest.mark.parametrize("dtn", list(DT))
def test_restatement_equals_torch(dtn, kind):
    dt = DT[dtn]
    rng = np.random.default_rng(list(DT).index(dtn) * 10 + ["randn", "ties", "wide", "special"].index(kind))
    sizes = [1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 33, 1000, 4097, 32767, 32768, 32769, 65537, 100003]
    old = torch.get_num_threads()
    try:
        for threads in (1, 2, 3, 5, 8):
            torch.set_num_threads(threads)
            for n in sizes:
                raw = _make(kind, n, rng, dt)
                want = torch.linalg.vector_norm(_torch_tensor(raw, dt)).item()
                got = do.torch_l2_norm(raw, dt, threads)
                assert _same(got, want), (dtn, kind, threads, n, got, want)
    finally:
        torch.set_num_threads(old)


def test_fp32_restatement_equals_torch_across_threads():
    """fp32's order does not depend on the thread count (one reduction per output); every tail length
    (n % 8: the group of 4 rounded squares, then fma) and the sizes below 8."""
    rng = np.random.default_rng(7)
    old = torch.get_num_threads()
    try:
        for threads in (1, 3, 8):
            torch.set_num_threads(threads)
            for n in list(range(1, 41)) * 6 + [100003, 1 << 18]:
                x = (rng.standard_normal(n) * 1e-3).astype(np.float32)
                want = torch.linalg.vector_norm(torch.from_numpy(x)).item()
                assert _same(float(so.torch_l2_norm(x)), want)
    finally:
        torch.set_num_threads(old)
