"""Deterministic input recipes shared by the golden generator and the parity tests.

Inputs are built with numpy's PCG64 ``default_rng`` (integer-exact and table-driven, identical on
every host running this image), so a fixture may store a recipe plus SHA-256 digests instead of raw
bytes for the large cases.
"""

import hashlib
import math

import numpy as np

RESNET18_PARAMS = 11_689_512


def randn(shape, seed: int, mult: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(size=n, dtype=np.float32) * np.float32(mult)
    return x.reshape(shape)


def heavy_tail(shape, seed: int, mult: float) -> np.ndarray:
    """``randn`` with 0.1 % of the elements scaled ×100 (saturation variant)."""
    x = randn(shape, seed, mult).reshape(-1)
    rng = np.random.default_rng(seed + 1_000_003)
    k = max(1, x.size // 1000)
    idx = rng.choice(x.size, size=k, replace=False)
    x[idx] *= np.float32(100.0)
    return x.reshape(shape)


def make(recipe: dict) -> np.ndarray:
    kind = recipe["kind"]
    shape = tuple(recipe["shape"])
    if kind == "randn":
        return randn(shape, recipe["seed"], recipe["mult"])
    if kind == "heavy_tail":
        return heavy_tail(shape, recipe["seed"], recipe["mult"])
    raise ValueError(f"unknown recipe kind {kind}")


def bucket_sizes(layout: str, seed: int = 0, total: int = RESNET18_PARAMS, count: int = 256):
    """Per-tensor element counts of the C3 bucketed update: 256 tensors, Σ = 11,689,512."""
    if layout == "equal":
        base, rem = divmod(total, count)
        return [base + (1 if i < rem else 0) for i in range(count)]
    if layout == "loguniform":
        rng = np.random.default_rng(seed)
        raw = np.exp(rng.uniform(math.log(64), math.log(2_400_000), size=count))
        sizes = np.maximum(64, np.floor(raw / raw.sum() * total)).astype(np.int64)
        sizes[int(np.argmax(sizes))] += total - int(sizes.sum())
        return [int(s) for s in sizes]
    raise ValueError(layout)


def bucket_tensors(layout: str, seed: int, mult: float):
    """The C3 tensors as a name -> 2-D float32 array dict (each tensor its own seeded stream)."""
    out = {}
    for i, n in enumerate(bucket_sizes(layout, seed)):
        out[f"layer{i:03d}.weight"] = randn((1, n), seed * 100_003 + i, mult)
    return out


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()
