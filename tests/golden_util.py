"""Shared helpers: golden fixture access and NaN-aware bit comparisons."""

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_cache = {}


def manifest() -> dict:
    if "m" not in _cache:
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            _cache["m"] = json.load(f)
    return _cache["m"]


def small() -> "np.lib.npyio.NpzFile":
    if "s" not in _cache:
        _cache["s"] = np.load(os.path.join(GOLDEN, "slq_small.npz"))
    return _cache["s"]


def int4() -> "np.lib.npyio.NpzFile":
    if "i" not in _cache:
        _cache["i"] = np.load(os.path.join(GOLDEN, "int4.npz"))
    return _cache["i"]


def small_cases(groups=("raw", "edge")):
    m = manifest()
    return [c for g in groups for c in m[g]]


def f32_from_bits(b: int) -> np.float32:
    return np.array([b], dtype=np.uint32).view(np.float32)[0]


def bits_of(v) -> int:
    return int(np.array([v], dtype=np.float32).view(np.uint32)[0])


def same_f32(a, b) -> bool:
    """Bit-identical fp32 arrays, except that NaN payload bits are not compared (positions are)."""
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1)
    b = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def same_scale(v, golden_bits: int) -> bool:
    return same_f32(np.float32(v), f32_from_bits(golden_bits))
