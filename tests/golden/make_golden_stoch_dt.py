"""Golden vectors for the stochastic codecs on fp16 / bf16 / fp64 tensors, made by EXECUTING the reference.

Run in the build container (the reference tree exists only there):

    python tests/golden/make_golden_stoch_dt.py

Each case runs the reference channel in place (``Src/ADFL/Channel/quant.py:140-570`` loaded by
``ref_loader``; torch 2.10.0+rocm7.0) on a tensor of the case's dtype, with ``torch.rand_like`` replaced
for the duration of the call by recorded uniforms of that dtype (torch's own grid: k * 2^-11 for fp16,
k * 2^-8 for bf16, k * 2^-53 for fp64). Stored: the input and the uniforms (raw bits: uint16 for fp16 /
bf16, float64), the level / exponent bytes, the signs, the decoded fp32 floats, and the scale / scale_2
the reference put in the payload (fp64 bits of the Python float, or a marker for the 0-dim tensor of the
norm == 0 branch).

Outputs (data only):
  tests/golden/stoch_dt.npz            arrays per case: x, u, q, signs, deq
  tests/golden/stoch_dt_manifest.json  per case: codec, dtype, bits, shape, q dtype, scale, scale_2, size
"""

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import recipes  # noqa: E402
from ref_loader import load_reference  # noqa: E402

CODECS = {"qsgd": "QSGDChannel", "rqsgd": "RQSGDChannel", "cnat": "CNATChannel"}
DTYPES = {"float16": torch.float16, "bfloat16": torch.bfloat16, "float64": torch.float64}
GRID = {"float16": 11, "bfloat16": 8, "float64": 53}


def raw(t: torch.Tensor) -> np.ndarray:
    """Stored bits of a tensor: uint16 for fp16 / bf16, float64 for fp64."""
    if t.dtype == torch.float64:
        return t.numpy().copy()
    return t.view(torch.int16).numpy().view(np.uint16).copy()


def scale_record(v):
    if isinstance(v, torch.Tensor):
        assert v.ndim == 0
        return {"tensor": True, "dtype": str(v.dtype).replace("torch.", ""), "value": float(v.item())}
    if isinstance(v, int):
        return {"int": v}
    return {"f64_bits": int(np.array([float(v)], np.float64).view(np.uint64)[0])}


def uniforms(dtname: str, shape, seed: int) -> torch.Tensor:
    g = GRID[dtname]
    rng = np.random.default_rng(seed)
    if g == 53:
        k = rng.integers(0, 2 ** 53, size=shape, dtype=np.int64)
        return torch.from_numpy(k.astype(np.float64) * 2.0 ** -53)
    k = rng.integers(0, 2 ** g, size=shape, dtype=np.int64)
    return torch.from_numpy((k.astype(np.float32) * np.float32(2.0 ** -g))).to(DTYPES[dtname])


def run_case(ref, codec: str, bits: int, x: torch.Tensor, u: torch.Tensor):
    ch = getattr(ref.quant, CODECS[codec])(bits)
    calls = []
    orig = torch.rand_like

    def fake_rand_like(p, *a, **k):
        assert p.shape == u.shape and p.dtype == u.dtype, (p.shape, p.dtype, u.dtype)
        calls.append(1)
        return u.clone()

    torch.rand_like = fake_rand_like
    try:
        qp, _ = ch.on_client_send({"w": x.clone()})
    finally:
        torch.rand_like = orig
    dec, _ = ch.on_server_receive(qp)
    return ch, qp, dec, len(calls)


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    arrays, cases = {}, []

    def add(name, codec, bits, dtname, x: torch.Tensor, u: torch.Tensor):
        ch, qp, dec, ncalls = run_case(ref, codec, bits, x, u)
        p = qp.params["w"]
        arrays[f"{name}__x"] = raw(x)
        arrays[f"{name}__u"] = raw(u)
        arrays[f"{name}__q"] = p.data.numpy().view(np.uint8).copy()
        arrays[f"{name}__signs"] = p.signs.numpy().copy()
        arrays[f"{name}__deq"] = dec["w"].numpy().copy()
        assert dec["w"].dtype == torch.float32
        cases.append({"name": name, "codec": codec, "dtype": dtname, "bits": bits, "shape": list(x.shape),
                      "q_dtype": str(p.data.dtype).replace("torch.", ""), "scale": scale_record(p.scale),
                      "scale_2": scale_record(p.scale_2), "size": qp.size, "rand_calls": ncalls})

    k = 0
    for dtname, dt in DTYPES.items():
        # A. random cases
        for shape, scale in [((2, 5), 1e-2), ((33, 31), 1e-3), ((40, 123), 1.0), ((7, 300), 30.0)]:
            for codec, bit_set in [("qsgd", (8, 4, 2)), ("rqsgd", (8, 4)), ("cnat", (8, 4, 3))]:
                for bits in bit_set:
                    x = torch.from_numpy(recipes.randn(shape, 40 + k, scale)).to(dt)
                    add(f"{dtname}_{codec}_randn_{'x'.join(map(str, shape))}_b{bits}", codec, bits, dtname, x,
                        uniforms(dtname, shape, 5000 + k))
                    k += 1
        for codec in CODECS:   # bits past a byte: levels / exponents wrap through the u8 / i8 conversion
            x = torch.from_numpy(recipes.randn((9, 11), 9, 1e-2)).to(dt)
            add(f"{dtname}_{codec}_randn_9x11_b9", codec, 9, dtname, x, uniforms(dtname, (9, 11), 6000 + k))
            k += 1
        # B. edge cases in the dtype
        fi = torch.finfo(dt)
        tiny = fi.tiny
        nan, inf = float("nan"), float("inf")
        edges = {
            "zeros": torch.zeros(4, 4, dtype=dt),
            "negzero": torch.tensor([[0.0, -0.0, 1e-2, -2e-2]], dtype=dt),
            "nan": torch.tensor([[nan, 1.0, -2.0, 0.0]], dtype=dt),
            "posinf": torch.tensor([[inf, 1.0, -2.0, 0.0]], dtype=dt),
            "neginf": torch.tensor([[-inf, 1.0, 0.5, 0.0]], dtype=dt),
            "denormal": torch.tensor([[tiny / 4, -tiny / 8, 1e-2, 0.0, tiny]], dtype=dt),
            "huge": torch.tensor([[fi.max, -fi.max / 2, 1.0, 2.0]], dtype=dt),
            "const06": torch.full((50, 40), 0.6, dtype=dt),   # Src/ADFL/Channel/Tests/test_quant.py:117-123
        }
        # CNAT decision boundaries: |x| + eps within a few ulps of powers of two
        eps = fi.eps
        near = []
        for kk in (-6, -3, -1, 0, 1, 3, 7, 12):
            p = torch.tensor([2.0 ** kk - eps], dtype=torch.float64).to(dt)
            if dt == torch.float64:
                b = p.view(torch.int64)
                near.append((b + torch.arange(-24, 24)).view(torch.float64))
            else:
                b = p.view(torch.int16).to(torch.int32)
                near.append((b + torch.arange(-12, 12, dtype=torch.int32)).to(torch.int16).view(dt))
        near = torch.cat(near)
        edges["near_pow2"] = torch.stack([near, -near])
        for ename, x in edges.items():
            for codec in CODECS:
                for bits in (8, 4):
                    add(f"{dtname}_{codec}_edge_{ename}_b{bits}", codec, bits, dtname, x,
                        uniforms(dtname, tuple(x.shape), 7000 + k))
                    k += 1
        # uniforms at the extremes of the dtype's grid: 0 and 1 - 2^-g
        for codec in CODECS:
            x = torch.from_numpy(recipes.randn((16, 16), 55, 1e-2)).to(dt)
            for uname, uval in [("u0", 0.0), ("u1", 1.0 - 2.0 ** -GRID[dtname])]:
                add(f"{dtname}_{codec}_uconst_{uname}_b8", codec, 8, dtname, x, torch.full(x.shape, uval, dtype=dt))

    np.savez_compressed(os.path.join(HERE, "stoch_dt.npz"), **arrays)
    with open(os.path.join(HERE, "stoch_dt_manifest.json"), "w") as f:
        json.dump({"torch": torch.__version__, "generator": "tests/golden/make_golden_stoch_dt.py",
                   "cases": cases}, f, indent=1)
    print(f"{len(cases)} cases, {sum(a.nbytes for a in arrays.values()) / 1e6:.1f} MB raw")


if __name__ == "__main__":
    main()
