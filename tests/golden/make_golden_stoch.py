"""Golden vectors for the stochastic codecs (QSGD / RQSGD / CNAT), made by EXECUTING the reference.

Run in the build container (the reference tree exists only there):

    python tests/golden/make_golden_stoch.py

Each case runs the reference channel in place (``Src/ADFL/Channel/quant.py:140-570`` loaded by
``ref_loader``; torch 2.10.0+rocm7.0) with ``torch.rand_like`` replaced, for the duration of the call,
by a function returning recorded uniforms. The recorded uniforms go into the fixture with the input and
everything the reference produced: the level / exponent bytes, the signs, the norm (and RQSGD's minimum
factor) and the decoded floats. With those uniforms the oracle and the HIP codec must reproduce every
byte and every decoded bit; the L2 norm is compared within torch's fp32 accumulation error.

Outputs (data only):
  tests/golden/stoch.npz             arrays per case: x, u, q, signs, deq
  tests/golden/stoch_manifest.json   per case: codec, bits, shape, q dtype, scale / scale_2 (fp32 bits or
                                     a 0-dim-tensor marker), size, to_json, simulate_bandwidth bytes
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


def f32_bits(v) -> int:
    return int(np.array([float(v)], dtype=np.float32).view(np.uint32)[0])


def scale_record(v):
    """The reference stores norm.item() (a Python float holding an fp32 value), the 0-dim tensor itself on
    the norm == 0 branch (quant.py:228,369,514), or the int 0 for RQSGD's untouched scale_2."""
    if isinstance(v, torch.Tensor):
        assert v.ndim == 0 and v.dtype == torch.float32
        return {"tensor": True, "bits": f32_bits(v.item())}
    if isinstance(v, int):
        return {"int": v}
    s32 = np.float32(v)
    assert (np.isnan(v) and np.isnan(s32)) or float(s32) == float(v), v
    return {"bits": f32_bits(v)}


def run_case(ref, codec: str, bits: int, x: np.ndarray, u: np.ndarray):
    ch = getattr(ref.quant, CODECS[codec])(bits)
    t = torch.from_numpy(x.copy())
    ut = torch.from_numpy(u.copy())
    calls = []
    orig = torch.rand_like

    def fake_rand_like(p, *a, **k):
        assert p.shape == ut.shape and p.dtype == torch.float32
        calls.append(1)
        return ut.clone()

    torch.rand_like = fake_rand_like
    try:
        qp, _ = ch.on_client_send({"w": t})
    finally:
        torch.rand_like = orig
    dec, _ = ch.on_server_receive(qp)
    return ch, qp, dec, len(calls)


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    arrays, cases = {}, []

    def add(name, codec, bits, x, u_seed):
        x = np.ascontiguousarray(x, dtype=np.float32)
        u = np.random.default_rng(u_seed).random(x.size, dtype=np.float32).reshape(x.shape)
        ch, qp, dec, ncalls = run_case(ref, codec, bits, x, u)
        p = qp.params["w"]
        q = p.data.numpy()
        arrays[f"{name}__x"] = x
        arrays[f"{name}__u"] = u
        arrays[f"{name}__q"] = q.view(np.uint8)
        arrays[f"{name}__signs"] = p.signs.numpy()
        arrays[f"{name}__deq"] = dec["w"].numpy()
        cases.append({"name": name, "codec": codec, "bits": bits, "shape": list(x.shape),
                      "q_dtype": str(p.data.dtype).replace("torch.", ""), "scale": scale_record(p.scale),
                      "scale_2": scale_record(p.scale_2), "size": qp.size, "rand_calls": ncalls,
                      "levels": getattr(ch, "levels", None)})

    k = 0
    # A. random cases
    for shape in [(2, 5), (1, 17), (3, 7, 5), (33, 31), (128, 129), (40, 1023)]:
        for codec, bit_set in [("qsgd", (8, 4, 2)), ("rqsgd", (8, 4, 2)), ("cnat", (8, 4, 3))]:
            for bits in bit_set:
                add(f"{codec}_randn_{'x'.join(map(str, shape))}_b{bits}", codec, bits,
                    recipes.randn(shape, 10 + k, 1e-3), 1000 + k)
                k += 1
    for codec in CODECS:
        add(f"{codec}_heavy_64x257_b8", codec, 8, recipes.heavy_tail((64, 257), 7, 1e-3), 2000 + k)
        k += 1
        add(f"{codec}_unit_40x50_b8", codec, 8, recipes.randn((40, 50), 8, 1.0), 2000 + k)
        k += 1
        # bits past a byte: levels / exponents wrap through the u8 / i8 conversion
        add(f"{codec}_randn_9x11_b9", codec, 9, recipes.randn((9, 11), 9, 1e-3), 2000 + k)
        k += 1

    # B. edge cases
    nan, inf = np.float32(np.nan), np.float32(np.inf)
    edges = {
        "zeros": np.zeros((4, 4), np.float32),
        "negzero": np.array([[0.0, -0.0, 1e-3, -2e-3]], np.float32),
        "nan": np.array([[nan, 1.0, -2.0, 0.0]], np.float32),
        "posinf": np.array([[inf, 1.0, -2.0, 0.0]], np.float32),
        "neginf": np.array([[-inf, 1.0, 0.5, 0.0]], np.float32),
        "denormal": np.array([[1e-40, -1e-40, 1e-3, 0.0, 3e-45]], np.float32),
        "tiny_only": np.full((3, 3), 1e-30, np.float32),        # fp32 squares underflow: norm 0
        "huge": np.array([[1e30, -1e30, 1.0, 2.0]], np.float32),  # fp32 squares overflow: norm inf
        "sum_overflow": np.full((2, 8), 1e19, np.float32),       # squares finite, their fp32 sum is not
        "single": np.array([[0.0, 0.0, 3.0, 0.0]], np.float32),
        "const06": np.full((100, 100), 0.6, np.float32),         # Src/ADFL/Channel/Tests/test_quant.py:117-123
        "big_exp": np.array([[3e38, -1e38, 1e37, 2.5e-38]], np.float32),
    }
    # CNAT decision boundaries: |x| + eps within a few ulps of powers of two, across many binades
    near = []
    for kk in (-22, -20, -12, -10, -7, -3, -1, 0, 1, 4, 9, 20):
        p = np.float32(2.0 ** kk)
        base = np.float32(p - np.float32(2.0 ** -23)) if kk > -23 else p
        b = np.array([base], np.float32).view(np.uint32)[0]
        near.append((np.arange(int(b) - 24, int(b) + 24, dtype=np.uint32)).view(np.float32))
    near = np.concatenate(near)
    edges["near_pow2"] = np.stack([near, -near]).astype(np.float32)
    for ename, x in edges.items():
        for codec in CODECS:
            for bits in (8, 4):
                add(f"{codec}_edge_{ename}_b{bits}", codec, bits, x, 3000 + k)
                k += 1
    # uniforms at the extremes: 0 and the largest fp32 below 1
    for codec in CODECS:
        x = recipes.randn((16, 16), 55, 1e-3)
        for uname, uval in [("u0", 0.0), ("u1", np.nextafter(np.float32(1), np.float32(0)))]:
            name = f"{codec}_uconst_{uname}_b8"
            ch, qp, dec, ncalls = run_case(ref, codec, 8, x, np.full(x.shape, uval, np.float32))
            p = qp.params["w"]
            arrays[f"{name}__x"] = x
            arrays[f"{name}__u"] = np.full(x.shape, uval, np.float32)
            arrays[f"{name}__q"] = p.data.numpy().view(np.uint8)
            arrays[f"{name}__signs"] = p.signs.numpy()
            arrays[f"{name}__deq"] = dec["w"].numpy()
            cases.append({"name": name, "codec": codec, "bits": 8, "shape": list(x.shape),
                          "q_dtype": str(p.data.dtype).replace("torch.", ""), "scale": scale_record(p.scale),
                          "scale_2": scale_record(p.scale_2), "size": qp.size, "rand_calls": ncalls,
                          "levels": getattr(ch, "levels", None)})

    # C. channel-level facts: to_json, simulate_bandwidth bytes, passthrough of ndim <= 1
    facts = {"to_json": {}, "bandwidth": {}, "passthrough": {}}
    params = {"non_bias": torch.ones(2, 5), "bias": torch.ones(10)}
    for codec, cls in CODECS.items():
        for prefix in ("", "U"):
            name = prefix + cls
            facts["to_json"][name] = getattr(ref.quant, name)(8).to_json()
        ch = getattr(ref.quant, cls)(8)
        import time as _t
        orig_sleep = _t.sleep
        _t.sleep = lambda s: None
        try:
            facts["bandwidth"][cls] = ch.simulate_bandwidth(params, 1.0)  # seconds at 1 Mbps = bits / 1e6
        finally:
            _t.sleep = orig_sleep
        qp, _ = ch.on_client_send({"b": torch.arange(5, dtype=torch.float32), "n": torch.tensor(3)})
        pb, pn = qp.params["b"], qp.params["n"]
        facts["passthrough"][cls] = {"scale": pb.scale, "scale_2": pb.scale_2, "signs_dtype": str(pb.signs.dtype),
                                     "signs_numel": pb.signs.numel(), "size": qp.size,
                                     "n_dtype": str(pn.q_dtype)}

    np.savez_compressed(os.path.join(HERE, "stoch.npz"), **arrays)
    with open(os.path.join(HERE, "stoch_manifest.json"), "w") as f:
        json.dump({"torch": torch.__version__, "generator": "tests/golden/make_golden_stoch.py",
                   "cases": cases, **facts}, f, indent=1)
    print(f"{len(cases)} cases, {sum(a.nbytes for a in arrays.values()) / 1e6:.1f} MB raw")


if __name__ == "__main__":
    main()
