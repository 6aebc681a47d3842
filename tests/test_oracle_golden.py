"""CPU: pin both oracle restatements (C and numpy) to the reference's golden vectors.

The vectors were produced by executing Src/ADFL/Channel/quant.py in place (tests/golden/make_golden.py).
"""

import numpy as np
import pytest

import recipes
import slq_oracle as oracle
from golden_util import int4, manifest, same_f32, same_scale, small, small_cases

CASES = small_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_oracle_small_cases(case, impl):
    A = small()
    x, q_ref, d_ref = A[case["name"] + "__x"], A[case["name"] + "__q"], A[case["name"] + "__deq"]
    enc, dec = (oracle.encode, oracle.decode) if impl == "c" else (oracle.np_encode, oracle.np_decode)
    q, s = enc(x, case["bits"])
    assert np.array_equal(q, q_ref)
    assert same_scale(s, case["scale_bits"])
    assert same_f32(dec(q, s), d_ref)


RECIPES = manifest()["recipe"]


@pytest.mark.parametrize("case", RECIPES, ids=[f"{c['recipe']['kind']}{c['recipe']['shape']}_b{c['bits']}"
                                             for c in RECIPES])
def test_oracle_recipe_cases(case):
    x = recipes.make(case["recipe"])
    q, s = oracle.encode(x, case["bits"])
    assert same_scale(s, case["scale_bits"])
    assert recipes.sha256(q) == case["q_sha256"]
    assert recipes.sha256(oracle.decode(q, s)) == case["deq_sha256"]


@pytest.mark.parametrize("case", manifest()["bucket"], ids=lambda c: c["layout"])
def test_oracle_bucket_c3(case):
    tensors = recipes.bucket_tensors(case["layout"], case["seed"], case["mult"])
    assert [v.size for v in tensors.values()] == case["sizes"]
    sizes = np.array(case["sizes"], np.int64)
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    flat = np.concatenate([v.reshape(-1) for v in tensors.values()])
    q, scales = oracle.encode_batched(flat, offsets, sizes, case["bits"])
    for s, b in zip(scales, case["scale_bits"]):
        assert same_scale(s, b)
    assert recipes.sha256(q) == case["q_sha256"]
    d = np.concatenate([oracle.decode(q[o:o + n], s) for o, n, s in zip(offsets, sizes, scales)])
    assert recipes.sha256(d) == case["deq_sha256"]


@pytest.mark.parametrize("case", manifest()["int4"], ids=lambda c: c["name"])
def test_oracle_int4_layout(case):
    I = int4()
    q = I[f"int4_{case['name']}__q"]
    packed = I[f"int4_{case['name']}__packed"].view(np.uint8)
    unpacked = I[f"int4_{case['name']}__unpacked"].reshape(-1)
    assert np.array_equal(oracle.pack_int4(q), packed)
    assert np.array_equal(oracle.np_pack_int4(q), packed)
    assert np.array_equal(oracle.unpack_int4(packed, q.size), unpacked)
    assert np.array_equal(oracle.np_unpack_int4(packed, q.size), unpacked)


def test_oracle_int4_decode_is_unpack_then_dequantize():
    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 64, 1001):
        x = rng.standard_normal(n, dtype=np.float32)
        q, s = oracle.encode(x, 4)
        packed = oracle.pack_int4(q)
        assert same_f32(oracle.decode_int4(packed, n, s), oracle.decode(oracle.unpack_int4(packed, n), s))


def test_oracle_mean_matches_torch_stack_mean():
    """Examples/ray_ad.py:188: torch.stack(updates).mean(0) on the decoded payloads. Bit-exact on the
    vectorised body; torch's own scalar tail may round differently (<= 1 ulp)."""
    import torch
    rng = np.random.default_rng(4)
    for k in (2, 3, 8):
        n = 4096 * 3
        qs = [rng.integers(-128, 128, n, dtype=np.int8) for _ in range(k)]
        scales = (rng.random(k, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
        got = oracle.dequantize_mean(qs, scales)
        ref = torch.stack([torch.from_numpy(oracle.decode(q, s)) for q, s in zip(qs, scales)]).mean(0).numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
