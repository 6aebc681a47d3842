"""CPU: torch's summation order for the aggregate step, restated in the oracle, against torch itself and
against the reference executed in place (tests/golden/aggregate.npz, make_golden_aggregate.py).

* oracle.torch_sum_rows / torch_mean_rows (slq_oracle.c oracle_torch_sum_col) equal torch 2.10's CPU
  ``torch.sum(torch.stack(rows), dim=0)`` and ``stack(rows).mean(0)`` bit for bit over K = 1 .. 4100 rows
  and tensor sizes 1 .. 40001 (every branch: SEQ cascade, ILP4 tails, n < 8, n == 1) — single- and
  multi-threaded (the column split is at 32-column multiples, so the order does not depend on threads);
* the oracle's decode + mean of the reference's SLQ payloads equals the reference's simple_aggregate
  (Src/ADFL/model.py:221-234) for K = 1 .. 64 (bits 8) and 3 .. 20 (bits 4), and the peer mean
  stack([received..., own]).mean(0) (Examples/ray_ad.py:183-188) with the receiver's update exact;
* the oracle's decodes of the reference's own QSGD / RQSGD / CNAT payloads, averaged in torch's order,
  equal simple_aggregate of the reference's decodes at K = 5, 8, 16, 20;
* the q-error metrics (torch.sum to a scalar, cosine_similarity) are pinned in tests/test_qerror_order.py."""

import json
import os

import numpy as np
import pytest
import torch

import slq_oracle as oracle
import stoch_oracle as so
from golden_util import same_f32
from make_golden_aggregate import BIASES, SHAPES, client_arrays

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_cache = {}


def fixture():
    if "a" not in _cache:
        _cache["a"] = np.load(os.path.join(GOLDEN, "aggregate.npz"))
        with open(os.path.join(GOLDEN, "aggregate_manifest.json")) as f:
            _cache["m"] = json.load(f)
    return _cache["a"], _cache["m"]


def _bits_f32(rec):
    return np.array([rec["bits"]], np.uint32).view(np.float32)[0]


@pytest.mark.parametrize("threads", [1, 8])
def test_restatement_equals_torch(threads):
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        rng = np.random.default_rng(11 + threads)
        for k in list(range(1, 41)) + [63, 64, 65, 100, 255, 256, 257, 300, 1000, 4100]:
            for n in [1, 2, 3, 5, 7, 8, 9, 15, 31, 32, 33, 40, 63, 64, 65, 100, 1000, 40001]:
                if k * n > 4_000_000:
                    continue
                x = (rng.standard_normal((k, n)) * np.exp(rng.uniform(-8, 8, (k, n)))).astype(np.float32)
                rows = [torch.from_numpy(x[i].copy()) for i in range(k)]
                assert same_f32(oracle.torch_sum_rows(x), torch.sum(torch.stack(rows), dim=0).numpy()), (k, n)
                assert same_f32(oracle.torch_mean_rows(x), torch.stack(rows).mean(0).numpy()), (k, n)
    finally:
        torch.set_num_threads(old)


def test_restatement_multidim_and_special_values():
    """Stacks of N-d tensors reduce like [K, numel]; -0 columns sum to +0, NaN / inf propagate."""
    rng = np.random.default_rng(3)
    for shape in [(16, 3, 3, 3), (7, 5), (2, 3), (1, 1), (3, 1), (64, 129)]:
        for k in (5, 17, 20, 64):
            x = rng.standard_normal((k,) + shape).astype(np.float32)
            x.reshape(k, -1)[:, 0] = -0.0
            x.reshape(k, -1)[1, -1] = np.inf
            x.reshape(k, -1)[2, 1 % x[0].size] = np.nan
            t = torch.sum(torch.stack([torch.from_numpy(x[i].copy()) for i in range(k)]), dim=0).numpy()
            assert same_f32(oracle.torch_sum_rows(x.reshape(k, -1)), t.reshape(-1)), (shape, k)
            assert np.signbit(oracle.torch_sum_rows(x.reshape(k, -1))[0]) == np.signbit(t.reshape(-1)[0])


def _slq_decoded(bits, c):
    xs = client_arrays(c)
    out = {}
    for n in SHAPES:
        q, s = oracle.encode(xs[n], bits)
        out[n] = (q, s, oracle.decode(q, s))
    return xs, out


def test_fixture_inputs_are_the_recipe():
    _, m = fixture()
    for c, shas in enumerate(m["clients"]):
        xs = client_arrays(c)
        for n, h in shas.items():
            import recipes
            assert recipes.sha256(xs[n]) == h, (c, n)


@pytest.mark.parametrize("bits", [8, 4])
def test_oracle_mean_is_reference_simple_aggregate(bits):
    a, m = fixture()
    ks = m["k_slq"] if bits == 8 else m["k_slq4"]
    dec = [_slq_decoded(bits, c) for c in range(max(ks))]
    for k in ks:
        for n, shape in SHAPES.items():
            want = a[f"slq{bits}__k{k}__{n}"]
            qs = [dec[c][1][n][0] for c in range(k)]
            ss = [dec[c][1][n][1] for c in range(k)]
            # SLQChannel(4) keeps int8 codes (quant.py:102-103): the int8 mean at both widths
            assert same_f32(oracle.dequantize_mean(qs, ss), want), (k, n)
            # the same through the generic restatement on the decoded rows
            assert same_f32(oracle.torch_mean_rows([dec[c][1][n][2] for c in range(k)]), want), (k, n)
        for n in BIASES:  # passthrough entries: simple_aggregate of the raw tensors
            assert same_f32(oracle.torch_mean_rows([dec[c][0][n] for c in range(k)]), a[f"slq{bits}__k{k}__{n}"])


@pytest.mark.parametrize("bits", [8, 4])
def test_oracle_peer_mean_is_reference_expression(bits):
    a, m = fixture()
    dec = [_slq_decoded(bits, c) for c in range(max(m["k_peer"]))]
    for k in m["k_peer"]:
        me = k // 2
        for n, shape in SHAPES.items():
            rows = [dec[c][1][n][0] for c in range(k)]
            got = oracle.dequantize_mean_self(rows, [dec[c][1][n][1] for c in range(k)], int(np.prod(shape)), me,
                                              dec[me][0][n])
            assert same_f32(got, a[f"peer{bits}__k{k}__{n}"]), (k, n)


def stoch_decode(codec, bits, q, signs, scale, scale_2):
    levels = 2 ** bits - 1
    if codec == "qsgd":
        return so.qsgd_dequantize(q, signs, levels, scale)
    if codec == "rqsgd":
        return so.rqsgd_dequantize(q, signs, levels, scale, scale_2)
    return so.cnat_dequantize(q.view(np.int8), signs, scale)


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_stochastic_mean_of_reference_payloads(codec):
    a, m = fixture()
    bits = m["stoch"][codec][1]
    dec = []
    for c in range(max(m["k_stoch"])):
        d = {}
        for n, shape in SHAPES.items():
            rec = m["stoch_scales"][f"{codec}__c{c}__{n}"]
            scale = _bits_f32(rec["scale"])
            s2 = _bits_f32(rec["scale_2"]) if "bits" in rec["scale_2"] else np.float32(rec["scale_2"]["int"])
            q = a[f"{codec}__c{c}__{n}__q"]
            if scale == 0:
                d[n] = np.zeros(q.shape, np.float32)   # quant.py:246-247: zeros for a zero norm
            else:
                d[n] = stoch_decode(codec, bits, q, a[f"{codec}__c{c}__{n}__signs"], scale, s2)
        dec.append(d)
    for k in m["k_stoch"]:
        for n in SHAPES:
            assert same_f32(oracle.torch_mean_rows([dec[c][n] for c in range(k)]), a[f"{codec}__k{k}__{n}"]), (k, n)


def test_host_sum_rows_equals_torch_per_entry():
    """adfl_amd.sum_order.sum_rows (receive_mean's host aggregation of passthrough entries, all entries of a
    dict in one pass) equals each entry's own torch.sum(torch.stack(...), 0), and its self-check passes."""
    from adfl_amd import sum_order
    assert sum_order.self_check()
    g = torch.Generator().manual_seed(9)
    sizes = [2, 3, 5, 6, 7, 8, 9, 31, 32, 33, 64, 100, 1000, 4097]
    for k in (1, 2, 4, 5, 8, 15, 16, 17, 20, 33, 64, 65, 256, 300):
        ents = [torch.randn(k, n, generator=g) * torch.exp(torch.randn(k, n, generator=g) * 4) for n in sizes]
        ents[3][0, 1] = float("nan")
        ents[5][:, 0] = -0.0
        got = sum_order.sum_rows(torch.cat(ents, dim=1), sizes)
        want = torch.cat([torch.sum(torch.stack(list(e.unbind(0))), dim=0) for e in ents])
        assert same_f32(got.numpy(), want.numpy()), k
        assert np.array_equal(np.signbit(got.numpy()), np.signbit(want.numpy())), k
