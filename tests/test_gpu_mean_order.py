"""GPU: the mean kernels in torch's summation order, bit for bit, at the client counts ADFL runs.

Every fused mean — the flat peer mean after the exchange (adfl_slq_dequantize_mean[_self][_int4];
Examples/ray_ad.py:183-188, BASELINE configs[3]/[4] with 8 clients), the bucketed mean of a whole state dict
(adfl_slq_dequantize_mean_batched[_int4]) and the stochastic channels' aggregate
(adfl_stoch_dequantize_mean_batched) — sums the K decoded rows in the order torch 2.10's CPU
``torch.sum(torch.stack(rows), dim=0)`` takes (csrc/torch_sum_order.h) and divides by K, so it equals
``simple_aggregate`` (Src/ADFL/model.py:221-234) and ``stack(...).mean(0)`` exactly. Checked here against
the oracle (oracle/slq_oracle.c oracle_torch_sum_col, pinned to torch and to the reference executed in place
by tests/test_sum_order_golden.py) AND against torch's own CPU mean of the oracle's decodes, over:

* K = 2 .. 64 and 257 / 300 (the cascade's deep levels: a separate kernel instantiation from K = 256);
* ragged n (1, 3, 6, 7, 33, 1000, 4097, 300007): SEQ tiles, the ILP4 tail columns, n < 8 and n == 1;
* a zero-scale row and a NaN-scale row; the receiver's own row exact at self_row 0, 3, 7 and K - 1;
* int8 and int4-packed rows (the C5 exchange's flat int4 mean at K = 8 included)."""

import numpy as np
import pytest
import torch

import slq_oracle as oracle
import stoch_oracle as so
from golden_util import same_f32

pytestmark = pytest.mark.gpu

adfl_amd = pytest.importorskip("adfl_amd")
from adfl_amd import ops  # noqa: E402

DEV = torch.device("cuda", 0)


def _rows(k, n, packed, special, seed):
    """K synthetic payload rows (int8 codes, or int4-packed bytes) and scales with one special row."""
    rng = np.random.default_rng(seed)
    nb = (n + 1) // 2 if packed else n
    row = (nb + 15) // 16 * 16
    raw = np.zeros((k, row), np.uint8)
    raw[:, :nb] = rng.integers(0, 256, size=(k, nb), dtype=np.uint8)
    scales = (rng.uniform(0.5, 2.0, k) * 10.0 ** rng.integers(-6, 1, k)).astype(np.float32)
    if special == "zero" and k >= 2:
        scales[1] = 0.0
    if special == "nan" and k >= 3:
        scales[2] = np.nan
    return raw, scales


def _decode(raw_row, scale, n, packed):
    if packed:
        return oracle.decode_int4(raw_row, n, scale)
    return oracle.decode(raw_row[:n].view(np.int8), scale)


CASES = [(k, n) for k in (2, 5, 8, 16, 17, 20, 33, 64) for n in (1, 3, 6, 7, 33, 1000, 4097, 300007)]
CASES += [(257, n) for n in (1, 7, 33, 4097)] + [(300, 70001)]


@pytest.mark.parametrize("packed", [False, True], ids=["int8", "int4"])
@pytest.mark.parametrize("k,n", CASES)
def test_flat_mean_torch_order(k, n, packed):
    for special in ("none", "zero", "nan"):
        raw, scales = _rows(k, n, packed, special, seed=k * 1000 + n)
        rows_d = torch.from_numpy(raw).to(DEV)
        q = rows_d if packed else rows_d.view(torch.int8)
        sc = torch.from_numpy(scales).to(DEV)
        got = ops.dequantize_mean(q, sc, n, packed=packed).cpu().numpy()
        rows = [raw[r] if packed else raw[r, :n].view(np.int8) for r in range(k)]
        if packed:
            want = oracle.dequantize_mean_int4(rows, scales, n)
        else:
            want = oracle.dequantize_mean(rows, scales)
        assert same_f32(got, want), (special, k, n)
        dec = [torch.from_numpy(_decode(raw[r], scales[r], n, packed)) for r in range(k)]
        assert same_f32(got, torch.stack(dec).mean(0).numpy()), (special, k, n)


@pytest.mark.parametrize("packed", [False, True], ids=["int8", "int4"])
@pytest.mark.parametrize("k,n", [(8, 1), (8, 7), (8, 33), (8, 4097), (8, 300007), (8, (1 << 20) + 5),
                                 (16, 1000), (20, 4097), (257, 33)])
def test_flat_mean_self_torch_order(k, n, packed):
    """The receiving peer's mean (own update exact, appended after the received rows): the C4 / C5 shape at
    K = 8 with self_row 0, 3, 7 (and K - 1 elsewhere), a zero-scale and a NaN-scale row."""
    rng = np.random.default_rng(n + k)
    selfs = (0, 3, 7) if k == 8 else (0, k - 1)
    for special in ("zero", "nan"):
        raw, scales = _rows(k, n, packed, special, seed=7 * n + k)
        q = torch.from_numpy(raw).to(DEV)
        q = q if packed else q.view(torch.int8)
        sc = torch.from_numpy(scales).to(DEV)
        for me in selfs:
            x = rng.standard_normal(n, dtype=np.float32) * np.float32(1e-3)
            x[0] = -0.0
            got = ops.dequantize_mean(q, sc, n, self_row=me, self_x=torch.from_numpy(x).to(DEV),
                                      packed=packed).cpu().numpy()
            rows = [raw[r] if packed else raw[r, :n].view(np.int8) for r in range(k)]
            want = oracle.dequantize_mean_self(rows, scales, n, me, x, packed=packed)
            assert same_f32(got, want), (special, me)
            dec = [torch.from_numpy(_decode(raw[r], scales[r], n, packed)) for r in range(k) if r != me]
            ref = torch.stack(dec + [torch.from_numpy(x)]).mean(0).numpy()   # ray_ad.py:188
            assert same_f32(got, ref), (special, me)


SIZES = [1, 2, 3, 6, 7, 9, 31, 33, 100, 8192, 8193, 16415, 70001]


@pytest.mark.parametrize("packed,align", [(False, 1), (False, 64), (True, 2), (True, 64)])
@pytest.mark.parametrize("k", [5, 8, 16, 20, 257])
def test_batched_mean_torch_order(k, packed, align):
    """A whole state dict per row (per-tensor scales): each tensor's columns in its own order (its SEQ tiles
    end below n & ~31 of THAT tensor, whatever the bucket offset), own row exact or not."""
    lay = ops.BucketLayout(SIZES, align=align)
    rng = np.random.default_rng(k + align)
    nb = (lay.total + 1) // 2 if packed else lay.total
    row = (nb + 15) // 16 * 16
    raw = rng.integers(0, 256, size=(k, row), dtype=np.uint8)
    scales = (rng.uniform(0.5, 2.0, (k, len(SIZES))) * 10.0 ** rng.integers(-5, 1, (k, len(SIZES)))).astype(np.float32)
    scales[1, 2] = 0.0
    scales[min(2, k - 1), 5] = np.nan
    q = torch.from_numpy(raw).to(DEV)
    q = q if packed else q.view(torch.int8)
    sc = torch.from_numpy(scales).to(DEV)
    x = rng.standard_normal(lay.total, dtype=np.float32) * np.float32(1e-2)
    for me in (-1, k // 2):
        kw = {} if me < 0 else {"self_row": me, "self_x": torch.from_numpy(x).to(DEV)}
        got = ops.dequantize_mean_batched(q, sc, lay, packed=packed, **kw).cpu().numpy()
        rows = [raw[r] for r in range(k)] if packed else [raw[r, :lay.total].view(np.int8) for r in range(k)]
        want = oracle.dequantize_mean_batched(rows, scales, lay.offsets, lay.sizes, lay.total, self_row=me,
                                              self_x=x if me >= 0 else None, packed=packed)
        assert same_f32(got, want), me
        for t, (o, n) in enumerate(zip(lay.offsets.tolist(), SIZES)):   # torch's own mean per tensor
            dec = []
            for r in range(k):
                if r == me:
                    continue
                if packed:
                    dec.append(oracle.decode_int4(raw[r], lay.total, scales[r, t])[o:o + n])
                else:
                    dec.append(oracle.decode(raw[r, o:o + n].view(np.int8), scales[r, t]))
            if me >= 0:
                dec.append(x[o:o + n])
            ref = torch.stack([torch.from_numpy(np.ascontiguousarray(d)) for d in dec]).mean(0).numpy()
            assert same_f32(got[o:o + n], ref), (me, t, n)


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
@pytest.mark.parametrize("k", [5, 8, 16, 20, 257])
def test_stoch_batched_mean_torch_order(codec, k):
    from adfl_amd import stoch as sops
    bits = 4 if codec == "rqsgd" else 8
    lay = ops.BucketLayout(SIZES, align=1)
    rng = np.random.default_rng(31 * k)
    row = (lay.total + 15) // 16 * 16
    lv = rng.integers(0, 2 ** bits if codec != "cnat" else 256, size=(k, row), dtype=np.uint8)
    if codec == "cnat":   # exponents in [-128, 127] as int8 bytes, clamped to the codec's range
        lv = np.clip(lv.view(np.int8), -2 ** (bits - 1), 2 ** (bits - 1) - 1).view(np.uint8)
    sg = rng.choice(np.array([-1, 0, 1], np.int8), size=(k, row))
    norms = (rng.uniform(0.5, 2.0, (k, len(SIZES))) * 10.0 ** rng.integers(-4, 1, (k, len(SIZES)))).astype(np.float32)
    norms[1, 3] = 0.0
    mins = (norms * rng.uniform(0.0, 0.5, norms.shape)).astype(np.float32)
    got = sops.dequantize_mean_batched(codec, torch.from_numpy(lv).to(DEV), torch.from_numpy(sg).to(DEV),
                                       torch.from_numpy(norms).to(DEV), lay, bits,
                                       mins=torch.from_numpy(mins).to(DEV) if codec == "rqsgd" else None).cpu().numpy()
    for t, (o, n) in enumerate(zip(lay.offsets.tolist(), SIZES)):
        dec = []
        for r in range(k):
            if norms[r, t] == 0:
                dec.append(np.zeros(n, np.float32))
            elif codec == "qsgd":
                dec.append(so.qsgd_dequantize(lv[r, o:o + n], sg[r, o:o + n], 2 ** bits - 1, norms[r, t]))
            elif codec == "rqsgd":
                dec.append(so.rqsgd_dequantize(lv[r, o:o + n], sg[r, o:o + n], 2 ** bits - 1, norms[r, t], mins[r, t]))
            else:
                dec.append(so.cnat_dequantize(lv[r, o:o + n].view(np.int8), sg[r, o:o + n], norms[r, t]))
        assert same_f32(got[o:o + n], oracle.torch_mean_rows(dec)), t
        assert same_f32(got[o:o + n], torch.stack([torch.from_numpy(d) for d in dec]).mean(0).numpy()), t


def test_mean_rejects_too_many_rows_and_bad_scales():
    """More rows than the cascade restatement covers is an argument error, and the ops reject scales the
    kernel would misread (host, fp64, short, transposed)."""
    q = torch.zeros(2, 32, dtype=torch.int8, device=DEV)
    with pytest.raises(ValueError):
        ops.dequantize_mean(q, torch.ones(2), 32)                                   # host scales
    with pytest.raises(ValueError):
        ops.dequantize_mean(q, torch.ones(2, dtype=torch.float64, device=DEV), 32)  # fp64
    lay = ops.BucketLayout([10, 20], align=1)
    qb = torch.zeros(2, 32, dtype=torch.int8, device=DEV)
    with pytest.raises(ValueError):
        ops.dequantize_mean_batched(qb, torch.ones(2, 1, device=DEV), lay)          # too few per row
    with pytest.raises(ValueError):
        ops.dequantize_mean_batched(qb, torch.ones(2, 2), lay)                      # host
    # a transposed [T, K] view: the op takes it as [K, T] only through a contiguous copy
    sc_t = torch.tensor([[1.0, 2.0], [3.0, 4.0]], device=DEV).t()
    got = ops.dequantize_mean_batched(torch.ones(2, 32, dtype=torch.int8, device=DEV), sc_t, lay).cpu()
    assert torch.equal(got[:10], torch.full((10,), 1.5)) and torch.equal(got[10:30], torch.full((20,), 3.5))
    with pytest.raises(ValueError):
        ops.decode_batched(qb[0], torch.ones(1, device=DEV), lay)                   # short scales
    with pytest.raises(ValueError):
        ops.decode_batched(qb[0], torch.ones(2), lay)                               # host scales
    with pytest.raises(ValueError):
        ops.decode_batched_int4(qb[0].view(torch.uint8), torch.ones(2, dtype=torch.float64, device=DEV),
                                ops.BucketLayout([10, 20], align=2))
    lib = adfl_amd._lib.load()
    big = 1 << 20
    assert lib.adfl_slq_dequantize_mean(q.data_ptr(), 32, big, 32, q.data_ptr(), 1, q.data_ptr(), None) != 0
