"""GPU: the single-launch CNAT encode with a per-tensor arrival counter (adfl_cnat_encode_arrival,
VERDICT r03 item 7) equals the multi-launch and the register-resident encodes bit for bit: exponents, signs
and norms, with in-kernel Philox and with injected uniforms, on buckets with 1..16 chunks per tensor,
all-zero tensors (the norm == 0 rewrite of the whole tensor by its last block), NaN / inf tensors, compact
and aligned layouts, and across repeated launches (the counters reset themselves)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from adfl_amd import ops, stoch  # noqa: E402

DEV = torch.device("cuda", 0)


def _bucket(sizes, align, seed):
    lay = ops.BucketLayout(sizes, align=align)
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(lay.total, device=DEV, generator=g) * 1e-3
    return lay, x


def _enc(x, lay, **kw):
    # zeroed planes: the alignment padding between tensors belongs to no chunk and is never written
    e0 = torch.zeros(lay.total, dtype=torch.int8, device=DEV)
    s0 = torch.zeros(lay.total, dtype=torch.int8, device=DEV)
    e, s, n = stoch.cnat_encode_batched(x, lay, 8, exps=e0, signs=s0, **kw)
    return e.clone(), s.clone(), n.clone()


def _same(a, b):
    for u, v in zip(a, b):
        assert torch.equal(u.view(torch.uint8) if u.dtype != torch.float32 else u.view(torch.int32),
                           v.view(torch.uint8) if v.dtype != torch.float32 else v.view(torch.int32))


@pytest.mark.parametrize("align", [1, 64])
def test_arrival_equals_multi_launch_and_resident(align):
    sizes = [8192 * k + r for k in range(0, 16) for r in (1, 37, 4096)][:40] + [45663] * 8 + [1, 2, 3, 7]
    sizes = [s for s in sizes if s <= 16 * 8192]
    lay, x = _bucket(sizes, align, 7)
    # zero, NaN, inf tensors
    o = lay.offsets
    x[o[3]:o[3] + sizes[3]] = 0.0
    x[o[5]:o[5] + sizes[5]] = 0.0
    x[o[5] + 7] = -0.0
    x[o[8] + 11] = float("nan")
    x[o[9] + 5] = float("inf")
    for kw in ({"seed": 3, "counter": 11}, {"uniforms": torch.rand(lay.total, device=DEV)}):
        ref = _enc(x, lay, resident=False, arrival=False, **kw)
        res = _enc(x, lay, arrival=False, **kw)
        arr = _enc(x, lay, arrival=True, **kw)
        _same(ref, res)
        _same(ref, arr)
        for _ in range(3):
            _same(ref, _enc(x, lay, arrival=True, **kw))
    assert int(stoch._arrival_counters(lay, DEV)[:lay.ntensors].abs().sum()) == 0


def test_arrival_c3_equal_layout():
    base, rem = divmod(11_689_512, 256)
    lay, x = _bucket([base + (1 if i < rem else 0) for i in range(256)], 1, 1)
    ref = _enc(x, lay, resident=False, arrival=False, seed=5)
    _same(ref, _enc(x, lay, arrival=True, seed=5))
