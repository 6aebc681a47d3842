"""GPU: adfl_bucket_gather / adfl_bucket_scatter (csrc/bucket_copy.hip) — a device state dict staged into
its bucket and handed back as owned tensors in one launch each way: byte-identical to torch.cat / per-slot
copies, for 1/2/4/8-byte elements, compact layouts (every offset phase), aligned layouts (pads untouched),
source / destination views at every phase mod 16, qint8 payloads; and the argument checks."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from adfl_amd import ops  # noqa: E402

DEV = torch.device("cuda", 0)
SIZES = [1, 3, 16, 17, 8191, 8192, 8193, 40000, 5, 70001, 2]


def _rand(n, dtype, g):
    raw = torch.randint(0, 256, (n * torch.tensor([], dtype=dtype).element_size(),), dtype=torch.uint8,
                        device=DEV, generator=g)
    return raw.view(dtype)


@pytest.mark.parametrize("dtype", [torch.uint8, torch.float16, torch.float32, torch.float64])
@pytest.mark.parametrize("align", [1, 64])
def test_gather_then_scatter_round_trip(dtype, align):
    g = torch.Generator(device=DEV).manual_seed(3)
    lay = ops.BucketLayout(SIZES, align=align)
    # sources at every phase: views into a larger buffer at offsets 0, 1, 2, ...
    srcs = []
    for i, n in enumerate(SIZES):
        base = _rand(n + 16, dtype, g)
        srcs.append(base[i % 16:i % 16 + n])
    bucket = _rand(lay.total, dtype, g)                  # pads hold garbage that must survive
    before = bucket.clone()
    ops.bucket_gather(srcs, lay, bucket)
    torch.cuda.synchronize()
    b = bucket.view(torch.uint8).cpu().numpy()
    es = bucket.element_size()
    covered = np.zeros(lay.total * es, bool)
    for t, (o, n) in enumerate(zip(lay.offsets.tolist(), SIZES)):
        want = srcs[t].contiguous().view(torch.uint8).cpu().numpy()
        assert np.array_equal(b[o * es:(o + n) * es], want), t
        covered[o * es:(o + n) * es] = True
    assert np.array_equal(b[~covered], before.view(torch.uint8).cpu().numpy()[~covered])   # pads untouched
    # scatter back into fresh tensors, and into views at odd phases
    outs = [torch.empty(n, dtype=dtype, device=DEV) for n in SIZES]
    ops.bucket_scatter(bucket, lay, outs)
    views = []
    for i, n in enumerate(SIZES):
        base = torch.zeros(n + 16, dtype=dtype, device=DEV)
        views.append(base[(i * 7) % 16:(i * 7) % 16 + n])
    ops.bucket_scatter(bucket, lay, views)
    torch.cuda.synchronize()
    for t in range(len(SIZES)):
        s = srcs[t].view(torch.uint8).cpu().numpy()
        assert np.array_equal(outs[t].view(torch.uint8).cpu().numpy(), s), t
        assert np.array_equal(views[t].view(torch.uint8).cpu().numpy(), s), t


def test_qint8_payloads_gather_and_scatter():
    """qint8 tensors are read and written through their own storage (no int8 view objects)."""
    lay = ops.BucketLayout([5, 9000, 3], align=1)
    x = [torch.randn(n, device=DEV) for n in (5, 9000, 3)]
    qs = [torch.quantize_per_tensor(t, 0.01, 0, torch.qint8) for t in x]
    bucket = torch.empty(lay.total, dtype=torch.int8, device=DEV)
    ops.bucket_gather(qs, lay, bucket)
    outs = [torch._empty_affine_quantized((n,), scale=0.01, zero_point=0, dtype=torch.qint8, device=DEV)
            for n in (5, 9000, 3)]
    ops.bucket_scatter(bucket, lay, outs)
    torch.cuda.synchronize()
    for q, o in zip(qs, outs):
        assert torch.equal(q.int_repr(), o.int_repr())


def test_argument_checks():
    lay = ops.BucketLayout([4, 4], align=1)
    bucket = torch.empty(8, device=DEV)
    with pytest.raises(ValueError):
        ops.bucket_gather([torch.empty(4, device=DEV)], lay, bucket)            # tensor count
    with pytest.raises(ValueError):
        ops.bucket_gather([torch.empty(4, device=DEV), torch.empty(5, device=DEV)], lay, bucket)   # size
    with pytest.raises(ValueError):
        ops.bucket_scatter(bucket, lay, [torch.empty(4, device=DEV), torch.empty(4, dtype=torch.float64,
                                                                                  device=DEV)])  # element size
    with pytest.raises(ValueError):
        ops.bucket_scatter(bucket, lay, [torch.empty(4, device=DEV), torch.empty(8, device=DEV)[::2]])
    from adfl_amd import _lib
    lib = _lib.load()
    assert lib.adfl_bucket_gather(16, 16, 1, 16, 3, None) == -1
    assert lib.adfl_bucket_scatter(16, None, 1, 16, 4, None) == -1
    assert lib.adfl_bucket_scatter(16, 16, 0, 16, 4, None) == 0    # nothing to copy
