"""GPU: fused decode + accumulate into K models (adfl_slq_dequantize_add_batched, SLQChannel.receive_add_)
against the reference's route — on_client_receive then add_parameters_inpace(model, decoded, 1, 1)
(Src/ADFL/Client/pool.py:62-75, Src/ADFL/Server/qafel.py:176-179, Src/ADFL/model.py:337-347) — bit for bit."""

import copy

import numpy as np
import pytest
import torch

import slq_oracle as oracle

pytestmark = pytest.mark.gpu

from adfl_amd import ops  # noqa: E402
from adfl_amd.Channel import SLQChannel  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("align", [64, 1, 2])
@pytest.mark.parametrize("sizes,k", [([1, 3, 5, 8192, 8193, 70001], 3), ([1 << 20], 1), ([64] * 300, 8),
                                     ([7, 1, 8191, 8195, 13, 40000, 2], 2)])
def test_dequantize_add_matches_oracle(sizes, k, align):
    """Aligned buckets (offsets multiples of 64: 16-byte path) and compact ones (align 1 / 2: offsets with every
    residue mod 4, the element-wise path; include/adfl_slq.h no longer requires 4-element offsets)."""
    rng = np.random.default_rng(len(sizes) * 10 + k)
    lay = ops.BucketLayout(sizes, align=align)
    flat = np.zeros(lay.total, np.float32)
    xs = []
    for off, n in zip(lay.offsets, sizes):
        x = rng.standard_normal(n, dtype=np.float32) * np.float32(1e-3)
        flat[off:off + n] = x
        xs.append(x)
    q, s = ops.encode_batched(torch.from_numpy(flat).to(DEV), lay, 8)
    models = [[torch.from_numpy(rng.standard_normal(n, dtype=np.float32)).to(DEV) for n in sizes] for _ in range(k)]
    before = [[m.cpu().numpy() for m in model] for model in models]
    ops.dequantize_add_batched(q, s, lay, models)
    torch.cuda.synchronize()
    qh, sh = q.cpu().numpy(), s.cpu().numpy()
    for mk, bk in zip(models, before):
        for t, (m, b, off, n) in enumerate(zip(mk, bk, lay.offsets, sizes)):
            d = oracle.np_decode(qh[off:off + n], sh[t])
            want = (b + d).astype(np.float32)
            assert np.array_equal(m.cpu().numpy().view(np.uint32), want.view(np.uint32)), (t, n)


def test_dequantize_add_rejects_bad_targets():
    lay = ops.BucketLayout([10, 20])
    q = torch.zeros(lay.total, dtype=torch.int8, device=DEV)
    s = torch.ones(2, device=DEV)
    good = [torch.zeros(10, device=DEV), torch.zeros(20, device=DEV)]
    with pytest.raises(ValueError, match="16-byte aligned fp32"):
        ops.dequantize_add_batched(q, s, lay, [[good[0], torch.zeros(21, device=DEV)]])
    with pytest.raises(ValueError, match="16-byte aligned fp32"):
        ops.dequantize_add_batched(q, s, lay, [[good[0], torch.zeros(21, device=DEV)[1:]]])


def _model(seed, device):
    g = torch.Generator().manual_seed(seed)
    m = {"conv.weight": torch.randn(64, 3, 3, 3, generator=g), "fc.weight": torch.randn(10, 513, generator=g),
         "fc.bias": torch.randn(10, generator=g), "bn.num_batches_tracked": torch.tensor(7),
         "emb.weight": torch.randn(1001, 33, generator=g)}
    return {k: v.to(device) for k, v in m.items()}


@pytest.mark.parametrize("target_device", ["cuda", "cpu"])
def test_channel_receive_add_matches_reference_route(target_device):
    """receive_add_ == on_client_receive + add_parameters_inpace(t, decoded, 1, 1, to_float=False) for each t."""
    ch = SLQChannel(8)
    update = {k: v * 1e-2 if v.is_floating_point() else v for k, v in _model(1, "cpu").items()}
    c, _ = ch.on_client_send(update)
    targets = [_model(10 + i, target_device) for i in range(3)]
    expect = [copy.deepcopy({k: v.cpu() for k, v in t.items()}) for t in targets]
    decoded, _ = ch.on_client_receive(c)
    for t in expect:  # the reference's route (model.py:337-347), on the host
        for key in decoded:
            t[key].mul_(1).add_(decoded[key], alpha=1)
    secs = ch.receive_add_(c, targets)
    assert secs >= 0
    for t, e in zip(targets, expect):
        for key in e:
            got = t[key].cpu()
            assert got.dtype == e[key].dtype
            assert torch.equal(got.view(-1).view(torch.int32) if got.is_floating_point() else got,
                               e[key].view(-1).view(torch.int32) if got.is_floating_point() else e[key]), key


def test_receive_add_back_to_back_cpu_payloads():
    """Consecutive receive_add_ calls with different CPU payloads: the pinned staging of call i+1 must not be
    rewritten while call i's H2D still reads it. Each accumulation equals the reference route."""
    ch = SLQChannel(8)
    updates = []
    for i in range(4):
        u = {k: v * 10.0 ** (-i) if v.is_floating_point() else v for k, v in _model(100 + i, "cpu").items()}
        updates.append(ch.on_client_send(u)[0])
    targets = [_model(50, "cuda")]
    expect = copy.deepcopy({k: v.cpu() for k, v in targets[0].items()})
    for c in updates:
        ch.receive_add_(c, targets)
        dec, _ = ch.on_client_receive(c)
        for key in dec:
            expect[key].mul_(1).add_(dec[key], alpha=1)
    for key in expect:
        got = targets[0][key].cpu()
        if got.is_floating_point():
            assert torch.equal(got.view(-1).view(torch.int32), expect[key].view(-1).view(torch.int32)), key
        else:
            assert torch.equal(got, expect[key]), key
