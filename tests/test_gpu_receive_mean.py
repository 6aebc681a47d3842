"""GPU: SLQChannel.receive_mean / PackedSLQChannel.receive_mean — a synchronous server decoding K client
updates and averaging them, simple_aggregate([on_server_receive(c)[0] for c in updates])
(Src/ADFL/Strategy/simple.py:83-89 over Src/ADFL/model.py:221-234), with the quantized tensors decoded and
averaged in one HIP launch.

* against simple_aggregate over the channel's own per-update decode (restated below: torch.stack, sum over
  dim 0, / K — the reference function's three ops): bit-identical for every K (the kernels sum in torch's
  CPU order, csrc/torch_sum_order.h; the reference itself executed at K = 1 .. 64 is
  tests/test_gpu_aggregate_golden.py);
* the quantized tensors bit for bit against the oracle's torch-order mean of the decoded payloads
  (oracle.dequantize_mean / dequantize_mean_int4) for every K;
* passthrough entries (biases, 0-dim int64 counters) exactly as simple_aggregate computes them."""

import numpy as np
import pytest
import torch

import slq_oracle as oracle

pytestmark = pytest.mark.gpu

adfl_amd = pytest.importorskip("adfl_amd")
from adfl_amd.Channel import PackedSLQChannel, SLQChannel  # noqa: E402

SHAPES = {"conv1.weight": (64, 3, 7, 7), "fc.weight": (10, 513), "layer.weight": (257, 255), "tiny.weight": (1, 3),
          "big.weight": (300, 1000), "one.weight": (1, 1), "six.weight": (2, 3), "rag.weight": (37, 101)}


def simple_aggregate(parameters):
    """Src/ADFL/model.py:221-234."""
    out = {}
    with torch.no_grad():
        for name in parameters[0].keys():
            out[name] = torch.sum(torch.stack([p[name] for p in parameters], dim=0), dim=0) / len(parameters)
    return out


def _client(k):
    g = torch.Generator().manual_seed(100 + k)
    d = {n: torch.randn(s, generator=g) * (10.0 ** -(i % 3)) for i, (n, s) in enumerate(SHAPES.items())}
    d["fc.bias"] = torch.randn(10, generator=g)
    d["bn.num_batches_tracked"] = torch.tensor(7 + k, dtype=torch.int64)
    return d


def _same(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.numpy().reshape(-1).view(np.uint8),
                                                                         b.numpy().reshape(-1).view(np.uint8))


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 10, 16, 17, 20])
def test_receive_mean_matches_simple_aggregate(k, packed):
    ch = PackedSLQChannel(4) if packed else SLQChannel(8)
    updates = [ch.on_client_send(_client(r))[0] for r in range(k)]
    decoded = [ch.on_server_receive(u)[0] for u in updates]
    want = simple_aggregate(decoded)
    got, t = ch.receive_mean(updates)
    assert t > 0 and list(got) == list(want)
    for n in want:
        assert got[n].device.type == "cpu" and got[n].shape == want[n].shape and got[n].dtype == want[n].dtype, n
        if n in SHAPES:
            # the oracle's torch-order mean of the same payloads
            numel = int(np.prod(SHAPES[n]))
            if packed:
                ref = oracle.dequantize_mean_int4([u.params[n].data.view(torch.uint8).numpy() for u in updates],
                                                  [u.params[n].scale for u in updates], numel)
            else:
                ref = oracle.dequantize_mean([u.params[n].data.int_repr().numpy() for u in updates],
                                             [u.params[n].data.q_scale() for u in updates])
            assert np.array_equal(got[n].numpy().reshape(-1).view(np.uint32), ref.view(np.uint32)), n
        assert _same(got[n], want[n]), n
    got["fc.weight"].add_(1.0)   # owned and writable


def test_receive_mean_device_updates_and_c3_layout():
    """Device-resident updates stay on the device; a C3-sized dict (ResNet-18's 11.7 M parameters in 256
    tensors, equal layout) from 4 clients is one launch and bit-identical to simple_aggregate (on CPU copies,
    as the reference aggregates)."""
    import recipes
    sizes = recipes.bucket_sizes("equal")
    ch = SLQChannel(8)
    dev = torch.device("cuda", 0)
    updates = []
    for r in range(4):
        g = torch.Generator(device=dev).manual_seed(r)
        updates.append(ch.on_client_send({f"t{i}.weight": torch.randn(1, n, device=dev, generator=g) * 1e-3
                                          for i, n in enumerate(sizes)})[0])
    got, _ = ch.receive_mean(updates)
    want = simple_aggregate([{n: t.cpu() for n, t in ch.on_server_receive(u)[0].items()} for u in updates])
    for n in want:
        assert got[n].is_cuda and torch.equal(got[n].cpu(), want[n]), n


@pytest.mark.parametrize("packed", [False, True])
def test_receive_mean_device_payloads_small(packed):
    """Device-resident payloads (the per-tensor device staging path) for both channels, K = 3: the result
    stays on the device and equals simple_aggregate of the channel's own decodes as the reference runs it,
    on CPU tensors (model.py:195-197 hands the strategies CPU state dicts), bit for bit. (torch's GPU sum
    over dim 0 may group the additions differently.)"""
    ch = PackedSLQChannel(4) if packed else SLQChannel(8)
    dev = torch.device("cuda", 0)
    updates = [ch.on_client_send({n: t.to(dev) if t.ndim > 1 else t for n, t in _client(r).items()})[0]
               for r in range(3)]
    got, _ = ch.receive_mean(updates)
    want = simple_aggregate([{n: t.cpu() for n, t in ch.on_server_receive(u)[0].items()} for u in updates])
    for n in want:
        assert got[n].is_cuda == (n in SHAPES) and torch.equal(got[n].cpu(), want[n]), n


def test_receive_mean_errors():
    ch = SLQChannel(8)
    with pytest.raises(AssertionError):
        ch.receive_mean([])
    u1 = ch.on_client_send({"w": torch.randn(4, 4)})[0]
    u2 = ch.on_client_send({"w": torch.randn(4, 5)})[0]
    with pytest.raises(RuntimeError):   # torch.stack of unequal shapes, as simple_aggregate raises
        ch.receive_mean([u1, u2])


@pytest.mark.parametrize("channel", ["SLQChannel", "QSGDChannel"])
def test_receive_mean_falls_back_when_torch_sums_in_another_order(channel, monkeypatch):
    """If this torch's CPU sum order is not the one the device mean kernels restate (sum_order.self_check
    fails), receive_mean aggregates every entry on the host as the reference does — still simple_aggregate
    of the channel's own decodes, bit for bit — and warns once (the device and host halves of
    one aggregate must not disagree)."""
    import importlib
    from adfl_amd import sum_order
    from adfl_amd.Channel import quant
    C = importlib.import_module("adfl_amd.Channel")
    ch = getattr(C, channel)(8)
    updates = [ch.on_client_send(_client(r))[0] for r in range(5)]
    decoded = [ch.on_server_receive(u)[0] for u in updates]
    want = simple_aggregate(decoded)
    monkeypatch.setattr(sum_order, "self_check", lambda: False)
    monkeypatch.setattr(quant, "_ORDER_WARNED", [False])
    with pytest.warns(RuntimeWarning, match="sum order"):
        got, _ = ch.receive_mean(updates)
    for n in want:
        assert _same(got[n], want[n]), n
