"""GPU: QSGDChannel / RQSGDChannel / CNATChannel.receive_mean — a synchronous server decoding K client
updates and averaging them, simple_aggregate([on_server_receive(c)[0] for c in updates])
(Src/ADFL/Strategy/simple.py:83-89 over Src/ADFL/model.py:221-234), with the encoded tensors decoded and
averaged in one HIP launch (adfl_stoch_dequantize_mean_batched).

* against simple_aggregate over the channel's own per-update decode: bit-identical for every K (the kernel
  sums in torch's CPU order, csrc/torch_sum_order.h; columns of -0 decodes sum to +0 as torch's do);
* the encoded tensors bit for bit against the oracle's decodes (oracle/stoch_oracle.py) averaged in
  torch's order (oracle.torch_mean_rows), for every K; the reference's own payloads and aggregates at
  K = 5 .. 20 are in tests/test_gpu_aggregate_golden.py;
* all-zero tensors (the reference's norm == 0 payload), fp16 tensors (decoded to fp32), biases and int64
  counters (aggregated as simple_aggregate does), device-resident payloads;
* receive_add_ (the client pool's add_to_model_all, QAFeL's hidden-state update): bit-identical to
  on_client_receive + add_parameters_inpace (Src/ADFL/model.py:337-347) for device and host models."""

import numpy as np
import pytest
import torch

import slq_oracle as oracle
import stoch_oracle as so

pytestmark = pytest.mark.gpu

adfl_amd = pytest.importorskip("adfl_amd")
from adfl_amd.Channel import CNATChannel, QSGDChannel, RQSGDChannel  # noqa: E402

SHAPES = {"conv1.weight": (64, 3, 7, 7), "fc.weight": (10, 513), "layer.weight": (257, 255), "tiny.weight": (1, 3),
          "big.weight": (300, 1000)}
CHANNELS = {"qsgd": (QSGDChannel, 8), "rqsgd": (RQSGDChannel, 4), "cnat": (CNATChannel, 8)}


def simple_aggregate(parameters):
    """Src/ADFL/model.py:221-234."""
    out = {}
    with torch.no_grad():
        for name in parameters[0].keys():
            out[name] = torch.sum(torch.stack([p[name] for p in parameters], dim=0), dim=0) / len(parameters)
    return out


def _client(k):
    g = torch.Generator().manual_seed(200 + k)
    d = {n: torch.randn(s, generator=g) * (10.0 ** -(i % 3)) for i, (n, s) in enumerate(SHAPES.items())}
    d["zero.weight"] = torch.zeros(7, 9)                                     # norm == 0 payload
    d["half.weight"] = (torch.randn(33, 65, generator=g) * 1e-2).half()      # fp16: decoded to fp32
    d["fc.bias"] = torch.randn(10, generator=g)
    d["bn.num_batches_tracked"] = torch.tensor(7 + k, dtype=torch.int64)
    return d


def _bits(t: torch.Tensor) -> np.ndarray:
    return t.numpy().reshape(-1).view(np.uint32)


def _oracle_decode(codec, p, bits):
    q = p.data.numpy().reshape(-1)
    s = p.signs.numpy().reshape(-1)
    if codec == "qsgd":
        return so.qsgd_dequantize(q.view(np.uint8), s, 2 ** bits - 1, float(p.scale))
    if codec == "rqsgd":
        return so.rqsgd_dequantize(q.view(np.uint8), s, 2 ** bits - 1, float(p.scale), float(p.scale_2))
    return so.cnat_dequantize(q.view(np.int8), s, float(p.scale))


def _oracle_mean(codec, updates, name, bits):
    rows = []
    for u in updates:
        p = u.params[name]
        rows.append(np.zeros(p.data.numel(), np.float32) if float(p.scale) == 0 else _oracle_decode(codec, p, bits))
    return oracle.torch_mean_rows(rows)   # simple_aggregate's sum order, then / K


@pytest.mark.parametrize("codec", list(CHANNELS))
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 16, 20])
def test_receive_mean_matches_simple_aggregate(codec, k):
    cls, bits = CHANNELS[codec]
    ch = cls(bits)
    torch.manual_seed(k)
    updates = [ch.on_client_send(_client(r))[0] for r in range(k)]
    decoded = [ch.on_server_receive(u)[0] for u in updates]
    want = simple_aggregate(decoded)
    got, t = ch.receive_mean(updates)
    assert t > 0 and list(got) == list(want)
    for n in want:
        assert got[n].device.type == "cpu" and got[n].shape == want[n].shape and got[n].dtype == want[n].dtype, n
        if want[n].dtype == torch.float32 and want[n].ndim > 1:
            assert np.array_equal(_bits(got[n]), _oracle_mean(codec, updates, n, bits).view(np.uint32)), n
        assert np.array_equal(got[n].numpy().reshape(-1).view(np.uint8),
                              want[n].numpy().reshape(-1).view(np.uint8)), n
    got["fc.weight"].add_(1.0)   # owned and writable


@pytest.mark.parametrize("codec", list(CHANNELS))
def test_receive_mean_negative_zero_columns(codec):
    """Decodes of -0 (level 0 with sign -1, or min_factor 0 for RQSGD) in every update: the mean is +0, as
    torch's sum from zero gives, not the -0 a sum seeded with the first row would."""
    cls, bits = CHANNELS[codec]
    ch = cls(bits)
    x = torch.full((4, 64), -1e-30)
    x[0, 0] = -1.0    # the norm: every other element quantizes to level 0 with sign -1
    x[0, 1] = 0.0     # RQSGD's min factor 0: its level-0 decodes are 0 * sign
    updates = [ch.on_client_send({"w": x.clone()})[0] for _ in range(2)]
    decoded = [ch.on_server_receive(u)[0] for u in updates]
    want = simple_aggregate(decoded)["w"]
    got = ch.receive_mean(updates)[0]["w"]
    assert np.array_equal(_bits(got), _bits(want))
    if codec != "cnat":
        assert (torch.signbit(decoded[0]["w"]) & (decoded[0]["w"] == 0)).any()   # -0 decodes present
        assert not (torch.signbit(got) & (got == 0)).any()


@pytest.mark.parametrize("codec", list(CHANNELS))
def test_receive_mean_device_payloads(codec):
    """Device-resident updates (K = 3): the encoded tensors' mean stays on the device and equals
    simple_aggregate of the channel's own decodes on CPU copies, bit for bit."""
    cls, bits = CHANNELS[codec]
    ch = cls(bits)
    dev = torch.device("cuda", 0)
    updates = [ch.on_client_send({n: t.to(dev) if t.ndim > 1 else t for n, t in _client(r).items()})[0]
               for r in range(3)]
    got, _ = ch.receive_mean(updates)
    want = simple_aggregate([{n: t.cpu() for n, t in ch.on_server_receive(u)[0].items()} for u in updates])
    for n in want:
        assert got[n].is_cuda == (want[n].ndim > 1), n
        assert torch.equal(got[n].cpu(), want[n]), n


def test_receive_mean_errors():
    ch = QSGDChannel(8)
    with pytest.raises(AssertionError):
        ch.receive_mean([])
    u1 = ch.on_client_send({"w": torch.randn(4, 4)})[0]
    u2 = ch.on_client_send({"w": torch.randn(4, 5)})[0]
    with pytest.raises(RuntimeError):   # torch.stack of unequal shapes, as simple_aggregate raises
        ch.receive_mean([u1, u2])


def add_parameters_inpace(model, delta):
    """Src/ADFL/model.py:337-347 with alpha = beta = 1, to_float=False."""
    with torch.no_grad():
        for n in model:
            model[n].mul_(1).add_(delta[n].to(model[n].device), alpha=1)


@pytest.mark.parametrize("codec", list(CHANNELS))
@pytest.mark.parametrize("where", ["cuda", "cpu"])
def test_receive_add_matches_decode_then_add(codec, where):
    cls, bits = CHANNELS[codec]
    ch = cls(bits)
    c_params = ch.on_server_send(_client(0))[0]
    base = [_client(10 + m) for m in range(2)]
    for m in base:
        m["half.weight"] = m["half.weight"].float()   # models in fp32; the update was encoded from fp16
    dev = torch.device(where, 0) if where == "cuda" else torch.device("cpu")
    mine = [{n: t.clone().to(dev) if t.ndim > 1 else t.clone() for n, t in m.items()} for m in base]
    ref = [{n: t.clone() for n, t in m.items()} for m in base]
    t = ch.receive_add_(c_params, mine)
    decoded = ch.on_client_receive(c_params)[0]
    for m in ref:
        add_parameters_inpace(m, decoded)
    assert t > 0
    for a, b in zip(mine, ref):
        for n in b:
            assert a[n].device.type == (where if b[n].ndim > 1 else "cpu"), n
            assert np.array_equal(a[n].cpu().numpy().reshape(-1).view(np.uint8), b[n].numpy().reshape(-1).view(np.uint8)), n
