"""GPU: the channels' aggregate step against the reference executed in place (tests/golden/aggregate.npz,
made by tests/golden/make_golden_aggregate.py; no reference code on this box, only its outputs).

* SLQChannel(8).receive_mean over K client updates equals the reference's simple_aggregate of its own
  decodes (Src/ADFL/model.py:221-234; Src/ADFL/Strategy/simple.py:83-89) bit for bit at K = 1 .. 64 —
  the 10 / 16 / 20 clients Src/main.py runs included — biases and the int64 counter included;
  SLQChannel(4) and PackedSLQChannel(4) (whose int4 packing aliases only out-of-range codes, i.e. the
  inf / NaN tensors) at K = 3 .. 20;
* the peer mean (Examples/ray_ad.py:183-188: received rows, own update exact and last, stack().mean(0))
  through ops.dequantize_mean per tensor;
* QSGDChannel / RQSGDChannel / CNATChannel.receive_mean fed the reference's OWN payloads (its torch.rand_like
  draws) equals the reference's simple_aggregate of its decodes at K = 5, 8, 16, 20;
* SLQChannel.send_with_q_error's metrics are within 1e-5 of the reference's parameter_relative_mse /
  parameter_cosine_similarity (Src/ADFL/model.py:256-323, Src/ADFL/Client/worker.py:186-189), which
  reduce in fp32."""

import json
import os

import numpy as np
import pytest
import torch

from golden_util import same_f32
from make_golden_aggregate import BIASES, SHAPES, client_dict

pytestmark = pytest.mark.gpu

adfl_amd = pytest.importorskip("adfl_amd")
from adfl_amd import ops  # noqa: E402
from adfl_amd.Channel import CNATChannel, PackedSLQChannel, QSGDChannel, RQSGDChannel, SLQChannel  # noqa: E402
from adfl_amd.model import QuantParameter, QuantParameters  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = torch.device("cuda", 0)
_cache = {}


def fixture():
    if "a" not in _cache:
        _cache["a"] = np.load(os.path.join(GOLDEN, "aggregate.npz"))
        with open(os.path.join(GOLDEN, "aggregate_manifest.json")) as f:
            _cache["m"] = json.load(f)
    return _cache["a"], _cache["m"]


def _check(got: torch.Tensor, want: np.ndarray, what):
    assert got.device.type == "cpu", what
    g = got.numpy()
    assert g.dtype == want.dtype and g.shape == want.shape, (what, g.dtype, want.dtype, g.shape, want.shape)
    if g.dtype == np.float32:
        assert same_f32(g, want), what
        assert np.array_equal(np.signbit(g[~np.isnan(g)]), np.signbit(want[~np.isnan(want)])), what
    else:
        assert np.array_equal(g, want), what


@pytest.mark.parametrize("bits", [8, 4])
def test_slq_receive_mean_is_reference_simple_aggregate(bits):
    a, m = fixture()
    ks = m["k_slq"] if bits == 8 else m["k_slq4"]
    ch = SLQChannel(bits)
    updates = [ch.on_client_send(client_dict(c))[0] for c in range(max(ks))]
    for k in ks:
        got, _ = ch.receive_mean(updates[:k])
        assert list(got) == list(SHAPES) + list(BIASES) + ["bn.num_batches_tracked"]
        for n, t in got.items():
            _check(t, a[f"slq{bits}__k{k}__{n}"], (k, n))


def test_packed_receive_mean_is_reference_simple_aggregate():
    """PackedSLQChannel(4) carries SLQChannel(4)'s codes two per byte; its aggregate equals the reference's
    SLQChannel(4) aggregate except where pack_4bit aliases an out-of-range code (127, the code of NaN x*inv:
    only client 9's inf tensor 'six.weight' from K = 10 on)."""
    a, m = fixture()
    ch = PackedSLQChannel(4)
    updates = [ch.on_client_send(client_dict(c))[0] for c in range(max(m["k_slq4"]))]
    for k in m["k_slq4"]:
        got, _ = ch.receive_mean(updates[:k])
        for n, t in got.items():
            if n == "six.weight" and k > 9:
                continue
            _check(t, a[f"slq4__k{k}__{n}"], (k, n))


@pytest.mark.parametrize("bits", [8, 4])
def test_peer_mean_is_reference_expression(bits):
    """Receiving client k // 2 of K: the K - 1 received SLQ payloads and its own fp32 update, last and exact."""
    a, m = fixture()
    ch = SLQChannel(bits)
    clients = [client_dict(c) for c in range(max(m["k_peer"]))]
    updates = [ch.on_client_send(c)[0] for c in clients]
    for k in m["k_peer"]:
        me = k // 2
        for n in SHAPES:
            numel = int(np.prod(SHAPES[n]))
            row = (numel + 15) // 16 * 16
            rows = torch.zeros(k, row, dtype=torch.int8)
            for r in range(k):
                rows[r, :numel] = updates[r].params[n].data.int_repr().reshape(-1)
            scales = torch.tensor([updates[r].params[n].data.q_scale() for r in range(k)], dtype=torch.float32)
            got = ops.dequantize_mean(rows.to(DEV), scales.to(DEV), numel, self_row=me,
                                      self_x=clients[me][n].reshape(-1).to(DEV)).cpu()
            _check(got.view(SHAPES[n]), a[f"peer{bits}__k{k}__{n}"], (k, n))


def _stoch_updates(codec, a, m, k):
    """The reference's own payloads for clients 0 .. k-1, as QuantParameters (quant.py:205-218 fields)."""
    bits = m["stoch"][codec][1]
    out = []
    for c in range(k):
        x = client_dict(c)
        qp = QuantParameters({}, 0)
        for n, t in x.items():
            if n in SHAPES:
                rec = m["stoch_scales"][f"{codec}__c{c}__{n}"]
                sbits = np.array([rec["scale"]["bits"]], np.uint32).view(np.float32)[0]
                scale = torch.tensor(float(sbits)) if rec["scale"].get("tensor") else float(sbits)
                s2r = rec["scale_2"]
                scale_2 = s2r["int"] if "int" in s2r else float(np.array([s2r["bits"]], np.uint32).view(np.float32)[0])
                q = torch.from_numpy(a[f"{codec}__c{c}__{n}__q"].copy())
                if codec == "cnat":
                    q = q.view(torch.int8)
                signs = torch.from_numpy(a[f"{codec}__c{c}__{n}__signs"].copy())
                qp.params[n] = QuantParameter(data=q, bits=bits, scale=scale, signs=signs, shape=t.shape,
                                              dtype=t.dtype, q_dtype=q.dtype, scale_2=scale_2)
                qp.size += q.nbytes
            else:
                qp.params[n] = QuantParameter(data=t, bits=bits, scale=1, signs=torch.zeros(1, dtype=torch.uint8),
                                              shape=t.shape, dtype=t.dtype, q_dtype=t.dtype)
        out.append(qp)
    return out


@pytest.mark.parametrize("codec", ["qsgd", "rqsgd", "cnat"])
def test_stoch_receive_mean_of_reference_payloads(codec):
    a, m = fixture()
    cls = {"qsgd": QSGDChannel, "rqsgd": RQSGDChannel, "cnat": CNATChannel}[codec]
    ch = cls(m["stoch"][codec][1])
    updates = _stoch_updates(codec, a, m, max(m["k_stoch"]))
    for k in m["k_stoch"]:
        got, _ = ch.receive_mean(updates[:k])
        for n, t in got.items():
            _check(t, a[f"{codec}__k{k}__{n}"], (k, n))


@pytest.mark.parametrize("bits", [8, 4])
def test_send_with_q_error_vs_reference(bits):
    """The worker's q-error metrics (Src/ADFL/Client/worker.py:186-189) equal the reference's Python doubles
    bit for bit on every client, NaN / inf clients included (qerror.py, csrc/qerror_ref.hip)."""
    _, m = fixture()
    ch = SLQChannel(bits)
    same = lambda a, b: (np.isnan(a) and np.isnan(b)) or a == b  # noqa: E731
    old = torch.get_num_threads()
    torch.set_num_threads(8)  # the generator's (tests/golden/make_golden_aggregate.py)
    try:
        for c in range(len(m["clients"])):
            ref = m["q_error"][f"slq{bits}_c{c}"]
            rmse, rcos = float(ref["mse"]), float(ref["cos"])
            _, _, mse, cos = ch.send_with_q_error(client_dict(c))
            assert same(mse, rmse) and same(cos, rcos), (c, mse, rmse, cos, rcos)
    finally:
        torch.set_num_threads(old)
