"""CPU: host-side behaviour of the stochastic channels (QSGD / RQSGD / CNAT and their U* variants) that
needs no GPU: names, to_json, simulate_bandwidth, passthrough and empty-tensor branches, pickling, and
the loud failure without a device. Expected values come from the reference (tests/golden/stoch_manifest.json
facts, produced by make_golden_stoch.py executing Src/ADFL/Channel/quant.py:140-570)."""

import json
import os
import pickle

import pytest
import torch

import adfl_amd
from adfl_amd import stoch
from adfl_amd.Channel import (CNATChannel, IdentityChannel, QSGDChannel, RQSGDChannel, UCNATChannel, UQSGDChannel,
                              URQSGDChannel)
from adfl_amd.model import QuantParameters
from conftest import GOLDEN

FACTS = json.load(open(os.path.join(GOLDEN, "stoch_manifest.json")))
ALL = [QSGDChannel, UQSGDChannel, RQSGDChannel, URQSGDChannel, CNATChannel, UCNATChannel]


@pytest.mark.parametrize("cls", ALL, ids=lambda c: c.__name__)
def test_to_json_matches_reference(cls):
    assert cls(8).to_json() == FACTS["to_json"][cls.__name__]


@pytest.mark.parametrize("cls", [QSGDChannel, RQSGDChannel, CNATChannel], ids=lambda c: c.__name__)
def test_simulate_bandwidth_matches_reference(cls, monkeypatch):
    monkeypatch.setattr("time.sleep", lambda s: None)
    params = {"non_bias": torch.ones(2, 5), "bias": torch.ones(10)}
    assert cls(8).simulate_bandwidth(params, 1.0) == pytest.approx(FACTS["bandwidth"][cls.__name__], rel=1e-12)


def test_reference_test_bandwidth_values(monkeypatch):
    """Src/ADFL/Channel/Tests/test_quant.py:59,77,96,115: 442 / 474 bps make the transfer take 1 s."""
    monkeypatch.setattr("time.sleep", lambda s: None)
    params = {"non_bias": torch.randn(2, 5), "bias": torch.randn(10)}
    assert QSGDChannel(8).simulate_bandwidth(params, 442 / 1_000_000) == pytest.approx(1.0)
    assert UQSGDChannel(8).simulate_bandwidth(params, 442 / 1_000_000) == pytest.approx(1.0)
    assert RQSGDChannel(8).simulate_bandwidth(params, 474 / 1_000_000) == pytest.approx(1.0)
    assert CNATChannel(8).simulate_bandwidth(params, 442 / 1_000_000) == pytest.approx(1.0)


@pytest.mark.parametrize("cls", [QSGDChannel, RQSGDChannel, CNATChannel], ids=lambda c: c.__name__)
def test_passthrough_only_dict_needs_no_device(cls):
    b = torch.arange(5, dtype=torch.float32)
    n = torch.tensor(3)
    qp, _ = cls(8).on_client_send({"b": b, "n": n})
    ref = FACTS["passthrough"][cls.__name__]
    pb = qp.params["b"]
    assert pb.data is b and pb.scale == ref["scale"] and pb.scale_2 == ref["scale_2"]
    assert str(pb.signs.dtype) == ref["signs_dtype"] and pb.signs.numel() == ref["signs_numel"]
    assert qp.size == ref["size"] and str(qp.params["n"].q_dtype) == ref["n_dtype"]
    dec, _ = cls(8).on_server_receive(qp)
    assert dec["b"].data_ptr() == b.data_ptr() and dec["n"].data_ptr() == n.data_ptr()


@pytest.mark.parametrize("cls", [QSGDChannel, RQSGDChannel, CNATChannel], ids=lambda c: c.__name__)
def test_empty_matrix_takes_the_zero_branch_without_a_device(cls):
    """vector_norm of an empty tensor is 0: uint8 zeros_like, int8 ones_like, tensor(0.) scale."""
    qp, _ = cls(8).on_client_send({"w": torch.empty(0, 4)})
    p = qp.params["w"]
    assert p.data.dtype == torch.uint8 and p.data.shape == (0, 4) and p.signs.dtype == torch.int8
    assert isinstance(p.scale, torch.Tensor) and p.scale.item() == 0.0 and qp.size == 0
    dec, _ = cls(8).on_server_receive(qp)
    assert dec["w"].shape == (0, 4) and dec["w"].dtype == torch.float32


@pytest.mark.parametrize("cls", [UQSGDChannel, URQSGDChannel, UCNATChannel], ids=lambda c: c.__name__)
def test_unidirectional_server_send_is_identity(cls):
    x = torch.randn(3, 4)
    c, t = cls(8).on_server_send({"w": x})
    ref_c, _ = IdentityChannel(no_compute_time=True).on_server_send({"w": x})
    assert type(c) is type(ref_c) and t == 0
    d, _ = cls(8).on_client_receive(c)
    assert torch.equal(d["w"], x)


def test_channels_are_picklable_and_stateless():
    for cls in ALL:
        ch = pickle.loads(pickle.dumps(cls(4)))
        assert isinstance(ch, cls) and vars(ch) == {"bits": 4, "levels": 15}


def test_receive_asserts_quant_parameters():
    with pytest.raises(AssertionError):
        QSGDChannel(8).on_server_receive({"w": torch.zeros(2, 2)})
    assert isinstance(QuantParameters({}, 0), QuantParameters)


def test_integer_tensors_raise_the_reference_error():
    """The reference's first op on an integer tensor, torch.linalg.vector_norm, raises (quant.py:226,367,512);
    fp16 / bf16 / fp64 tensors are encoded in their own dtype (tests/test_gpu_stoch_dt.py)."""
    for cls in (QSGDChannel, RQSGDChannel, CNATChannel):
        with pytest.raises(RuntimeError, match="Expected a floating point or complex tensor as input. Got Long"):
            cls(8).on_client_send({"w": torch.ones(2, 2, dtype=torch.int64)})
        with pytest.raises(RuntimeError, match="Got Int"):
            cls(8).on_client_send({"w": torch.ones(0, 2, dtype=torch.int32)})


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_silent_cpu_fallback():
    for cls in (QSGDChannel, RQSGDChannel, CNATChannel):
        with pytest.raises(Exception):
            cls(8).on_client_send({"w": torch.randn(4, 4)})
    with pytest.raises(ValueError, match="device tensor"):
        stoch.qsgd_encode_batched(torch.randn(16), adfl_amd.ops.BucketLayout([16]), 8)


def test_rng_stream_is_seeded_from_torch():
    torch.manual_seed(3)
    a = stoch.RngStream()
    torch.manual_seed(3)
    b = stoch.RngStream()
    assert a.seed == b.seed
    assert a.take(10) == (a.seed, 0) and a.take(1) == (a.seed, 3) and a.counter == 4


@pytest.mark.parametrize("cls", [QSGDChannel, RQSGDChannel, CNATChannel], ids=lambda c: c.__name__)
def test_receive_mean_and_add_without_encoded_entries_need_no_device(cls):
    """Passthrough entries and empty matrices (the zero branch) aggregate and accumulate on the host as
    simple_aggregate / add_parameters_inpace do (Src/ADFL/model.py:221-234, 337-347); no updates asserts."""
    ch = cls(8)
    ups = [ch.on_client_send({"b": torch.arange(5, dtype=torch.float32) * (k + 1), "w": torch.empty(0, 4),
                              "n": torch.tensor(3 + k)})[0] for k in range(3)]
    got, t = ch.receive_mean(ups)
    assert t > 0 and list(got) == ["b", "w", "n"]
    assert torch.equal(got["b"], torch.arange(5, dtype=torch.float32) * 2)
    assert got["w"].shape == (0, 4) and got["w"].dtype == torch.float32
    want_n = torch.sum(torch.stack([torch.tensor(3 + k) for k in range(3)]), dim=0) / 3   # true division: fp32
    assert torch.equal(got["n"], want_n) and got["n"].dtype == want_n.dtype
    with pytest.raises(AssertionError):
        ch.receive_mean([])
    model = {"b": torch.ones(5), "w": torch.zeros(0, 4), "n": torch.tensor(1)}
    ch.receive_add_(ups[0], [model])
    assert torch.equal(model["b"], torch.arange(5, dtype=torch.float32) + 1) and model["n"].item() == 4
