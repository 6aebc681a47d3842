"""CPU: host-side logic of the drop-in boundary against the reference's golden metadata.

No GPU is touched: bandwidth accounting, to_json, payload types, IdentityChannel (USLQ's uncompressed
direction), error behaviour, picklability and the bucket layout. The HIP path must fail loudly here."""

import pickle

import numpy as np
import pytest
import torch

import recipes
from adfl_amd import model, ops
from adfl_amd.Channel import IdentityChannel, SLQChannel, USLQChannel
from golden_util import manifest


def _bw_params():
    return {"non_bias": torch.from_numpy(recipes.randn((2, 5), 41, 1.0)),
            "bias": torch.from_numpy(recipes.randn((10,), 42, 1.0)),
            "conv": torch.from_numpy(recipes.randn((4, 3, 3, 3), 43, 1.0)),
            "nbt": torch.tensor(3, dtype=torch.int64)}


def test_get_parameter_info_reference_test():
    """Src/ADFL/Tests/test_model.py:6-20, asserted the same way."""
    params = {"non_bias_1": torch.randn(2, 2), "non_bias_2": torch.randn(3, 2, 2),
              "bias_1": torch.randn(10), "bias_2": torch.randn(4)}
    p = model.get_parameter_info(params)
    assert p.num_non_bias_w == 2 * 2 + 3 * 2 * 2 and p.num_non_bias_t == 2
    assert p.num_bias_w == 10 + 4 and p.num_bias_t == 2


@pytest.mark.parametrize("entry", manifest()["bandwidth"], ids=lambda e: f"{e['channel']}-{e['bits']}-{e['mbps']}")
def test_simulate_bandwidth_matches_reference(entry):
    ch = {"SLQChannel": lambda: SLQChannel(entry["bits"]), "USLQChannel": lambda: USLQChannel(entry["bits"]),
          "IdentityChannel": lambda: IdentityChannel(no_compute_time=True)}[entry["channel"]]()
    assert ch.simulate_bandwidth(_bw_params(), entry["mbps"]) == entry["seconds"]


def test_simulate_bandwidth_reference_test_values():
    """Src/ADFL/Channel/Tests/test_quant.py:16-21: 80 + 32 + 320 bits at 432 bps -> 1 s (not slept here)."""
    params = {"non_bias": torch.randn(2, 5), "bias": torch.randn(10)}
    assert SLQChannel(8).simulate_bandwidth(params, 432e12 / 1e6 / 1e12 * 1e9) == pytest.approx(1e-9)


def test_to_json_matches_reference():
    g = manifest()["to_json"]
    assert SLQChannel(8).to_json() == g["SLQChannel_8"]
    assert USLQChannel(4).to_json() == g["USLQChannel_4"]
    assert IdentityChannel(no_compute_time=False).to_json() == g["IdentityChannel"]


def test_identity_channel_round_trip():
    """Src/ADFL/Channel/Tests/test_channel.py:6-49 with the constructor kwarg the class actually takes."""
    x = torch.randn(2, 5)
    ch = IdentityChannel(no_compute_time=False)
    c, t = ch.on_server_send({"hi": x})
    d, _ = ch.on_client_receive(c)
    assert torch.equal(x, d["hi"]) and t >= 0
    y = torch.randn(2, 5)
    c, _ = ch.on_client_send({"hi": y})
    d, _ = ch.on_server_receive(c)
    assert torch.equal(y, d["hi"])


def test_uslq_server_send_is_identity_and_sized_like_reference():
    g = {e["what"]: e for e in manifest()["size"]}
    bp, t = USLQChannel(8).on_server_send(_bw_params())
    ref = g["USLQChannel(8).on_server_send bw_params"]
    assert type(bp).__name__ == ref["type"] and bp.size == ref["size"] and t == 0.0
    back, _ = USLQChannel(8).on_client_receive(bp)
    for k, v in _bw_params().items():
        assert torch.equal(back[k], v)


def test_payload_types_have_reference_fields():
    assert [f for f in model.QuantParameter.__dataclass_fields__] == \
        ["data", "bits", "scale", "signs", "shape", "dtype", "q_dtype", "scale_2"]
    assert [f for f in model.QuantParameters.__dataclass_fields__] == ["params", "size"]
    assert [f for f in model.ByteParameter.__dataclass_fields__] == ["data", "shape", "dtype"]


@pytest.mark.parametrize("t,msg", [
    (torch.randn(2, 2, dtype=torch.float64), "Quantize only works on Float Tensor, got Double"),
    (torch.randn(2, 2, dtype=torch.float16), "Quantize only works on Float Tensor, got Half"),
    (torch.randn(2, 2).bfloat16(), "Quantize only works on Float Tensor, got BFloat16"),
    (torch.ones(2, 2, dtype=torch.int64), "Quantize only works on Float Tensor, got Long"),
    (torch.empty(0, 4), "Expected reduction dim to be specified for input.numel\\(\\) == 0"),
])
def test_reference_error_messages(t, msg):
    """Same exception type and message as the reference's ATen path (quant.py:100-103)."""
    with pytest.raises(RuntimeError, match=msg):
        ops.require_quantizable(t)
    q_max = 127
    with pytest.raises(RuntimeError, match=msg):  # what the reference itself raises
        scale = torch.max(torch.abs(t)) / q_max
        torch.quantize_per_tensor(t, float(scale), 0, dtype=torch.qint8)
    with pytest.raises(RuntimeError, match=msg):  # and the channel raises before touching a device
        SLQChannel(8).on_client_send({"w": t})


def test_channel_is_picklable_and_stateless():
    ch = SLQChannel(8)
    ch2 = pickle.loads(pickle.dumps(ch))
    assert vars(ch2) == {"bits": 8}
    assert isinstance(pickle.loads(pickle.dumps(USLQChannel(4))), USLQChannel)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_silent_cpu_fallback():
    """Without a GPU the product path raises instead of computing on the CPU."""
    with pytest.raises(Exception):
        SLQChannel(8).on_client_send({"w": torch.randn(4, 4)})
    with pytest.raises(ValueError, match="device tensor"):
        ops.encode(torch.randn(4, 4), 8)


def test_passthrough_only_dict_needs_no_device():
    """A dict with nothing to quantize never reaches the GPU (quant.py:80-81)."""
    b = torch.randn(5)
    qp, _ = SLQChannel(8).on_client_send({"b": b, "n": torch.tensor(1)})
    assert qp.params["b"].data is b and qp.params["b"].scale == 1 and qp.size == 5 * 4 + 8
    dec, _ = SLQChannel(8).on_server_receive(qp)
    assert dec["b"].data_ptr() == b.data_ptr()  # `q_param.data.data`: a new view of the same storage


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 16, 17, 20, 64])
def test_receive_mean_passthrough_entries_are_simple_aggregate(k):
    """receive_mean over updates with nothing quantized: simple_aggregate's own values on the host
    (Src/ADFL/model.py:221-234: stack, sum over dim 0, / K; an int64 counter becomes fp32), key order of
    the first update, no device. The entries are summed batched (concatenated per dtype: int64 with K
    elementwise adds, fp32 in torch's own summation order per entry, adfl_amd.sum_order) and one-element
    fp32 entries at K >= 8 per entry; every value, sign of zero included, must equal the per-entry call's."""
    ch = SLQChannel(8)
    g = torch.Generator().manual_seed(k)
    ups = []
    for r in range(k):
        d = {f"b{i}": torch.randn(1 + (i * 37) % 300, generator=g) * 10.0 ** (i % 7 - 3) for i in range(40)}
        d["zeros"] = torch.tensor([-0.0, 0.0, -0.0 if r % 2 else 0.0])
        d["n"] = torch.tensor(3 + r)
        d["big"] = torch.randn(40000, generator=g)    # above torch's grain size (multi-threaded sum)
        d["one"] = torch.randn(1, generator=g)        # torch's inner-sum kernel from K = 8
        d["i64v"] = torch.arange(5, dtype=torch.int64) * (r + 1)
        ups.append(ch.on_client_send(d)[0])
    got, t = ch.receive_mean(ups)
    assert list(got) == list(ups[0].params) and t >= 0
    for name in got:
        want = torch.sum(torch.stack([u.params[name].data for u in ups], dim=0), dim=0) / len(ups)
        assert got[name].dtype == want.dtype and got[name].shape == want.shape, name
        assert torch.equal(got[name], want) and torch.equal(torch.signbit(got[name]), torch.signbit(want)), name
    before = {n: v.clone() for n, v in got.items()}
    got["b0"].add_(1.0)   # each entry owns its storage: writing one leaves the others as they were
    assert all(torch.equal(got[n], before[n]) for n in got if n != "b0")
    assert got["b0"].untyped_storage().nbytes() == got["b0"].numel() * 4


def test_receive_mean_rejects_what_simple_aggregate_rejects():
    ch = SLQChannel(8)
    with pytest.raises(AssertionError):
        ch.receive_mean([])
    with pytest.raises(AssertionError):
        ch.receive_mean([{"b": torch.zeros(2)}])   # not QuantParameters (quant.py:68)


def test_bucket_layout():
    lay = ops.BucketLayout([10, 8192, 8193, 64])
    assert lay.offsets.tolist() == [0, 64, 8256, 16512] and lay.total == 16576
    assert lay.nchunks == 5 and all(o % 64 == 0 for o in lay.offsets)
    compact = ops.BucketLayout([10, 8192, 8193, 64], align=1)
    assert compact.offsets.tolist() == [0, 10, 8202, 16395] and compact.total == 16459
    assert [c.start for c in compact.chunks] == [0, 10, 8202, 16394, 16395]
    lay = ops.BucketLayout(recipes.bucket_sizes("loguniform"))
    assert sum(recipes.bucket_sizes("loguniform")) == recipes.RESNET18_PARAMS
    assert lay.ntensors == 256 and lay.total >= recipes.RESNET18_PARAMS
    assert sum(c.len for c in lay.chunks) == recipes.RESNET18_PARAMS
    with pytest.raises(ValueError):
        ops.BucketLayout([4, 0])
    assert lay.max_tensor_chunks == max(c.nchunks for c in lay.chunks) and lay.nwork == 0  # loguniform: two-pass


def test_encode_mode_selection(monkeypatch):
    """ADFL_SLQ_ENCODE picks the bucketed encode; the product default is 'auto' (resident / two-pass) and a
    bad value fails loudly instead of silently choosing one."""
    monkeypatch.delenv("ADFL_SLQ_ENCODE", raising=False)
    assert ops._encode_mode() == "auto"
    for m in ("auto", "resident", "twopass"):
        monkeypatch.setenv("ADFL_SLQ_ENCODE", m)
        assert ops._encode_mode() == m
    for bad in ("fastest", "coop"):   # the cooperative encode was removed in round 3
        monkeypatch.setenv("ADFL_SLQ_ENCODE", bad)
        with pytest.raises(ValueError, match="ADFL_SLQ_ENCODE"):
            ops._encode_mode()
    monkeypatch.setenv("ADFL_SLQ_ENCODE", "fastest")
    with pytest.raises(ValueError, match="ADFL_SLQ_ENCODE"):
        ops._encode_mode()


def test_oracle_not_imported_by_product_package():
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'ad-federatedlearning_amd'); import adfl_amd, adfl_amd.ops, "
            "adfl_amd.Channel; bad = [m for m in sys.modules if 'oracle' in m or m.startswith('ADFL')]; "
            "assert not bad, bad")
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run([sys.executable, "-c", code], check=True, cwd=repo)


def test_packed_channel_host_rules():
    from adfl_amd.Channel import PackedSLQChannel
    with pytest.raises(ValueError, match="bits"):
        PackedSLQChannel(8)
    assert PackedSLQChannel(4).to_json() == {"name": "PackedSLQChannel", "bits": 4}
    assert PackedSLQChannel(4).simulate_bandwidth(_bw_params(), 1e12) == SLQChannel(4).simulate_bandwidth(
        _bw_params(), 1e12)


@pytest.mark.parametrize("k", [1, 2, 4, 5, 8, 9, 16, 20])
def test_aggregate_entries_matches_simple_aggregate(k):
    """receive_mean's host aggregate of the passthrough entries (biases, counters, running statistics: native
    classification, K concatenated rows, torch's sum order, owned results) equals simple_aggregate
    (Src/ADFL/model.py:221-234) entry by entry, bit for bit: fp32 of every tail shape, int64 counters (-> fp32),
    one-element entries, empty and fp16 entries (per entry through torch)."""
    import torch
    from adfl_amd.Channel import quant
    g = torch.Generator().manual_seed(k)
    names = [f"b{i}" for i in range(40)] + ["cnt", "one", "e", "h"]
    parts = []
    for r in range(k):
        p = {f"b{i}": torch.randn(1 + i * 7, generator=g) for i in range(40)}
        p.update(cnt=torch.tensor(5 + r, dtype=torch.int64), one=torch.randn(1, generator=g), e=torch.empty(0),
                 h=torch.randn(3, generator=g).half())
        parts.append(p)
    got = quant._aggregate_entries(names, parts)
    for n in names:
        want = quant._simple_aggregate([p[n] for p in parts])
        assert got[n].dtype == want.dtype and got[n].shape == want.shape, n
        assert torch.equal(got[n].reshape(-1).view(torch.uint8), want.reshape(-1).view(torch.uint8)), n
