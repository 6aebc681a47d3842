"""GPU: the drop-in Channel surface (SLQChannel / USLQChannel) against the reference's golden output.

Mirrors the reference's own codec test flow (Src/ADFL/Channel/Tests/test_quant.py:126-161: server->client
and client->server round trips) but asserts values instead of printing them."""

import pickle

import numpy as np
import pytest
import torch

import recipes
from golden_util import manifest, same_f32, same_scale, small

pytestmark = pytest.mark.gpu

adfl_amd = pytest.importorskip("adfl_amd")
from adfl_amd.Channel import SLQChannel, USLQChannel  # noqa: E402
from adfl_amd.model import ByteParameters, QuantParameters  # noqa: E402


def _golden_dict(names):
    A = small()
    return {n: torch.from_numpy(A[n + "__x"].copy()) for n in names}


def test_c1_two_client_round_trip_matches_golden():
    """C1 shape (Examples/ray_async.py:63-70): [10,3072] weight + [10] bias, both directions."""
    m = {c["name"]: c for c in manifest()["raw"]}
    A = small()
    w = torch.from_numpy(A["c1_fc_weight_b8__x"].copy())
    b = torch.from_numpy(recipes.randn((10,), 31, 1.0))
    ch = SLQChannel(bits=8)
    for send, recv in ((ch.on_server_send, ch.on_client_receive), (ch.on_client_send, ch.on_server_receive)):
        qp, t_enc = send({"fc.weight": w, "fc.bias": b})
        assert isinstance(qp, QuantParameters) and t_enc > 0
        p = qp.params["fc.weight"]
        assert p.data.dtype == torch.qint8 and p.data.device.type == "cpu"
        assert np.array_equal(p.data.int_repr().numpy(), A["c1_fc_weight_b8__q"])
        assert isinstance(p.scale, float) and same_scale(p.scale, m["c1_fc_weight_b8"]["scale_bits"])
        assert p.data.q_scale() == p.scale and p.data.q_zero_point() == 0
        assert qp.params["fc.bias"].data is b and qp.params["fc.bias"].scale == 1
        assert qp.size == m["c1_fc_weight_b8"]["size"] + b.nbytes
        dec, t_dec = recv(qp)
        assert same_f32(dec["fc.weight"].numpy(), A["c1_fc_weight_b8__deq"])
        assert dec["fc.weight"].dtype == torch.float32 and dec["fc.weight"].shape == w.shape
        dec["fc.weight"].add_(1.0)  # owned and writable, as strategies require
        assert dec["fc.bias"].data_ptr() == b.data_ptr()


@pytest.mark.parametrize("bits", [8, 4, 2])
def test_whole_dict_of_golden_cases(bits):
    """Every small golden case of this bit width in ONE dict -> one bucketed launch per pass."""
    cases = [c for g in ("raw", "edge") for c in manifest()[g] if c["bits"] == bits]
    A = small()
    params = {c["name"]: torch.from_numpy(A[c["name"] + "__x"].copy()) for c in cases}
    params["bias"] = torch.randn(7)
    params["num_batches_tracked"] = torch.tensor(3, dtype=torch.int64)
    ch = SLQChannel(bits=bits)
    qp, _ = ch.on_client_send(params)
    dec, _ = ch.on_server_receive(qp)
    assert list(qp.params) == list(params) and list(dec) == list(params)
    for c in cases:
        p = qp.params[c["name"]]
        assert np.array_equal(p.data.int_repr().numpy(), A[c["name"] + "__q"]), c["name"]
        assert same_scale(p.scale, c["scale_bits"]), c["name"]
        assert same_f32(dec[c["name"]].numpy(), A[c["name"] + "__deq"]), c["name"]
    assert qp.params["num_batches_tracked"].data is params["num_batches_tracked"]


def test_passthrough_metadata_matches_reference():
    g = manifest()["passthrough"]
    bias = torch.from_numpy(recipes.randn((10,), 31, 1.0))
    nbt = torch.tensor(7, dtype=torch.int64)
    ivec = torch.arange(5, dtype=torch.int64)
    qp, _ = SLQChannel(8).on_client_send({"bias": bias, "num_batches_tracked": nbt, "ivec": ivec})
    for (name, p), src in zip(qp.params.items(), (bias, nbt, ivec)):
        ref = g[name]
        assert (p.data is src) == ref["same_object"]
        assert p.scale == ref["scale"] and type(p.scale).__name__ == ref["scale_type"]
        assert str(p.dtype) == ref["dtype"] and str(p.q_dtype) == ref["q_dtype"]
        assert list(p.shape) == ref["shape"] and p.bits == ref["bits"]
        assert p.signs.tolist() == ref["signs"] and str(p.signs.dtype) == ref["signs_dtype"]
    assert qp.size == g["__size__"]
    meta = manifest()["quant_meta"]
    w = SLQChannel(8).on_client_send({"w": torch.ones(2, 3)})[0].params["w"]
    assert str(w.q_dtype) == meta["q_dtype"] and str(w.data.dtype) == meta["data_dtype"]
    assert w.scale_2 == meta["scale_2"] and type(w.scale).__name__ == meta["scale_type"]


def test_uslq_directions():
    params = {"w": torch.randn(33, 31), "b": torch.randn(31)}
    ch = USLQChannel(bits=8)
    bp, t = ch.on_server_send(params)
    assert isinstance(bp, ByteParameters) and t == 0.0
    back, _ = ch.on_client_receive(bp)
    assert torch.equal(back["w"], params["w"])
    qp, _ = ch.on_client_send(params)
    assert isinstance(qp, QuantParameters)
    dec, _ = ch.on_server_receive(qp)
    assert dec["w"].shape == (33, 31)
    assert ch.to_json() == manifest()["to_json"]["USLQChannel_4"] | {"bits": 8}


def test_device_resident_dict_stays_on_device():
    dev = torch.device("cuda", 0)
    x = torch.randn(257, 129, device=dev)
    qp, _ = SLQChannel(8).on_client_send({"w": x, "cpu_w": x.cpu()})
    assert qp.params["w"].data.is_cuda and not qp.params["cpu_w"].data.is_cuda
    assert torch.equal(qp.params["w"].data.int_repr().cpu(), qp.params["cpu_w"].data.int_repr())
    assert qp.params["w"].scale == qp.params["cpu_w"].scale
    dec, _ = SLQChannel(8).on_server_receive(qp)
    assert dec["w"].is_cuda and torch.equal(dec["w"].cpu(), dec["cpu_w"])


def test_all_device_dict_and_c3_loguniform_vs_golden():
    """C3 (loguniform layout) as a CUDA-resident state dict through the Channel: golden scales and SHA."""
    case = [c for c in manifest()["bucket"] if c["layout"] == "loguniform"][0]
    tensors = recipes.bucket_tensors(case["layout"], case["seed"], case["mult"])
    params = {k: torch.from_numpy(v).cuda() for k, v in tensors.items()}
    qp, _ = SLQChannel(8).on_client_send(params)
    dec, _ = SLQChannel(8).on_server_receive(qp)
    names = list(params)
    assert all(qp.params[k].data.is_cuda and dec[k].is_cuda for k in names)
    for k, b in zip(names, case["scale_bits"]):
        assert same_scale(qp.params[k].scale, b), k
    q_cat = np.concatenate([qp.params[k].data.int_repr().cpu().numpy().reshape(-1) for k in names])
    d_cat = np.concatenate([dec[k].cpu().numpy().reshape(-1) for k in names])
    assert recipes.sha256(q_cat) == case["q_sha256"]
    assert recipes.sha256(d_cat) == case["deq_sha256"]


def test_results_survive_later_calls():
    """Staging buffers are reused between calls; returned payloads and decoded tensors must not be."""
    ch = SLQChannel(8)
    a = {"w": torch.randn(300, 41), "v": torch.randn(7, 3)}
    b = {"w": torch.randn(300, 41) * 5, "v": torch.randn(7, 3) * 5}
    qa, _ = ch.on_client_send(a)
    qa_bytes = {k: p.data.int_repr().clone() for k, p in qa.params.items()}
    da, _ = ch.on_server_receive(qa)
    da_copy = {k: v.clone() for k, v in da.items()}
    qb, _ = ch.on_client_send(b)
    db, _ = ch.on_server_receive(qb)
    for k in a:
        assert torch.equal(qa.params[k].data.int_repr(), qa_bytes[k])
        assert torch.equal(da[k], da_copy[k])
        assert not torch.equal(da[k], db[k])
    da["w"].mul_(2.0)  # writable; does not touch the other decoded tensors
    assert torch.equal(da["v"], da_copy["v"])


def test_concurrent_threads_share_one_device_safely():
    """ADFL's peer clients decode on a receive thread while the training thread encodes
    (Examples/ray_ad.py): the per-device staging is serialised, results stay exact."""
    import threading
    import slq_oracle as oracle
    ch = SLQChannel(8)
    errors = []

    def work(seed):
        try:
            g = torch.Generator().manual_seed(seed)
            params = {f"w{i}": torch.randn(64 + seed, 33 + i, generator=g) * (seed + 1) for i in range(5)}
            for _ in range(5):
                qp, _ = ch.on_client_send(params)
                dec, _ = ch.on_server_receive(qp)
                for k, v in params.items():
                    q_ref, s_ref = oracle.encode(v.numpy(), 8)
                    assert np.array_equal(qp.params[k].data.int_repr().numpy(), q_ref)
                    assert same_f32(dec[k].numpy(), oracle.decode(q_ref, s_ref))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors


def test_send_with_q_error_matches_reference_metrics():
    """worker.py:176,186-189 in one call: payload identical to on_client_send, metrics equal to the
    reference's parameter_relative_mse / parameter_cosine_similarity (exclude_bias=True) computed on
    the decoded dict (restated here exactly as Src/ADFL/model.py:256-323 computes them)."""
    g = torch.Generator().manual_seed(3)
    params = {f"w{i}": torch.randn(50 + 17 * i, 31, generator=g) * 10.0 ** (-i) for i in range(6)}
    params["bias"] = torch.randn(31, generator=g)
    ch = SLQChannel(8)
    qp, c_time, mse, cos = ch.send_with_q_error(params)
    qp2, _ = ch.on_client_send(params)
    for k in params:
        a, b = qp.params[k].data, qp2.params[k].data
        assert torch.equal(a.int_repr(), b.int_repr()) if a.is_quantized else a is b
    dec, _ = ch.on_server_receive(qp)
    keys = [k for k in params if params[k].ndim > 1]
    count = sum(params[k].numel() for k in keys)
    num = sum(torch.sum((params[k] - dec[k]) ** 2).item() for k in keys) / count
    den = sum(torch.sum((params[k] - torch.zeros_like(params[k])) ** 2).item() for k in keys) / count
    ref_cos = torch.nn.functional.cosine_similarity(torch.cat([params[k].flatten() for k in keys]),
                                                    torch.cat([dec[k].flatten() for k in keys]), dim=0).item()
    assert mse == num / den and cos == ref_cos  # model.py:256-323's doubles, bit for bit
    assert c_time > 0


def test_channel_pickles_without_device_state():
    ch = SLQChannel(8)
    SLQChannel(8).on_client_send({"w": torch.randn(4, 4)})  # warm the per-process cache
    ch2 = pickle.loads(pickle.dumps(ch))
    assert ch2.bits == 8 and vars(ch2) == {"bits": 8}


def test_payload_pickles_compactly():
    """Ray pickles the payload; each tensor owns its storage (no shared staging buffer rides along)."""
    qp, _ = SLQChannel(8).on_client_send({"a": torch.randn(64, 64), "b": torch.randn(4096, 16)})
    blob = pickle.dumps(qp.params["a"])
    assert len(blob) < 64 * 64 + 2048


def test_reference_errors():
    ch = SLQChannel(8)
    with pytest.raises(RuntimeError, match="Quantize only works on Float Tensor, got Double"):
        ch.on_client_send({"w": torch.randn(2, 2, dtype=torch.float64)})
    with pytest.raises(RuntimeError, match="Quantize only works on Float Tensor, got Long"):
        ch.on_client_send({"w": torch.ones(2, 2, dtype=torch.int64)})
    with pytest.raises(RuntimeError, match="numel\\(\\) == 0"):
        ch.on_client_send({"w": torch.empty(0, 3)})
    with pytest.raises(AssertionError):
        ch.on_server_receive(ByteParameters({}, 0))


@pytest.mark.parametrize("bits", [4, 2])
def test_packed_channel_vs_golden(bits):
    """PackedSLQChannel: every golden case of this width in one dict; payload = pack_4bit(reference SLQ
    payload) (the reference's own layout functions, pinned by tests/golden/int4.npz), decode = unpack +
    dequantize, half the bytes of SLQChannel's payload."""
    import slq_oracle as oracle
    from adfl_amd.Channel import PackedSLQChannel
    cases = [c for g in ("raw", "edge") for c in manifest()[g] if c["bits"] == bits]
    A = small()
    params = {c["name"]: torch.from_numpy(A[c["name"] + "__x"].copy()) for c in cases}
    params["bias"] = torch.randn(9)
    ch = PackedSLQChannel(bits)
    qp, _ = ch.on_client_send(params)
    dec, _ = ch.on_server_receive(qp)
    total = 0
    for c in cases:
        p = qp.params[c["name"]]
        q_ref = A[c["name"] + "__q"]
        p_ref = oracle.pack_int4(q_ref)
        assert p.data.dtype == torch.int8 and p.data.ndim == 1 and p.q_dtype == torch.int8
        assert tuple(p.shape) == q_ref.shape and p.dtype == torch.float32 and p.bits == bits
        assert np.array_equal(p.data.numpy().view(np.uint8), p_ref), c["name"]
        assert same_scale(p.scale, c["scale_bits"])
        assert same_f32(dec[c["name"]].numpy(), oracle.decode_int4(p_ref, q_ref.size, p.scale)), c["name"]
        total += p.data.nbytes
    assert qp.params["bias"].data is params["bias"]
    assert qp.size == total + params["bias"].nbytes
    assert ch.to_json() == {"name": "PackedSLQChannel", "bits": bits}
    blob = len(pickle.dumps(qp.params[cases[0]["name"]]))
    assert blob < qp.params[cases[0]["name"]].data.nbytes + 2048


def test_packed_channel_device_dict():
    from adfl_amd.Channel import PackedSLQChannel
    x = torch.randn(333, 77, device="cuda")
    qp, _ = PackedSLQChannel(4).on_client_send({"w": x, "b": torch.randn(5, device="cuda")})
    assert qp.params["w"].data.is_cuda and qp.params["w"].data.numel() == (333 * 77 + 1) // 2
    dec, _ = PackedSLQChannel(4).on_server_receive(qp)
    ref, _ = SLQChannel(4).on_server_receive(SLQChannel(4).on_client_send({"w": x.cpu()})[0])
    assert torch.equal(dec["w"].cpu(), ref["w"])  # values in [-7, 7]: packing is lossless vs int8 SLQ


def test_packed_send_with_q_error():
    """PackedSLQChannel.send_with_q_error (inherited surface): payload identical to on_client_send, metrics
    equal to the reference's formulas on the packed channel's own decode (model.py:256-323)."""
    from adfl_amd.Channel import PackedSLQChannel
    g = torch.Generator().manual_seed(4)
    params = {f"w{i}": torch.randn(33 + 13 * i, 17, generator=g) * 10.0 ** (-i) for i in range(5)}
    params["w_odd"] = torch.randn(3, 7, generator=g)       # odd element count: the zero-padded last byte
    params["bias"] = torch.randn(17, generator=g)
    ch = PackedSLQChannel(4)
    qp, c_time, mse, cos = ch.send_with_q_error(params)
    qp2, _ = ch.on_client_send(params)
    for k in params:
        a, b = qp.params[k].data, qp2.params[k].data
        assert torch.equal(a, b) if params[k].ndim > 1 else a is b
    dec, _ = ch.on_server_receive(qp)
    keys = [k for k in params if params[k].ndim > 1]
    count = sum(params[k].numel() for k in keys)
    num = sum(torch.sum((params[k] - dec[k]) ** 2).item() for k in keys) / count
    den = sum(torch.sum((params[k] - torch.zeros_like(params[k])) ** 2).item() for k in keys) / count
    ref_cos = torch.nn.functional.cosine_similarity(torch.cat([params[k].flatten() for k in keys]),
                                                    torch.cat([dec[k].flatten() for k in keys]), dim=0).item()
    assert mse == num / den and cos == ref_cos
    assert c_time > 0


@pytest.mark.parametrize("channel", ["SLQChannel", "PackedSLQChannel", "QSGDChannel", "CNATChannel"])
def test_decoded_tensors_are_independently_owned(channel):
    """Decode hands back one owned tensor per entry, as the reference does (quant.py:107-112): no views of
    a shared bucket, so keeping one update (FedBuff, Src/ADFL/Strategy/fed_buff.py:75,90) keeps only its
    own bytes alive and pickling one tensor ships only that tensor. Encode payloads likewise."""
    import importlib
    C = importlib.import_module("adfl_amd.Channel")
    ch = getattr(C, channel)(4 if channel == "PackedSLQChannel" else 8)
    g = torch.Generator().manual_seed(5)
    params = {f"w{i}": torch.randn(256, 64 + i, generator=g) for i in range(6)}
    params["b"] = torch.randn(64, generator=g)
    qp, _ = ch.on_client_send(params)
    dec, _ = ch.on_server_receive(qp)
    for k in params:
        if params[k].ndim <= 1:
            continue
        t = dec[k]
        assert not t.is_pinned() and t.is_contiguous() and t.dtype == torch.float32
        assert t.untyped_storage().nbytes() == t.nbytes, k
        assert len(pickle.dumps(t)) < t.nbytes + 2048, k
        d = qp.params[k].data
        assert d.untyped_storage().nbytes() == d.nbytes, k
    ptrs = sorted(dec[k].data_ptr() for k in params if params[k].ndim > 1)
    assert len(set(ptrs)) == len(ptrs)
    # a second call must not alias or overwrite the first call's outputs
    before = {k: dec[k].clone() for k in dec}
    ch.on_server_receive(ch.on_client_send({k: v * 3 for k, v in params.items()})[0])
    for k in dec:
        assert torch.equal(dec[k], before[k]), k
