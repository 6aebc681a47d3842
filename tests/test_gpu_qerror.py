"""GPU: the reference's q-error metrics on the device (csrc/qerror_ref.hip through adfl_qerror_ref, the
norms through adfl_torch_norms), bit for bit:

* SLQChannel(bits).send_with_q_error == the reference's doubles on the ResNet-18-sized and grain-edge dicts
  of tests/golden/qerror_manifest.json (the reference executed in place) at 1 / 3 / 8 / 16 threads; the
  small dicts of aggregate_manifest.json are in test_gpu_aggregate_golden.py;
* qerror.reference_sums == torch.sum((x - d) ** 2), torch.sum(x ** 2) per tensor and the cosine's sum,
  computed by torch itself on this box's CPU, for random dicts with every branch of the order (tensors of
  1..7 elements, the 32,768 grain, the level steps, NaN / inf / zeros) at several thread counts;
* PackedSLQChannel (int4 buckets, padded layout) against the oracle restatement on its own decode.
"""

import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from conftest import GOLDEN  # noqa: E402

import make_golden_qerror as mgq  # noqa: E402
import recipes  # noqa: E402
import slq_oracle as so  # noqa: E402

from adfl_amd import qerror  # noqa: E402
from adfl_amd.Channel import PackedSLQChannel, SLQChannel  # noqa: E402

DEV = torch.device("cuda", 0)


def _same(a, b):
    return (np.isnan(a) and np.isnan(b)) or a == b


def _threads(t):
    class _T:
        def __enter__(self):
            self.old = torch.get_num_threads()
            torch.set_num_threads(t)

        def __exit__(self, *a):
            torch.set_num_threads(self.old)
    return _T()


@pytest.mark.parametrize("name", ["edges", "resnet18"])
def test_send_with_q_error_equals_reference_model_sizes(name):
    m = json.load(open(os.path.join(GOLDEN, "qerror_manifest.json")))
    e = m["dicts"][name]
    spec = mgq.dicts()[name]
    params = {}
    for i, (n, s, mult) in enumerate(spec):
        x = recipes.randn(s, e["seed0"] + i, mult)
        assert recipes.sha256(x) == e["sha256"][n]
        params[n] = torch.from_numpy(x)
    for bits in mgq.BITS:
        ch = SLQChannel(bits)
        for t in mgq.THREADS:
            with _threads(t):
                _, _, mse, cos = ch.send_with_q_error(params)
            ref = e["metrics"][f"slq{bits}_t{t}"]
            assert mse == float(ref["mse"]) and cos == float(ref["cos"]), (name, bits, t, mse, cos, ref)


@pytest.mark.parametrize("name", ["edges", "resnet18"])
def test_worker_q_error_call_sequence_with_dropin_metrics(name):
    """Src/ADFL/Client/worker.py:176,186-189 unchanged except for where the two metric functions come from
    (adfl_amd.model's device drop-ins for ADFL.model's): on_client_send, then
    on_server_receive of the payload, then parameter_relative_mse / parameter_cosine_similarity(exclude_bias=True)
    == the reference's doubles (the reference executed in place, tests/golden/qerror_manifest.json)."""
    from adfl_amd import model as am
    m = json.load(open(os.path.join(GOLDEN, "qerror_manifest.json")))
    e = m["dicts"][name]
    spec = mgq.dicts()[name]
    params = {}
    for i, (n, s, mult) in enumerate(spec):
        params[n] = torch.from_numpy(recipes.randn(s, e["seed0"] + i, mult))
    for bits in mgq.BITS:
        ch = SLQChannel(bits)
        for t in (1, 8):
            with _threads(t):
                c_params, _ = ch.on_client_send(params)
                d_params, _ = ch.on_server_receive(c_params)
                mse = am.parameter_relative_mse(params, d_params, exclude_bias=True)
                cos = am.parameter_cosine_similarity(params, d_params, exclude_bias=True)
            ref = e["metrics"][f"slq{bits}_t{t}"]
            assert mse == float(ref["mse"]) and cos == float(ref["cos"]), (name, bits, t, mse, cos, ref)


def test_dropin_metrics_with_biases_and_errors():
    """exclude_bias=False counts the 1-D entries too; an empty selection gives 0.0 / the cat error; key and shape
    mismatches raise the reference's AssertionError (model.py:266-277, :303-312)."""
    from adfl_amd import model as am
    g = torch.Generator().manual_seed(3)
    a = {"w": torch.randn(40, 33, generator=g), "b": torch.randn(40, generator=g), "n": torch.randn(70001, 1, generator=g)}
    b = {k: v + torch.randn(v.shape, generator=g) * 1e-2 for k, v in a.items()}
    for eb in (True, False):
        keep = [k for k in a if not eb or a[k].ndim > 1]
        num = sum(torch.sum((a[k] - b[k]) ** 2).item() for k in keep) / sum(a[k].numel() for k in keep)
        den = sum(torch.sum((a[k] - 0) ** 2).item() for k in keep) / sum(a[k].numel() for k in keep)
        cos = F.cosine_similarity(torch.cat([a[k].flatten() for k in keep]), torch.cat([b[k].flatten() for k in keep]),
                                  dim=0).item()
        assert am.parameter_relative_mse(a, b, eb) == num / den
        assert am.parameter_cosine_similarity(a, b, eb) == cos
    only_bias = {"b": a["b"]}
    assert am.parameter_relative_mse(only_bias, {"b": b["b"]}, True) == 0.0
    with pytest.raises(RuntimeError):
        am.parameter_cosine_similarity(only_bias, {"b": b["b"]}, True)
    with pytest.raises(AssertionError):
        am.parameter_relative_mse(a, {"w": b["w"]}, True)


def _torch_sums(xs, ds, t):
    """What model.py:256-323 reduces, by torch itself on the CPU with t threads."""
    with _threads(t):
        e = [torch.sum((torch.from_numpy(x) - torch.from_numpy(d)) ** 2).item() for x, d in zip(xs, ds)]
        s = [torch.sum((torch.from_numpy(x) - 0) ** 2).item() for x in xs]
        va = torch.cat([torch.from_numpy(x) for x in xs])
        vb = torch.cat([torch.from_numpy(d) for d in ds])
        c = F.cosine_similarity(va, vb, dim=0).item()
    return e, s, c


def _dict(rng, sizes, kind):
    xs, ds = [], []
    for n in sizes:
        x = (rng.standard_normal(n) * np.exp2(rng.integers(-6, 6))).astype(np.float32)
        d = (x + rng.standard_normal(n).astype(np.float32) * np.float32(1e-2) * np.abs(x)).astype(np.float32)
        if kind == "special" and n > 3:
            x[rng.integers(0, n)] = np.inf if n % 2 else np.nan
        if kind == "zeros":
            x[:] = 0.0
            d[:] = 0.0
        xs.append(x)
        ds.append(d)
    return xs, ds


@pytest.mark.parametrize("kind", ["randn", "special", "zeros"])
@pytest.mark.parametrize("threads", [1, 2, 7, 8, 16])
def test_reference_sums_equal_torch(threads, kind):
    rng = np.random.default_rng(threads * 10 + len(kind))
    sizes = [1, 2, 3, 5, 7, 8, 9, 31, 33, 100, 4097, 8192, 8193, 32767, 32768, 32769, 65536, 70001, 131073,
             262145, 600_007]
    xs, ds = _dict(rng, sizes, kind)
    x = torch.from_numpy(np.concatenate(xs)).to(DEV)
    d = torch.from_numpy(np.concatenate(ds)).to(DEV)
    e, s, c = qerror.reference_sums(x, d, sizes, threads=threads)
    we, ws, wc = _torch_sums(xs, ds, threads)
    for t in range(len(sizes)):
        assert _same(float(e[t]), we[t]) and _same(float(s[t]), ws[t]), (threads, kind, sizes[t], e[t], we[t], s[t], ws[t])
    assert _same(c, wc), (threads, kind, c, wc)


def test_reference_sums_large_single_tensor():
    """One 2^25 + 3 element tensor: level step 32 in every range at 1 thread, two-pass at 16."""
    n = (1 << 25) + 3
    g = torch.Generator().manual_seed(3)
    xc = torch.randn(n, generator=g) * 1e-2
    dc = xc + torch.randn(n, generator=g) * 1e-4
    x, d = xc.to(DEV), dc.to(DEV)
    for t in (1, 16):
        e, s, c = qerror.reference_sums(x, d, [n], threads=t)
        we, ws, wc = _torch_sums([xc.numpy()], [dc.numpy()], t)
        assert float(e[0]) == we[0] and float(s[0]) == ws[0] and c == wc, (t, e, we, s, ws, c, wc)


def test_packed_channel_metrics_equal_oracle_on_its_decode():
    rng = np.random.default_rng(11)
    params = {f"w{i}": torch.from_numpy((rng.standard_normal((3, n)) * 1e-2).astype(np.float32))
              for i, n in enumerate((5, 1001, 12_289, 40_001))}
    ch = PackedSLQChannel(4)
    for t in (1, 8):
        with _threads(t):
            cp, _, mse, cos = ch.send_with_q_error(params)
            dec, _ = ch.on_server_receive(cp)
        xs = [params[k].numpy() for k in params]
        ds = [dec[k].numpy() for k in params]
        wm, wc = so.qerror_metrics(xs, ds, t)
        assert mse == wm and cos == wc, (t, mse, wm, cos, wc)
