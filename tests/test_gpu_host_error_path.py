"""GPU: a range-pipelined host-to-host channel call that fails part-way — an output allocation
raising while the later ranges' H2D, kernels and D2H are still queued — waits for that device work before the
exception leaves (quant._drain), so the next call, which gathers into the same pinned and device staging
buffers, returns exactly what a call on a clean channel returns.

The failure is injected into the native output-creation call of the second staging range (adfl_torchhost's
empty_qint8_like / empty_f32_like / empty_like_dtype), for SLQ's encode and decode
(quant._encode_host_dict / _decode_host_dict) and QSGD's and CNAT's (stoch._encode_stoch_host /
_decode_stoch_host); the stochastic encodes are seeded through torch's CPU generator as the reference's
rand_like would be.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

from adfl_amd import _torchhost  # noqa: E402
from adfl_amd.Channel.quant import CNATChannel, QSGDChannel, SLQChannel  # noqa: E402


class _Boom(RuntimeError):
    pass


def _params(seed: int):
    """~4.4 M fp32 elements in ragged tensors: eight staging ranges, tensors cut by range edges."""
    g = torch.Generator().manual_seed(seed)
    sizes = [70_000, 3, 300_000, 8192 * 5 + 7, 123_457, 64, 1_000_003, 17] * 3
    p = {f"l{i}.weight": torch.randn(1, n, generator=g) * 1e-3 for i, n in enumerate(sizes)}
    p["l0.bias"] = torch.randn(10, generator=g)
    return p


class _FailOn:
    """Make the native call `name` raise on its `call`-th use inside the block."""

    def __init__(self, name: str, call: int):
        self.mod, self.name, self.call, self.n = _torchhost.get(), name, call, 0

    def __enter__(self):
        self.orig = getattr(self.mod, self.name)

        def f(*a, **k):
            self.n += 1
            if self.n == self.call:
                raise _Boom(self.name)
            return self.orig(*a, **k)

        setattr(self.mod, self.name, f)
        return self

    def __exit__(self, *exc):
        setattr(self.mod, self.name, self.orig)


def _payload_bytes(c):
    out = {}
    for k, p in c.params.items():
        d = p.data
        if d.is_quantized:
            d = d.int_repr()
        s = p.signs if isinstance(p.signs, torch.Tensor) else torch.zeros(1)
        out[k] = (d.clone(), s.clone(), float(p.scale))
    return out


def _same_payload(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k][0], b[k][0]) and torch.equal(a[k][1], b[k][1]), k
        assert a[k][2] == b[k][2] or (a[k][2] != a[k][2] and b[k][2] != b[k][2]), k


def _same_dict(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k].view(-1).view(torch.int32) if a[k].dtype == torch.float32 else a[k],
                           b[k].view(-1).view(torch.int32) if b[k].dtype == torch.float32 else b[k]), k


def _encode(ch, params, seed):
    torch.manual_seed(seed)
    c, _ = ch.on_client_send(params)
    return c


@pytest.mark.parametrize("make,call", [(lambda: SLQChannel(8), "empty_qint8_like"),
                                       (lambda: QSGDChannel(8), "empty_like_dtype"),
                                       (lambda: CNATChannel(8), "empty_like_dtype")])
def test_encode_after_a_failed_encode_is_clean(make, call):
    ch = make()
    p1, p2 = _params(1), _params(2)
    want = _payload_bytes(_encode(ch, p2, 7))            # a clean channel's payload of p2
    with _FailOn(call, 3), pytest.raises(_Boom):
        _encode(ch, p1, 5)                                # fails on the second range's outputs
    got = _payload_bytes(_encode(ch, p2, 7))
    _same_payload(got, want)
    torch.cuda.synchronize()


@pytest.mark.parametrize("make", [lambda: SLQChannel(8), lambda: QSGDChannel(8), lambda: CNATChannel(8)])
def test_decode_after_a_failed_decode_is_clean(make):
    ch = make()
    c1, c2 = _encode(ch, _params(3), 1), _encode(ch, _params(4), 2)
    want, _ = ch.on_server_receive(c2)
    with _FailOn("empty_f32_like", 2), pytest.raises(_Boom):
        ch.on_server_receive(c1)                          # fails on the second range's outputs
    got, _ = ch.on_server_receive(c2)
    _same_dict(got, want)
    torch.cuda.synchronize()
