"""SLQ channels backed by the MI355X HIP codec — drop-in for ``Src/ADFL/Channel/quant.py:15-137``.

``SLQChannel`` / ``USLQChannel`` keep the reference's names, constructor, six-method surface,
``to_json`` output, ``simulate_bandwidth`` formula, payload types and error behaviour. What changes is
where the arithmetic runs: the reference loops over the state dict calling ATen CPU ops per tensor
(quant.py:74-112); here the whole dict is bucketed into one 64-element-aligned flat buffer, moved to
the GPU once, encoded by two HIP launches (absmax partials -> scale + quantize, per-tensor scales),
and the int8 payload comes back in one copy. Decode is one HIP launch. Output is bit-identical to the
reference: int8 payload, fp32 scale and dequantized floats (tests/golden).

Contract kept from the reference:
* inputs are CPU tensors (callers ``.cpu()``, Src/ADFL/model.py:195-197) — CUDA tensors are also
  accepted and then stay on the device;
* ``ndim <= 1`` tensors pass through untouched with ``scale = 1`` (quant.py:80-81, same object);
* ``QuantParameter.data`` is a ``torch.qint8`` tensor (zero point 0) and ``scale`` a Python float;
* decode returns new, owned, writable fp32 tensors (strategies mutate them in place);
* a non-fp32 ``ndim > 1`` tensor raises ``RuntimeError: Quantize only works on Float Tensor, got …``;
  an empty one raises torch.max's ``RuntimeError``; ``_receive`` asserts ``QuantParameters``;
* the channel object holds no device state (it is pickled into every Ray actor): buffers live in a
  per-process, per-device cache created lazily on first use.

There is no CPU fallback: without a GPU and the built HIP library these methods raise.
"""

import time
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

from .. import ops
from ..model import (CompressedParameters, Parameters, QuantParameter, QuantParameters, get_parameter_info)
from .channel import Channel, IdentityChannel

_LAYOUT_CACHE_MAX = 16


class _DeviceStaging:
    """Per-process, per-device reusable buffers (pinned host + device), grown on demand."""

    def __init__(self, device: torch.device):
        self.device = device
        self._bufs: Dict[str, torch.Tensor] = {}
        self.layouts: "OrderedDict[Tuple[int, ...], ops.BucketLayout]" = OrderedDict()

    def buf(self, key: str, numel: int, dtype: torch.dtype, pinned: bool = False) -> torch.Tensor:
        t = self._bufs.get(key)
        if t is None or t.numel() < numel:
            numel = max(numel, 1)
            if pinned:
                t = torch.empty(numel, dtype=dtype, pin_memory=True)
            else:
                t = torch.empty(numel, dtype=dtype, device=self.device)
            self._bufs[key] = t
        return t[:numel]

    def layout(self, sizes: Tuple[int, ...]) -> ops.BucketLayout:
        lay = self.layouts.get(sizes)
        if lay is None:
            lay = ops.BucketLayout(sizes)
            self.layouts[sizes] = lay
            if len(self.layouts) > _LAYOUT_CACHE_MAX:
                self.layouts.popitem(last=False)
        else:
            self.layouts.move_to_end(sizes)
        return lay


_STAGING: Dict[int, _DeviceStaging] = {}


def _staging() -> _DeviceStaging:
    idx = torch.cuda.current_device()
    st = _STAGING.get(idx)
    if st is None:
        st = _DeviceStaging(torch.device("cuda", idx))
        _STAGING[idx] = st
    return st


def _encode_dict(params: Parameters, names: List[str], bits: int):
    """Encode the ndim>1 tensors `names` of `params` in one bucketed pass.

    Returns {name: (qint8 tensor on the input's device, python float scale)}."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    sizes = tuple(int(t.numel()) for t in tensors)
    lay = st.layout(sizes)
    x_dev = st.buf("x", lay.total, torch.float32)
    on_cpu = [not t.is_cuda for t in tensors]
    if any(on_cpu):
        x_host = st.buf("x_host", lay.total, torch.float32, pinned=True)
        for t, off, n, cpu in zip(tensors, lay.offsets, lay.sizes, on_cpu):
            if cpu:
                x_host[int(off):int(off) + int(n)].view(t.shape).copy_(t)
        x_dev.copy_(x_host, non_blocking=True)  # one H2D for the whole bucket
    for t, off, n, cpu in zip(tensors, lay.offsets, lay.sizes, on_cpu):
        if not cpu:  # after the H2D, which would overwrite these slices
            x_dev[int(off):int(off) + int(n)].view(t.shape).copy_(t)
    q_dev, s_dev = ops.encode_batched(x_dev, lay, bits, q=st.buf("q", lay.total, torch.int8),
                                      scales=st.buf("scales", lay.ntensors, torch.float32),
                                      partials=st.buf("partials", lay.nchunks, torch.int32))
    scales_host = st.buf("scales_host", lay.ntensors, torch.float32, pinned=True)
    scales_host.copy_(s_dev, non_blocking=True)
    if any(on_cpu):
        q_host = st.buf("q_host", lay.total, torch.int8, pinned=True)
        q_host.copy_(q_dev, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    out = {}
    for i, (name, t, off, n, cpu) in enumerate(zip(names, tensors, lay.offsets, lay.sizes, on_cpu)):
        scale = float(scales_host[i])
        src = (q_host if cpu else q_dev)[int(off):int(off) + int(n)]
        qt = torch._make_per_tensor_quantized_tensor(src.clone().view(t.shape), scale, 0)
        out[name] = (qt, scale)
    return out


def _decode_dict(items: List[Tuple[str, torch.Tensor]]) -> Dict[str, torch.Tensor]:
    """Decode qint8 tensors (per-tensor affine, zero point 0) in one bucketed pass."""
    st = _staging()
    dev = st.device
    sizes = tuple(int(q.numel()) for _, q in items)
    lay = st.layout(sizes)
    on_cpu = [not q.is_cuda for _, q in items]
    q_dev = st.buf("dq", lay.total, torch.int8)
    if any(on_cpu):
        q_host = st.buf("dq_host", lay.total, torch.int8, pinned=True)
    scales_host = st.buf("dscales_host", lay.ntensors, torch.float32, pinned=True)
    for i, ((name, q), off, n, cpu) in enumerate(zip(items, lay.offsets, lay.sizes, on_cpu)):
        if q.qscheme() != torch.per_tensor_affine or q.dtype != torch.qint8 or q.q_zero_point() != 0:
            raise ValueError(f"SLQChannel: '{name}' is not a per-tensor qint8 payload with zero point 0")
        scales_host[i] = q.q_scale()  # rounds to the fp32 scale fbgemm's dequantize uses
        if cpu:
            q_host[int(off):int(off) + int(n)].view(q.shape).copy_(q.int_repr())
    if any(on_cpu):
        q_dev.copy_(q_host, non_blocking=True)  # one H2D for the whole bucket
    for (name, q), off, n, cpu in zip(items, lay.offsets, lay.sizes, on_cpu):
        if not cpu:
            q_dev[int(off):int(off) + int(n)].view(q.shape).copy_(q.int_repr())
    s_dev = st.buf("dscales", lay.ntensors, torch.float32)
    s_dev.copy_(scales_host, non_blocking=True)
    out_dev = ops.decode_batched(q_dev, s_dev, lay, out=st.buf("dout", lay.total, torch.float32))
    if any(on_cpu):
        out_host = st.buf("dout_host", lay.total, torch.float32, pinned=True)
        out_host.copy_(out_dev, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    res = {}
    for (name, q), off, n, cpu in zip(items, lay.offsets, lay.sizes, on_cpu):
        src = (out_host if cpu else out_dev)[int(off):int(off) + int(n)]
        res[name] = src.clone().view(q.shape)  # owned and writable (strategies mutate in place)
    return res


class SLQChannel(Channel):
    """Bi-directional symmetric linear quantization (quant.py:15-112) on the MI355X HIP codec."""

    def __init__(self, bits: int) -> None:
        self.bits = bits

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return self._send(params)

    def on_server_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return self._receive(c_params)

    def on_client_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return self._send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return self._receive(c_params)

    def to_json(self) -> Dict:
        return {"name": self.__class__.__name__, "bits": self.bits}

    def simulate_bandwidth(self, params: Parameters, mbps: float) -> float:
        """self.bits for weights, 32 bits for biases, 32 bits per scale (quant.py:47-58)."""
        p_info = get_parameter_info(params)
        num_bytes = p_info.num_non_bias_w * self.bits / 8
        num_bytes += p_info.num_bias_w * 4
        num_bytes += p_info.num_non_bias_t * 4
        transfer_time = num_bytes / (mbps * 1_000_000 / 8)
        time.sleep(transfer_time)
        return transfer_time

    def _send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        s_time = time.perf_counter()
        q_params = self._quantize_params(params, self.bits)
        return q_params, time.perf_counter() - s_time

    def _receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        assert isinstance(c_params, QuantParameters)
        s_time = time.perf_counter()
        quant = [(name, p.data) for name, p in c_params.params.items() if p.data.ndim > 1 and p.data.is_quantized]
        decoded = _decode_dict(quant) if quant else {}
        params = {}
        for name, p in c_params.params.items():
            if name in decoded:
                params[name] = decoded[name]
            elif p.data.ndim > 1:
                params[name] = p.data.data.dequantize()  # non-quantized payload: what quant.py:110 does
            else:
                params[name] = p.data.data  # passthrough (quant.py:111-112)
        return params, time.perf_counter() - s_time

    def _quantize_params(self, params: Parameters, bits: int) -> QuantParameters:
        """Biases and running metrics (ndim <= 1) are not quantized (quant.py:74-94)."""
        names = [name for name, p in params.items() if p.ndim > 1]
        for name in names:
            ops.require_quantizable(params[name])
        encoded = _encode_dict(params, names, bits) if names else {}
        q_params = QuantParameters({}, 0)
        for name, param in params.items():
            if name in encoded:
                q_param, scale = encoded[name]
            else:
                q_param, scale = param, 1
            q_params.params[name] = QuantParameter(
                data=q_param, bits=bits, scale=scale, signs=torch.zeros(1, dtype=torch.uint8),
                shape=param.shape, dtype=param.dtype, q_dtype=q_param.dtype)
            q_params.size += q_param.nbytes
        return q_params


class USLQChannel(SLQChannel):
    """Uni-directional SLQ (quant.py:115-137): only client -> server is quantized."""

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return IdentityChannel(no_compute_time=True).on_server_send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return IdentityChannel(no_compute_time=True).on_client_receive(c_params)

    def to_json(self) -> Dict:
        return {"name": self.__class__.__name__, "bits": self.bits}


HipSLQChannel = SLQChannel
HipUSLQChannel = USLQChannel
