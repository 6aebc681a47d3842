"""Payload types of the codec and the bandwidth accounting helper.

Field-for-field mirror of ``Src/ADFL/model.py:18-66`` (``Parameters``, ``QuantParameter``,
``QuantParameters``, ``ByteParameter``, ``ByteParameters``, ``CompressedParameters``,
``ParameterInfo``) and ``get_parameter_info`` (``Src/ADFL/model.py:206-218``).

Drop-in interop: when the reference ``ADFL.model`` module is already imported in this process (an
ADFL experiment that plugs our channel into ``TrainingConfig.channel``), its dataclasses are reused,
so payloads produced by our channels are instances of the very classes the rest of ADFL sees.
"""

import sys
from dataclasses import dataclass
from typing import Dict, Union

import torch

Parameters = Dict[str, torch.Tensor]

_ref = sys.modules.get("ADFL.model")
_NAMES = ("QuantParameter", "QuantParameters", "ByteParameter", "ByteParameters", "MixedParameters",
          "ParameterInfo")

if _ref is not None and all(hasattr(_ref, n) for n in _NAMES):
    QuantParameter = _ref.QuantParameter
    QuantParameters = _ref.QuantParameters
    ByteParameter = _ref.ByteParameter
    ByteParameters = _ref.ByteParameters
    MixedParameters = _ref.MixedParameters
    ParameterInfo = _ref.ParameterInfo
else:
    @dataclass
    class QuantParameter:
        data: torch.Tensor
        bits: int
        scale: float
        signs: torch.Tensor  # used by QSGD-family codecs; SLQ stores zeros(1, uint8)
        shape: torch.Size
        dtype: torch.dtype
        q_dtype: torch.dtype
        scale_2: float = 0   # used by RQSGD

    @dataclass
    class QuantParameters:
        params: Dict[str, QuantParameter]
        size: int

    @dataclass
    class ByteParameter:
        data: bytes
        shape: torch.Size
        dtype: torch.dtype

    @dataclass
    class ByteParameters:
        params: Dict[str, ByteParameter]
        size: int

    @dataclass
    class MixedParameters:
        params: Dict[str, Union[QuantParameter, ByteParameter]]
        size: int

    @dataclass
    class ParameterInfo:
        num_non_bias_w: int
        num_non_bias_t: int
        num_bias_w: int
        num_bias_t: int

CompressedParameters = Union[QuantParameters, ByteParameters, MixedParameters]


def get_parameter_info(params: Parameters) -> ParameterInfo:
    """Counts of quantized ("non-bias", ndim > 1) and passthrough tensors/elements (model.py:206-218)."""
    p_info = ParameterInfo(0, 0, 0, 0)
    for tensor in params.values():
        if tensor.ndim > 1:
            p_info.num_non_bias_t += 1
            p_info.num_non_bias_w += tensor.numel()
        else:
            p_info.num_bias_t += 1
            p_info.num_bias_w += tensor.numel()
    return p_info


def _metric_pair(params_a: Parameters, params_b: Parameters, exclude_bias: bool):
    """The tensors Src/ADFL/model.py:264-323 reduces, in dict order (its asserts and its bias rule)."""
    assert params_a.keys() == params_b.keys()
    xs, ds = [], []
    for key in params_a:
        pa, pb = params_a[key], params_b[key]
        assert pa.shape == pb.shape
        if exclude_bias and (pa.ndim <= 1 or pb.ndim <= 1):
            continue
        xs.append(pa)
        ds.append(pb)
    return xs, ds


def _device_sums(xs, ds):
    """qerror.reference_sums of the two tensor lists, staged back to back on the channels' device."""
    from . import qerror
    for t in xs + ds:
        if t.dtype != torch.float32:
            raise NotImplementedError("adfl_amd.model: the device q-error metrics take fp32 parameters")
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.cat([t.reshape(-1) for t in xs]).to(dev, non_blocking=False)
    d = torch.cat([t.reshape(-1) for t in ds]).to(dev, non_blocking=False)
    return qerror.reference_sums(x, d, [int(t.numel()) for t in xs])


def parameter_relative_mse(params_a: Parameters, params_b: Parameters, exclude_bias: bool) -> float:
    """Drop-in for Src/ADFL/model.py:256-261 (parameter_relative_mse, with parameter_mse :264-283) computed on
    the device, bit for bit: every fp32 torch.sum((a - b) ** 2) and torch.sum((a - 0) ** 2) in torch's CPU order
    (qerror.reference_sums, csrc/qerror_ref.hip), turned into the same Python doubles in the same order."""
    from . import qerror
    xs, ds = _metric_pair(params_a, params_b, exclude_bias)
    if not xs:
        return 0.0
    e, s, c = _device_sums(xs, ds)
    return qerror.metrics(e, s, c, sum(int(t.numel()) for t in xs))[0]


def parameter_cosine_similarity(params_a: Parameters, params_b: Parameters, exclude_bias: bool) -> float:
    """Drop-in for Src/ADFL/model.py:301-323 (F.cosine_similarity of the fp32 concatenations, .item()) computed on
    the device, bit for bit (the dot product and both norms in torch's CPU order: qerror.reference_sums)."""
    xs, ds = _metric_pair(params_a, params_b, exclude_bias)
    if not xs:
        raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")
    return _device_sums(xs, ds)[2]
