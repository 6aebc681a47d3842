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
