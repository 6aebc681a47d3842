"""Host API of the reference's (deprecated) ``Src/ADFL/compression.py`` for the hot path's pieces — the
SLQ tensor codec and the int4 nibble layout — computed by the HIP kernels.

Same names, arguments, return types and devices as the reference:

* ``quantize_tensor(tensor, bits) -> (qint8 tensor, float scale)``      compression.py:26-33
* ``dequantize_tensor(q_param) -> tensor``                             compression.py:69-74
* ``pack_4bit(q_tensor) -> int8 tensor of ceil(n/2) packed bytes``      compression.py:35-48
* ``unpack_4bit(b_tensor: bytearray, shape) -> int8 tensor of shape``   compression.py:51-66

CPU inputs give CPU outputs (the computation itself runs on the current GPU: there is no CPU fallback),
device inputs stay on their device. ``pack_4bit`` keeps the reference's int8 wraparound for codes outside
[-8, 7] (127 packs to the nibble pair (7, -1)) and its zero pad for an odd count; like the reference it
works on a plain int8 tensor only (a qint8 tensor raises, as ``q_tensor + 8`` does there). The rest of the
deprecated module (byte serialization, mixed compression, ``compress_model``) is outside this repo's
scope.
"""

from typing import Tuple, Union

import torch

from . import ops
from .model import QuantParameter

__all__ = ["quantize_tensor", "dequantize_tensor", "pack_4bit", "unpack_4bit"]


def _device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device())


def quantize_tensor(tensor: torch.Tensor, bits: int) -> Tuple[torch.Tensor, float]:
    """compression.py:26-33 (= SLQChannel._quantize_tensor, quant.py:97-104): a per-tensor qint8 tensor
    (zero point 0) on the input's device and the scale as a Python float, bit-identical to the reference."""
    ops.require_quantizable(tensor)  # the reference's errors: non-fp32, empty (torch.max)
    x = tensor if tensor.is_cuda else tensor.to(_device())
    q, s = ops.encode(x.contiguous(), bits)
    scale = float(s.item())
    if not tensor.is_cuda:
        q = q.cpu()
    return torch._make_per_tensor_quantized_tensor(q.view(tensor.shape), scale, 0), scale


def dequantize_tensor(q_param: QuantParameter) -> torch.Tensor:
    """compression.py:69-74: ``data.dequantize()`` for an ndim > 1 payload, else the data unchanged."""
    data = q_param.data
    if data.ndim <= 1:
        return data.data
    if not (data.is_quantized and data.qscheme() == torch.per_tensor_affine and data.dtype == torch.qint8
            and data.q_zero_point() == 0):
        return data.data.dequantize()  # not an SLQ payload: the reference's own call
    q = torch.empty(0, dtype=torch.int8, device=data.device).set_(data.untyped_storage(), data.storage_offset(),
                                                                  data.shape, data.stride())
    dev = data.device if data.is_cuda else _device()
    # q_scale() is a double; the reference's dequantize uses it as fp32 (quant.py:110)
    scale = torch.tensor([data.q_scale()], dtype=torch.float32, device=dev)
    out = ops.decode(q.to(dev).contiguous(), scale).view(data.shape)
    return out if data.is_cuda else out.cpu()


def pack_4bit(q_tensor: torch.Tensor) -> torch.Tensor:
    """compression.py:35-48: byte i = ((q[2i] + 8) << 4) | (q[2i+1] + 8) in int8 arithmetic (high nibble =
    even element), one zero code appended to an odd count. Returns int8 [ceil(n/2)] on the input's device."""
    if q_tensor.is_quantized:
        raise NotImplementedError("pack_4bit: the reference packs a plain int8 tensor; a qint8 tensor "
                                  "fails in its `q_tensor + 8` (Src/ADFL/compression.py:46, :91-94)")
    if q_tensor.dtype != torch.int8:
        raise TypeError(f"pack_4bit: expected an int8 tensor, got {q_tensor.dtype}")
    n = q_tensor.numel()
    if n == 0:
        return torch.empty(0, dtype=torch.int8, device=q_tensor.device)
    q = q_tensor.reshape(-1)
    q = q if q.is_cuda else q.to(_device())
    packed = ops.pack_int4(q.contiguous()).view(torch.int8)
    return packed if q_tensor.is_cuda else packed.cpu()


def unpack_4bit(b_tensor: Union[bytearray, bytes, memoryview, torch.Tensor], shape: torch.Size) -> torch.Tensor:
    """compression.py:51-66: high nibble - 8, low nibble - 8 per byte, truncated to shape.numel(), reshaped.
    Takes the reference's bytearray (or bytes / a uint8 or int8 tensor); returns int8 of `shape` — on the
    tensor's device for a device tensor, on the CPU otherwise."""
    on_dev = isinstance(b_tensor, torch.Tensor) and b_tensor.is_cuda
    if isinstance(b_tensor, torch.Tensor):
        packed = b_tensor.reshape(-1).view(torch.uint8)
    else:
        packed = torch.frombuffer(bytearray(b_tensor), dtype=torch.uint8)
    shape = torch.Size(shape)
    n = shape.numel()
    if n > 2 * packed.numel():  # the reference's reshape of the truncated tensor fails the same way
        raise RuntimeError(f"shape '{list(shape)}' is invalid for input of size {2 * packed.numel()}")
    if n == 0:
        return torch.empty(shape, dtype=torch.int8, device=packed.device if on_dev else "cpu")
    p = packed if on_dev else packed.to(_device())
    q = ops.unpack_int4(p.contiguous(), list(shape))
    return q if on_dev else q.cpu()
