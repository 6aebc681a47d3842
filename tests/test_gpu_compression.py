"""GPU: adfl_amd.compression — the reference's compression.py functions on the hot path (quantize_tensor,
dequantize_tensor, pack_4bit, unpack_4bit: Src/ADFL/compression.py:26-74) with the reference's arguments
(CPU tensors, a bytearray for unpack_4bit) against the golden vectors the reference itself produced."""

import numpy as np
import pytest
import torch

from golden_util import int4, manifest, same_f32, same_scale, small, small_cases

pytestmark = pytest.mark.gpu

compression = pytest.importorskip("adfl_amd.compression")
from adfl_amd.model import QuantParameter  # noqa: E402

DEV = torch.device("cuda", 0)
INT4 = manifest()["int4"]


@pytest.mark.parametrize("case", INT4, ids=lambda c: c["name"])
@pytest.mark.parametrize("where", ["cpu", "cuda"])
def test_pack_unpack_4bit_vs_reference_vectors(case, where):
    I = int4()
    q = torch.from_numpy(I[f"int4_{case['name']}__q"].copy())
    packed_ref = I[f"int4_{case['name']}__packed"]
    unpacked_ref = I[f"int4_{case['name']}__unpacked"]
    src = q if where == "cpu" else q.to(DEV)
    packed = compression.pack_4bit(src)
    assert packed.dtype == torch.int8 and packed.device == src.device
    assert np.array_equal(packed.cpu().numpy(), packed_ref.view(np.int8))
    if where == "cpu":  # the reference's call shape: bytes of the packed payload + the original shape
        unpacked = compression.unpack_4bit(bytearray(packed_ref.tobytes()), q.shape)
        assert unpacked.device.type == "cpu"
    else:
        unpacked = compression.unpack_4bit(torch.from_numpy(packed_ref.copy()).to(DEV), q.shape)
        assert unpacked.is_cuda
    assert unpacked.dtype == torch.int8 and tuple(unpacked.shape) == tuple(q.shape)
    assert np.array_equal(unpacked.cpu().numpy(), unpacked_ref)


def test_pack_4bit_reference_edges():
    assert compression.pack_4bit(torch.empty(0, dtype=torch.int8)).numel() == 0
    odd = torch.tensor([-8, 7, 3], dtype=torch.int8)  # zero code appended: (3+8)<<4 | (0+8)
    assert compression.pack_4bit(odd).tolist() == [0x0F, (11 << 4 | 8) - 256]
    q8 = torch.quantize_per_tensor(torch.randn(4, 4), 0.1, 0, torch.qint8)
    with pytest.raises(NotImplementedError):  # the reference's 4-bit quantize_params path (compression.py:91-94)
        compression.pack_4bit(q8)
    with pytest.raises(RuntimeError, match="is invalid for input of size"):
        compression.unpack_4bit(bytearray(3), torch.Size([7]))


@pytest.mark.parametrize("case", small_cases(), ids=lambda c: c["name"])
def test_quantize_dequantize_tensor_vs_reference(case):
    A = small()
    x = torch.from_numpy(A[case["name"] + "__x"].copy())
    q, scale = compression.quantize_tensor(x, case["bits"])
    assert q.dtype == torch.qint8 and q.device.type == "cpu" and q.q_zero_point() == 0 and q.shape == x.shape
    assert np.array_equal(q.int_repr().numpy(), A[case["name"] + "__q"])
    assert same_scale(scale, case["scale_bits"]) and same_scale(q.q_scale(), case["scale_bits"])
    qp = QuantParameter(data=q, bits=case["bits"], scale=scale, signs=torch.zeros(1, dtype=torch.uint8),
                        shape=x.shape, dtype=x.dtype, q_dtype=q.dtype)
    d = compression.dequantize_tensor(qp)
    assert d.dtype == torch.float32 and d.device.type == "cpu"
    if x.ndim > 1:
        assert same_f32(d.numpy(), A[case["name"] + "__deq"])
    else:
        assert d.data_ptr() == q.data_ptr()  # ndim <= 1: the data itself (compression.py:73-74)


def test_quantize_tensor_errors_and_device_inputs():
    with pytest.raises(RuntimeError, match="Quantize only works on Float Tensor, got Double"):
        compression.quantize_tensor(torch.zeros(3, 3, dtype=torch.float64), 8)
    with pytest.raises(RuntimeError, match="Expected reduction dim"):
        compression.quantize_tensor(torch.zeros(0, 3), 8)
    x = torch.randn(33, 31, device=DEV) * 1e-3
    q, s = compression.quantize_tensor(x, 8)
    qc, sc = compression.quantize_tensor(x.cpu(), 8)
    assert q.is_cuda and s == sc and torch.equal(q.int_repr().cpu(), qc.int_repr())
