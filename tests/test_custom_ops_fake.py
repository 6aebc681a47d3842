"""CPU: every torch.ops.adfl.* op is registered with the schema §8b lists and a fake implementation, so
shapes and dtypes propagate under FakeTensorMode (what torch.compile traces with) without a GPU; the real
kernels are tested in tests/test_gpu_custom_ops.py. Also the caller-placed BucketLayout behind the batched
ops (offsets validated on the host)."""

import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import adfl_amd  # noqa: F401  registers torch.ops.adfl.*
from adfl_amd import ops

A = torch.ops.adfl
OPS = ["slq_absmax", "slq_encode", "slq_decode", "slq_encode_int4", "slq_decode_int4", "slq_encode_batched",
       "slq_decode_batched", "slq_encode_batched_int4", "slq_decode_batched_int4", "pack_int4", "unpack_int4",
       "slq_dequantize_mean", "slq_dequantize_mean_batched", "slq_dequantize_mean_batched_int4",
       "stoch_encode_batched", "stoch_decode_batched"]


def test_every_op_is_registered():
    for name in OPS:
        assert hasattr(A, name), name
    assert "Tensor? self_x" in str(A.slq_dequantize_mean.default._schema)


def test_fake_shapes_and_dtypes():
    off, siz = torch.tensor([0, 100, 50]), torch.tensor([40, 7, 50])
    with FakeTensorMode(allow_non_fake_inputs=True) as mode:
        x = mode.from_tensor(torch.empty(110, 3))
        flat = mode.from_tensor(torch.empty(107))
        a = A.slq_absmax(x)
        assert a.shape == () and a.dtype == torch.float32
        q, s = A.slq_encode(x, 8)
        assert q.shape == (110, 3) and q.dtype == torch.int8 and s.shape == (1,)
        assert A.slq_decode(q, s).dtype == torch.float32
        p, s4 = A.slq_encode_int4(x, 4)
        assert p.shape == (165,) and p.dtype == torch.uint8
        assert A.slq_decode_int4(p, 330, s4).shape == (330,)
        qb, sb = A.slq_encode_batched(flat, off, siz, 8)
        assert qb.shape == (107,) and qb.dtype == torch.int8 and sb.shape == (3,)
        assert A.slq_decode_batched(qb, sb, off, siz).shape == (107,)
        pb, _ = A.slq_encode_batched_int4(flat, off, siz, 4)
        assert pb.shape == (54,) and pb.dtype == torch.uint8
        assert A.slq_decode_batched_int4(pb, sb, off, siz, 107).shape == (107,)
        assert A.pack_int4(qb).shape == (54,)
        assert A.unpack_int4(pb, [9, 12]).shape == (9, 12)
        rows = mode.from_tensor(torch.empty(4, 128, dtype=torch.int8))
        m = A.slq_dequantize_mean(rows, mode.from_tensor(torch.empty(4)), 100, -1, None)
        assert m.shape == (100,) and m.dtype == torch.float32
        mb = A.slq_dequantize_mean_batched(rows, mode.from_tensor(torch.empty(4, 3)), off, siz, 107, -1, None)
        assert mb.shape == (107,) and mb.dtype == torch.float32
        prow = mode.from_tensor(torch.empty(4, 64, dtype=torch.uint8))
        mb4 = A.slq_dequantize_mean_batched_int4(prow, mode.from_tensor(torch.empty(4, 3)), off, siz, 107, -1, None)
        assert mb4.shape == (107,) and mb4.dtype == torch.float32
        for codec in ("qsgd", "rqsgd", "cnat"):
            lv, sg, nr, mn = A.stoch_encode_batched(flat, off, siz, codec, 8, 7, 0)
            assert lv.shape == (107,) and lv.dtype == (torch.int8 if codec == "cnat" else torch.uint8)
            assert sg.dtype == torch.int8 and nr.shape == (3,) and mn.shape == (3,)
            d = A.stoch_decode_batched(lv, sg, nr, mn, off, siz, codec, 8)
            assert d.shape == (107,) and d.dtype == torch.float32
        for dt in (torch.float16, torch.bfloat16, torch.float64):   # encoded in their own dtype's arithmetic
            lv, sg, nr, mn = A.stoch_encode_batched(mode.from_tensor(torch.empty(107, dtype=dt)), off, siz, "cnat",
                                                    8, 7, 0)
            assert lv.shape == (107,) and lv.dtype == torch.int8 and nr.dtype == torch.float32


def test_caller_placed_layout():
    lay = ops.layout_for(torch.tensor([100, 0, 20000]), torch.tensor([7, 90, 8193]))
    assert lay.total == 28193 and lay.ntensors == 3 and lay.nchunks == 1 + 1 + 2
    assert ops.layout_for(torch.tensor([100, 0, 20000]), torch.tensor([7, 90, 8193])) is lay   # cached
    with pytest.raises(ValueError, match="overlap"):
        ops.layout_for(torch.tensor([0, 50]), torch.tensor([60, 10]))
    with pytest.raises(ValueError, match="non-negative"):
        ops.layout_for(torch.tensor([-1, 50]), torch.tensor([6, 10]))
    with pytest.raises(ValueError, match="one non-negative offset per tensor"):
        ops.BucketLayout([5, 5], offsets=[0])
    even = ops.BucketLayout([3, 8], offsets=[10, 0])
    assert even.align % 2 == 0   # int4 ops accept it
