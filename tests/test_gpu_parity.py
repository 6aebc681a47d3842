"""GPU parity: the HIP codec (through the C ABI, via adfl_amd.ops) against the reference's golden
vectors and the oracle. Bar: bit-exact int8 payload, fp32 scale and dequantized floats (NaN positions
compared, NaN payload bits not)."""

import numpy as np
import pytest
import torch

import recipes
import slq_oracle as oracle
from golden_util import int4, manifest, same_f32, same_scale, small, small_cases

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("adfl_amd.ops")
DEV = torch.device("cuda", 0)

CASES = small_cases()


def _enc(x_np, bits):
    q, s = ops.encode(torch.from_numpy(np.ascontiguousarray(x_np)).to(DEV), bits)
    return q, s


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_small_cases(case):
    A = small()
    x, q_ref, d_ref = A[case["name"] + "__x"], A[case["name"] + "__q"], A[case["name"] + "__deq"]
    q, s = _enc(x, case["bits"])
    d = ops.decode(q, s)
    torch.cuda.synchronize()
    assert q.shape == x.shape and q.dtype == torch.int8
    assert np.array_equal(q.cpu().numpy(), q_ref)
    assert same_scale(s.item(), case["scale_bits"])
    assert same_f32(d.cpu().numpy(), d_ref)


RECIPES = manifest()["recipe"]


@pytest.mark.parametrize("case", RECIPES, ids=[f"{c['recipe']['kind']}{c['recipe']['shape']}_b{c['bits']}"
                                             for c in RECIPES])
def test_golden_recipe_cases(case):
    """Includes the 1 GiB C2 workload ([262144, 1024], the bench input shape) at bits 8 and 4."""
    x = torch.from_numpy(recipes.make(case["recipe"])).to(DEV)
    q, s = ops.encode(x, case["bits"])
    d = ops.decode(q, s)
    torch.cuda.synchronize()
    assert same_scale(s.item(), case["scale_bits"])
    assert recipes.sha256(q.cpu().numpy()) == case["q_sha256"]
    assert recipes.sha256(d.cpu().numpy()) == case["deq_sha256"]


def test_full_size_sign_symmetry():
    """Size-independent property at the bench size: encode(-x) == -encode(x) with the same scale."""
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(1 << 28, device=DEV, generator=g) * 1e-3
    q, s = ops.encode(x, 8)
    qn, sn = ops.encode(-x, 8)
    torch.cuda.synchronize()
    assert s.item() == sn.item()
    assert torch.equal(qn, -q)
    assert int(q.abs().max()) == 127


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 15, 16, 17, 31, 33, 63, 64, 65, 255, 256, 257, 4095, 4097,
                               65535, 65537, 1048575, 1048577, 4194305])
def test_ragged_lengths_vs_oracle(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n, dtype=np.float32) * np.float32(1e-2)
    for bits in (8, 4):
        q, s = _enc(x, bits)
        d = ops.decode(q, s)
        q_ref, s_ref = oracle.encode(x, bits)
        assert np.array_equal(q.cpu().numpy(), q_ref)
        assert same_f32(s.item(), s_ref)
        assert same_f32(d.cpu().numpy(), oracle.decode(q_ref, s_ref))


def test_special_values_at_many_positions():
    """NaN / inf / denormal at vector-body and tail positions of a ragged tensor."""
    rng = np.random.default_rng(9)
    for n, pos, val in [(1000, 0, np.inf), (1000, 999, -np.inf), (1001, 500, np.nan), (4099, 4098, np.nan),
                        (4099, 17, 1e-41), (333, 332, -np.inf)]:
        x = rng.standard_normal(n, dtype=np.float32)
        x[pos] = val
        q, s = _enc(x, 8)
        q_ref, s_ref = oracle.encode(x, 8)
        assert np.array_equal(q.cpu().numpy(), q_ref), (n, pos, val)
        assert same_f32(s.item(), s_ref)
        assert same_f32(ops.decode(q, s).cpu().numpy(), oracle.decode(q_ref, s_ref))


def test_non_contiguous_and_misaligned_inputs():
    base = torch.randn(300, 301, device=DEV)
    xt = base.t()                      # non-contiguous
    xo = base.reshape(-1)[1:90001]     # 4-byte offset from the allocation (not 16-byte aligned)
    for x in (xt, xo):
        q, s = ops.encode(x, 8)
        q_ref, s_ref = oracle.encode(x.cpu().contiguous().numpy(), 8)
        assert q.is_contiguous() and q.shape == x.shape
        assert np.array_equal(q.cpu().numpy(), q_ref)
        assert same_f32(s.item(), s_ref)


@pytest.mark.parametrize("case", manifest()["bucket"], ids=lambda c: c["layout"])
def test_bucketed_c3_vs_golden(case):
    """BASELINE config C3: ResNet-18-sized update in 256 tensors, per-tensor scales, one launch per pass."""
    tensors = recipes.bucket_tensors(case["layout"], case["seed"], case["mult"])
    lay = ops.BucketLayout(case["sizes"])
    flat = torch.zeros(lay.total, dtype=torch.float32)
    for (k, v), off in zip(tensors.items(), lay.offsets):
        flat[int(off):int(off) + v.size] = torch.from_numpy(v.reshape(-1))
    q, scales = ops.encode_batched(flat.to(DEV), lay, case["bits"])
    d = ops.decode_batched(q, scales, lay)
    torch.cuda.synchronize()
    sc = scales.cpu().numpy()
    for s, b in zip(sc, case["scale_bits"]):
        assert same_scale(s, b)
    qn, dn = q.cpu().numpy(), d.cpu().numpy()
    q_cat = np.concatenate([qn[int(o):int(o) + int(n)] for o, n in zip(lay.offsets, lay.sizes)])
    d_cat = np.concatenate([dn[int(o):int(o) + int(n)] for o, n in zip(lay.offsets, lay.sizes)])
    assert recipes.sha256(q_cat) == case["q_sha256"]
    assert recipes.sha256(d_cat) == case["deq_sha256"]


@pytest.mark.parametrize("align", [64, 1, 3])
def test_bucketed_ragged_and_specials_vs_oracle(align):
    """Aligned and compact (back-to-back, every chunk start misaligned) buckets."""
    rng = np.random.default_rng(11)
    sizes = [1, 17, 8191, 8192, 8193, 64, 3, 20000, 5, 1023, 1025, 16]
    lay = ops.BucketLayout(sizes, align=align)
    flat = np.zeros(lay.total, np.float32)
    for i, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -i)
    flat[lay.offsets[2] + 100] = np.nan
    flat[lay.offsets[4] + 8192] = -np.inf
    flat[lay.offsets[6]:lay.offsets[6] + 3] = 0.0
    for bits in (8, 4, 2):
        q, scales = ops.encode_batched(torch.from_numpy(flat).to(DEV), lay, bits)
        d = ops.decode_batched(q, scales, lay)
        qn, sn, dn = q.cpu().numpy(), scales.cpu().numpy(), d.cpu().numpy()
        for t, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
            q_ref, s_ref = oracle.encode(flat[o:o + n], bits)
            assert np.array_equal(qn[o:o + n], q_ref), (bits, t)
            assert same_f32(sn[t], s_ref), (bits, t)
            assert same_f32(dn[o:o + n], oracle.decode(q_ref, s_ref)), (bits, t)


@pytest.mark.parametrize("align", [64, 1])
@pytest.mark.parametrize("legacy", [False, True])
def test_bucketed_resident_boundary_vs_oracle(align, legacy):
    """Tensors at the one-block limit (65,536 elements = 8 chunks) and just past it (9 chunks), compact or
    aligned, NaN and +-inf at chunk edges: with a large tensor present the encode is the two-pass one;
    without it (the second half) the one-launch resident encode. `legacy` calls adfl_slq_encode_batched
    directly."""
    from adfl_amd import _lib
    rng = np.random.default_rng(21)
    sizes = [65536, 65537, 1, 65535, 131072 + 5, 16, 49152, 8192 * 8 + 8191, 3000, 65536 - 15]
    lay = ops.BucketLayout(sizes, align=align)
    assert lay.nwork == 0  # tensors above 65,536 elements: the two-pass encode
    flat = np.zeros(lay.total, np.float32)
    for i, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -(i % 5))
    flat[lay.offsets[0] + 65535] = np.inf          # last element of a resident tensor
    flat[lay.offsets[1] + 65536] = np.nan          # the 9th chunk's only element
    flat[lay.offsets[6]:lay.offsets[6] + 49152] = 0.0   # all-zero resident tensor: payload all 127
    flat[lay.offsets[9] + 7] = -np.inf
    x = torch.from_numpy(flat).to(DEV)
    for bits in (8, 3):
        if legacy:
            q = torch.empty(lay.total, dtype=torch.int8, device=DEV)
            sc = torch.empty(lay.ntensors, dtype=torch.float32, device=DEV)
            part = torch.empty(lay.nchunks, dtype=torch.int32, device=DEV)
            _lib.check(_lib.load().adfl_slq_encode_batched(
                x.data_ptr(), lay.device_chunks(DEV).data_ptr(), lay.nchunks, bits, q.data_ptr(), sc.data_ptr(),
                part.data_ptr(), torch.cuda.current_stream(DEV).cuda_stream))
        else:
            q, sc = ops.encode_batched(x, lay, bits)
        qn, sn = q.cpu().numpy(), sc.cpu().numpy()
        for t, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
            q_ref, s_ref = oracle.encode(flat[o:o + n], bits)
            assert np.array_equal(qn[o:o + n], q_ref), (bits, t)
            assert same_f32(sn[t], s_ref), (bits, t)
    small = [n for n in sizes if n <= 65536]
    lay = ops.BucketLayout(small, align=align)
    assert lay.nwork == len(small)
    flat = np.zeros(lay.total, np.float32)
    for i, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -(i % 5))
    flat[lay.offsets[0] + 65535] = np.nan
    flat[lay.offsets[3]:lay.offsets[3] + 49152] = 0.0
    flat[lay.offsets[6] + 3] = -np.inf
    q, sc = ops.encode_batched(torch.from_numpy(flat).to(DEV), lay, 8)
    qn, sn = q.cpu().numpy(), sc.cpu().numpy()
    for t, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        q_ref, s_ref = oracle.encode(flat[o:o + n], 8)
        assert np.array_equal(qn[o:o + n], q_ref), t
        assert same_f32(sn[t], s_ref), t


def test_bucketed_all_resident_is_one_launch():
    """C3's equal layout (256 x 45,662): every tensor fits one block, the encode is a single launch and still
    equals the oracle per tensor."""
    sizes = [11689512 // 256 + (1 if i < 11689512 % 256 else 0) for i in range(256)]
    lay = ops.BucketLayout(sizes)
    assert lay.nwork == 256
    rng = np.random.default_rng(5)
    flat = (rng.standard_normal(lay.total, dtype=np.float32) * np.float32(1e-3))
    q, sc = ops.encode_batched(torch.from_numpy(flat).to(DEV), lay, 8)
    qn, sn = q.cpu().numpy(), sc.cpu().numpy()
    for t in range(0, 256, 17):
        o, n = lay.offsets[t], lay.sizes[t]
        q_ref, s_ref = oracle.encode(flat[o:o + n], 8)
        assert np.array_equal(qn[o:o + n], q_ref) and same_f32(sn[t], s_ref), t


@pytest.mark.parametrize("case", manifest()["int4"], ids=lambda c: c["name"])
def test_int4_pack_unpack_vs_golden(case):
    I = int4()
    q = I[f"int4_{case['name']}__q"]
    packed_ref = I[f"int4_{case['name']}__packed"].view(np.uint8)
    unpacked_ref = I[f"int4_{case['name']}__unpacked"]
    packed = ops.pack_int4(torch.from_numpy(q).to(DEV))
    assert np.array_equal(packed.cpu().numpy(), packed_ref)
    unpacked = ops.unpack_int4(torch.from_numpy(packed_ref.copy()).to(DEV), q.shape)
    assert np.array_equal(unpacked.cpu().numpy(), unpacked_ref)


@pytest.mark.parametrize("n", [1, 2, 3, 31, 32, 33, 63, 64, 65, 4097, 1048577])
def test_int4_fused_encode_decode_vs_oracle(n):
    rng = np.random.default_rng(100 + n)
    x = rng.standard_normal(n, dtype=np.float32)
    if n > 40:
        x[n // 2] = np.nan if n % 2 else 0.0
    for bits in (4, 8, 2):
        packed, s = ops.encode_int4(torch.from_numpy(x).to(DEV), bits)
        q_ref, s_ref = oracle.encode(x, bits)
        p_ref = oracle.pack_int4(q_ref)
        assert np.array_equal(packed.cpu().numpy(), p_ref), bits
        assert same_f32(s.item(), s_ref)
        d = ops.decode_int4(packed, n, s)
        assert same_f32(d.cpu().numpy(), oracle.decode_int4(p_ref, n, s_ref))


def test_int4_zero_tensor_aliasing():
    """All-zero tensor: payload 127 aliases to nibbles (7, -1) exactly as pack_4bit does."""
    x = torch.zeros(4, 9, device=DEV)
    packed, s = ops.encode_int4(x, 4)
    q_ref, s_ref = oracle.encode(np.zeros((4, 9), np.float32), 4)
    assert np.array_equal(packed.cpu().numpy(), oracle.pack_int4(q_ref))
    assert s.item() == 0.0


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_dequantize_mean_vs_oracle_and_torch(k):
    rng = np.random.default_rng(k)
    n, row = 100003, 100016
    qs = rng.integers(-128, 128, (k, row), dtype=np.int8)
    scales = (rng.random(k, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
    got = ops.dequantize_mean(torch.from_numpy(qs).to(DEV), torch.from_numpy(scales).to(DEV), n).cpu().numpy()
    ref = oracle.dequantize_mean([q[:n] for q in qs], scales)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    torch_mean = torch.stack([torch.from_numpy(oracle.decode(q[:n], s)) for q, s in zip(qs, scales)]).mean(0)
    np.testing.assert_allclose(got, torch_mean.numpy(), rtol=1e-6, atol=0)  # north_star tolerance


def test_round_trip_is_graph_capturable():
    """The C ABI allocates nothing and never synchronises: a whole round trip captured in a HIP graph
    replays correctly on new data (include/adfl_slq.h contract)."""
    from adfl_amd import _lib
    lib = _lib.load()
    n = (1 << 20) + 37
    x = torch.empty(n, device=DEV)
    q = torch.empty(n, dtype=torch.int8, device=DEV)
    s = torch.empty(1, device=DEV)
    ws = ops.new_workspace(DEV)
    out = torch.empty(n, device=DEV)
    x.copy_(torch.randn(n, device=DEV))
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(g):
            sh = torch.cuda.current_stream().cuda_stream
            assert lib.adfl_slq_encode(x.data_ptr(), n, 8, q.data_ptr(), s.data_ptr(), ws.data_ptr(),
                                       ws.numel(), sh) == 0
            assert lib.adfl_slq_dequantize(q.data_ptr(), n, s.data_ptr(), out.data_ptr(), sh) == 0
    torch.cuda.current_stream().wait_stream(side)
    for seed in (1, 2):
        xn = np.random.default_rng(seed).standard_normal(n, dtype=np.float32) * np.float32(seed)
        x.copy_(torch.from_numpy(xn))
        g.replay()
        torch.cuda.synchronize()
        q_ref, s_ref = oracle.encode(xn, 8)
        assert np.array_equal(q.cpu().numpy(), q_ref)
        assert same_f32(out.cpu().numpy(), oracle.decode(q_ref, s_ref))


def test_custom_ops_registered():
    x = torch.randn(64, 33, device=DEV)
    q, s = torch.ops.adfl.slq_encode(x, 8)
    d = torch.ops.adfl.slq_decode(q, s)
    q_ref, s_ref = oracle.encode(x.cpu().numpy(), 8)
    assert np.array_equal(q.cpu().numpy(), q_ref)
    assert same_f32(d.cpu().numpy(), oracle.decode(q_ref, s_ref))
    p, s4 = torch.ops.adfl.slq_encode_int4(x, 4)
    d4 = torch.ops.adfl.slq_decode_int4(p, x.numel(), s4)
    assert d4.shape == (x.numel(),)


def test_reference_errors():
    with pytest.raises(RuntimeError, match="Quantize only works on Float Tensor, got Double"):
        ops.encode(torch.randn(3, 3, dtype=torch.float64, device=DEV), 8)
    with pytest.raises(RuntimeError, match="Quantize only works on Float Tensor, got BFloat16"):
        ops.encode(torch.randn(3, 3, device=DEV).bfloat16(), 8)
    with pytest.raises(RuntimeError, match="numel\\(\\) == 0"):
        ops.encode(torch.empty(0, 5, device=DEV), 8)
    from adfl_amd._lib import AdflError
    with pytest.raises(AdflError, match="bits"):
        ops.encode(torch.randn(3, 3, device=DEV), 0)


INT4_SIZES = {
    "small": [1, 2, 3, 31, 32, 33, 2047, 2048, 2049, 8191, 8192, 8193, 20001, 5, 4096 * 3 + 7],
    # one-block limit (65,536) and odd sizes right under it: the one-launch encode's head/tail pairs
    "boundary": [65536, 65535, 7, 65533, 2049, 31, 65534, 1, 4099, 8193],
    # a tensor past the limit: the two-pass encode for the whole bucket
    "large": [65537, 1, 33, 70001, 2048, 131075, 3],
}


@pytest.mark.parametrize("align", [2, 64])
@pytest.mark.parametrize("bits", [4, 2])
@pytest.mark.parametrize("kind", list(INT4_SIZES))
def test_bucketed_int4_vs_oracle(align, bits, kind):
    """Packed int4 buckets (PackedSLQChannel's kernels): per tensor, pack_4bit(SLQ(x)) and its decode."""
    rng = np.random.default_rng(40 + align + bits)
    sizes = INT4_SIZES[kind]
    lay = ops.BucketLayout(sizes, align=align)
    assert (lay.nwork == 0) == (kind == "large")
    flat = np.zeros(lay.total, np.float32)
    for i, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(2.0 ** -i)
    flat[lay.offsets[3]:lay.offsets[3] + lay.sizes[3]] = 0.0          # aliasing tensor (payload 127)
    flat[lay.offsets[4] + lay.sizes[4] // 2] = np.nan
    flat[lay.offsets[0] + lay.sizes[0] - 1] = -np.inf
    packed, scales = ops.encode_batched_int4(torch.from_numpy(flat).to(DEV), lay, bits)
    out = ops.decode_batched_int4(packed, scales, lay)
    pn, sn, dn = packed.cpu().numpy(), scales.cpu().numpy(), out.cpu().numpy()
    for t, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        q_ref, s_ref = oracle.encode(flat[o:o + n], bits)
        p_ref = oracle.pack_int4(q_ref)
        assert np.array_equal(pn[o // 2:o // 2 + p_ref.size], p_ref), (t, n)
        assert same_f32(sn[t], s_ref), t
        assert same_f32(dn[o:o + n], oracle.decode_int4(p_ref, n, s_ref)), t
