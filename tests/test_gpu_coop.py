"""GPU parity of the one-launch cooperative bucketed encode (adfl_slq_encode_batched_coop: chunk blocks of a
tensor meet through per-tensor sync words; the loop of Src/ADFL/Channel/quant.py:74-94 over quant.py:97-104).
Bar: bit-exact payload and scales against the golden SHA-256s and the oracle, the sync words zero again
after every launch, and the same bytes as the two-pass and resident encodes."""

import numpy as np
import pytest
import torch

import recipes
import slq_oracle as oracle
from golden_util import manifest, same_f32, same_scale

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("adfl_amd.ops")
from adfl_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)


def _coop(x, lay, bits, sync=None):
    q = torch.empty(lay.total, dtype=torch.int8, device=DEV)
    sc = torch.empty(lay.ntensors, dtype=torch.float32, device=DEV)
    part = torch.empty(lay.nchunks, dtype=torch.int32, device=DEV)
    st = torch.cuda.current_stream(DEV).cuda_stream
    sync = lay.device_sync(DEV, st) if sync is None else sync
    _lib.check(_lib.load().adfl_slq_encode_batched_coop(x.data_ptr(), lay.device_chunks(DEV).data_ptr(), lay.nchunks,
                                                       bits, q.data_ptr(), sc.data_ptr(), part.data_ptr(),
                                                       sync.data_ptr(), st))
    return q, sc, sync


def _check_vs_oracle(flat, lay, q, sc, bits):
    qn, sn = q.cpu().numpy(), sc.cpu().numpy()
    for t, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        q_ref, s_ref = oracle.encode(flat[o:o + n], bits)
        assert np.array_equal(qn[o:o + n], q_ref), (bits, t)
        assert same_f32(sn[t], s_ref), (bits, t)


def test_capacity_covers_c3():
    cap = _lib.load().adfl_slq_coop_capacity()
    assert cap >= 1607, cap  # the C3 log-uniform chunk table runs in one resident grid


@pytest.mark.parametrize("case", manifest()["bucket"], ids=lambda c: c["layout"])
@pytest.mark.parametrize("mode", ["coop", "twopass", "auto"])
def test_c3_golden_every_encode_mode(case, mode, monkeypatch):
    monkeypatch.setenv("ADFL_SLQ_ENCODE", mode)
    tensors = recipes.bucket_tensors(case["layout"], case["seed"], case["mult"])
    lay = ops.BucketLayout(case["sizes"])
    flat = torch.zeros(lay.total, dtype=torch.float32)
    for (k, v), off in zip(tensors.items(), lay.offsets):
        flat[int(off):int(off) + v.size] = torch.from_numpy(v.reshape(-1))
    q, scales = ops.encode_batched(flat.to(DEV), lay, case["bits"])
    torch.cuda.synchronize()
    for s, b in zip(scales.cpu().numpy(), case["scale_bits"]):
        assert same_scale(s, b)
    qn = q.cpu().numpy()
    q_cat = np.concatenate([qn[int(o):int(o) + int(n)] for o, n in zip(lay.offsets, lay.sizes)])
    assert recipes.sha256(q_cat) == case["q_sha256"]


@pytest.mark.parametrize("align", [64, 1, 3])
def test_ragged_specials_large_tensors_vs_oracle(align):
    """Tensors of 1 .. 300 chunks, compact and aligned; NaN / inf / all-zero tensors; chunk-edge specials.
    Every launch leaves the sync words zero (no block gave up waiting)."""
    rng = np.random.default_rng(31)
    sizes = [1, 8192 * 300 + 17, 65536, 65537, 3, 8193, 8192 * 40, 20000, 1 << 20, 5, 8192 * 2, 777777]
    lay = ops.BucketLayout(sizes, align=align)
    flat = np.zeros(lay.total, np.float32)
    for i, (o, n) in enumerate(zip(lay.offsets, lay.sizes)):
        flat[o:o + n] = rng.standard_normal(n, dtype=np.float32) * np.float32(10.0 ** -(i % 6))
    flat[lay.offsets[1] + 8192 * 300 + 16] = np.inf          # last element of the 301-chunk tensor
    flat[lay.offsets[3] + 65536] = np.nan                     # the 9th chunk's only element
    flat[lay.offsets[6]:lay.offsets[6] + 8192 * 40] = 0.0     # all-zero multi-chunk tensor
    flat[lay.offsets[8] + 8191] = -np.inf                     # chunk edge
    flat[lay.offsets[10] + 8192] = 1e-41                      # denormal, second chunk
    x = torch.from_numpy(flat).to(DEV)
    for bits in (8, 4, 2, 16):
        q, sc, sync = _coop(x, lay, bits)
        _check_vs_oracle(flat, lay, q, sc, bits)
        assert int(sync.count_nonzero()) == 0, bits


def test_many_launches_reuse_sync_and_match_two_pass():
    """200 back-to-back launches on one sync buffer, inputs changing every time: each equals the two-pass
    encode of the same input, and the buffer is zero at the end."""
    sizes = [8192 * k + (k % 7) for k in range(1, 40)] + [300000, 1, 2, 9000]
    lay = ops.BucketLayout(sizes, align=1)
    g = torch.Generator(device=DEV).manual_seed(3)
    st = torch.cuda.current_stream(DEV).cuda_stream
    sync = lay.device_sync(DEV, st)
    outs, xs = [], []
    for i in range(200):
        x = torch.randn(lay.total, device=DEV, generator=g) * (1.0 + i)
        q, sc, _ = _coop(x, lay, 8, sync)
        if i % 20 == 0:
            outs.append((q.clone(), sc.clone()))
            xs.append(x)
    torch.cuda.synchronize()
    assert int(sync.count_nonzero()) == 0
    part = torch.empty(lay.nchunks, dtype=torch.int32, device=DEV)
    for x, (q, sc) in zip(xs, outs):
        q2 = torch.empty_like(q)
        sc2 = torch.empty_like(sc)
        _lib.check(_lib.load().adfl_slq_encode_batched(x.data_ptr(), lay.device_chunks(DEV).data_ptr(), lay.nchunks,
                                                       8, q2.data_ptr(), sc2.data_ptr(), part.data_ptr(), st))
        assert torch.equal(q, q2) and torch.equal(sc, sc2)


def test_past_capacity_runs_two_pass():
    """A chunk table larger than the co-resident capacity takes the two-pass path (same bytes)."""
    cap = int(_lib.load().adfl_slq_coop_capacity())
    n = (cap + 64) * 8192
    lay = ops.BucketLayout([n // 2, n - n // 2])
    assert lay.nchunks > cap
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(lay.total, device=DEV, generator=g)
    q, sc, sync = _coop(x, lay, 8)
    q2, sc2 = ops.encode(x[:n // 2], 8)
    torch.cuda.synchronize()
    assert torch.equal(q[:n // 2], q2) and torch.equal(sc[:1], sc2.reshape(1))
    assert int(sync.count_nonzero()) == 0


def test_two_streams_own_sync_buffers(monkeypatch):
    """Encodes of one layout on two streams use separate sync buffers and both equal the oracle."""
    monkeypatch.setenv("ADFL_SLQ_ENCODE", "coop")
    sizes = [8192 * 50, 8192 * 3 + 1, 100]
    lay = ops.BucketLayout(sizes)
    rng = np.random.default_rng(8)
    f1 = rng.standard_normal(lay.total, dtype=np.float32)
    f2 = rng.standard_normal(lay.total, dtype=np.float32) * np.float32(3.0)
    x1, x2 = torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    res = []
    for s, x in ((s1, x1), (s2, x2)):
        with torch.cuda.stream(s):
            res.append(ops.encode_batched(x, lay, 8, partials=None))
    torch.cuda.synchronize()
    assert len(lay._device_sync) >= 2
    _check_vs_oracle(f1, lay, *res[0], 8)
    _check_vs_oracle(f2, lay, *res[1], 8)
