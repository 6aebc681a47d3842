"""GPU: beyond 32-bit element counts (8 GiB of fp32). Kept in its own file so it can be run (and
skipped) separately: it allocates ~27 GiB of device memory."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("adfl_amd.ops")
DEV = torch.device("cuda", 0)


def test_beyond_int32_element_count():
    """2^31 + 37 elements (8 GiB fp32): 64-bit indexing end to end. Checked on sampled positions at the
    start, around 2^31 and at the ragged tail against the oracle's elementwise rule, plus the scale."""
    n = (1 << 31) + 37
    x = torch.empty(n, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(5)
    # torch ops only ever see < 2^31-element pieces here; only the codec kernels see the whole buffer
    for a in range(0, n, 1 << 30):
        x[a:min(n, a + (1 << 30))].normal_(generator=g)
    x[n - 3:n - 2].fill_(7.5)  # the absmax sits in the tail
    q, s = ops.encode(x, 8)
    spans = [(0, 4096), ((1 << 31) - 4096, (1 << 31) + 4096), (n - 4096, n)]

    def sample(t):
        return np.concatenate([t[a:b].cpu().numpy() for a, b in spans])
    xs, qs = sample(x), sample(q)
    scale = np.float32(s.item())
    assert scale == np.float32(7.5) / np.float32(127)
    with np.errstate(all="ignore"):
        y = xs * (np.float32(1) / scale)
        want = np.rint(np.clip(y, -128, 127)).astype(np.int8)
    assert np.array_equal(qs, want)
    d = ops.decode(q, s)
    assert np.array_equal(sample(d), (qs.astype(np.float32) * scale).astype(np.float32))
    del d
    p, s4 = ops.encode_int4(x, 4)
    d4 = ops.decode_int4(p, n, s4)
    assert np.float32(s4.item()) == np.float32(7.5) / np.float32(7)
    got = sample(d4)
    with np.errstate(all="ignore"):
        q4 = np.rint(np.clip(xs * (np.float32(1) / np.float32(s4.item())), -128, 127)).astype(np.int8)
    assert np.array_equal(got, (q4.astype(np.float32) * np.float32(s4.item())).astype(np.float32))
    del x, q, p, d4
