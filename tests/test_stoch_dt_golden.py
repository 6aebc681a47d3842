"""CPU: the fp16 / bf16 / fp64 stochastic-codec oracle (oracle/stoch_dt_oracle.py) against the reference's
own outputs on tensors of those dtypes.

tests/golden/stoch_dt.npz was produced by executing the reference QSGD / RQSGD / CNAT channels
(Src/ADFL/Channel/quant.py:140-570) on fp16 / bf16 / fp64 tensors with recorded uniforms of the tensor's
dtype in place of torch.rand_like (tests/golden/make_golden_stoch_dt.py). Given the reference's norm and
the same uniforms, every level / exponent byte, sign and decoded float must match bit for bit; the oracle's
norms must equal torch's within torch's own accumulation error (max / min exactly).
"""

import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from golden_util import same_f32

import stoch_dt_oracle as do

MANIFEST = json.load(open(os.path.join(GOLDEN, "stoch_dt_manifest.json")))
ARR = np.load(os.path.join(GOLDEN, "stoch_dt.npz"))
CASES = MANIFEST["cases"]
DT = {"float16": do.DT_F16, "bfloat16": do.DT_BF16, "float64": do.DT_F64}


def scale_value(rec) -> float:
    if "int" in rec:
        return float(rec["int"])
    if rec.get("tensor"):
        return float(rec["value"])
    return float(np.array([rec["f64_bits"]], np.uint64).view(np.float64)[0])


def load_case(c):
    n = c["name"]
    return (ARR[f"{n}__x"], ARR[f"{n}__u"], ARR[f"{n}__q"], ARR[f"{n}__signs"], ARR[f"{n}__deq"],
            scale_value(c["scale"]), scale_value(c["scale_2"]))


def test_fixture_covers_every_codec_and_dtype():
    seen = {(c["codec"], c["dtype"]) for c in CASES}
    assert seen == {(k, d) for k in ("qsgd", "rqsgd", "cnat") for d in DT}
    assert all(c["rand_calls"] in (0, 1) for c in CASES)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference(c):
    x, u, q_ref, s_ref, d_ref, norm, scale2 = load_case(c)
    dt = DT[c["dtype"]]
    q, s = do.quantize(c["codec"], x, dt, c["bits"], norm, u)
    assert str(q.dtype) == c["q_dtype"]
    np.testing.assert_array_equal(q.view(np.uint8), q_ref)
    np.testing.assert_array_equal(s, s_ref)
    d = do.decode(c["codec"], q_ref, s_ref, c["bits"], norm, scale2)
    assert same_f32(d.reshape(d_ref.shape), d_ref)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_norms(c):
    """max / min norms exactly; L2 within torch's accumulation error (rounded to the dtype: at most one
    ulp of the dtype apart, or equal)."""
    x, _, _, _, _, norm, scale2 = load_case(c)
    dt = DT[c["dtype"]]
    if c["codec"] == "rqsgd":
        mine, mn = do.linf_norm(x, dt), do.lminf_norm(x, dt)
        if np.isnan(norm):
            assert np.isnan(mine)
        else:
            assert mine == norm
            if c["scale"].get("tensor") is None:
                assert (np.isnan(mn) and np.isnan(scale2)) or mn == scale2
        return
    mine = do.l2_norm(x, dt)
    if np.isnan(norm) or np.isinf(norm):
        assert (np.isnan(mine) and np.isnan(norm)) or mine == norm
        return
    if norm == 0:
        assert mine == 0
        return
    n = x.size
    if dt == do.DT_F64:
        assert abs(mine - norm) <= (n + 2) * 2.0 ** -52 * norm
    else:
        ulp = 2.0 ** -10 if dt == do.DT_F16 else 2.0 ** -7
        assert abs(mine - norm) <= ulp * norm * 1.01, (mine, norm)


def test_uniform_grids():
    """The Philox stream for these dtypes draws from torch.rand's grid for the dtype, in [0, 1)."""
    for dt, g in ((do.DT_F16, 11), (do.DT_BF16, 8), (do.DT_F64, 53)):
        u = do.to_compute(do.philox_uniforms_dt(dt, 4096, 1234, 5), dt).astype(np.float64)
        assert (u >= 0).all() and (u < 1).all()
        assert np.array_equal(u * 2.0 ** g, np.floor(u * 2.0 ** g))
        assert abs(u.mean() - 0.5) < 0.03
        # a prefix of a longer draw is the shorter draw; an offset start continues the stream
        v = do.philox_uniforms_dt(dt, 10, 1234, 5, start=7)
        assert np.array_equal(do.philox_uniforms_dt(dt, 17, 1234, 5)[7:], v)
