"""CPU, only where the reference tree exists (the build container; skipped on the GPU box): the drop-in
claims that need the real ADFL modules in the same process.

* With ADFL loaded first, adfl_amd's payload dataclasses ARE ADFL's classes, so the reference's own
  `assert isinstance(c_params, ...)` checks accept our payloads;
* the reference's IdentityChannel decodes what ours encodes and vice versa (USLQ's fp32 direction);
* bandwidth accounting and to_json agree on random state dicts (not just the golden one);
* adfl_amd.compression exposes the reference compression.py's hot-path functions with its parameter names.
Runs in a subprocess so the ADFL stubs never leak into other tests."""

import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
from ref_loader import reference_available  # noqa: E402

pytestmark = pytest.mark.skipif(not reference_available(), reason="reference tree not present")

CODE = r"""
import sys, torch
sys.path[:0] = [{golden!r}, {pkg!r}]
from ref_loader import load_reference
ref = load_reference()                      # ADFL.model etc. now in sys.modules
import adfl_amd
from adfl_amd import model
from adfl_amd.Channel import IdentityChannel, SLQChannel, USLQChannel
assert model.QuantParameter is ref.model.QuantParameter
assert model.QuantParameters is ref.model.QuantParameters
assert model.ByteParameters is ref.model.ByteParameters
torch.manual_seed(0)
for trial in range(20):
    params = {{}}
    for i in range(int(torch.randint(1, 8, (1,)))):
        nd = int(torch.randint(0, 4, (1,)))
        shape = tuple(int(s) for s in torch.randint(1, 6, (nd,)))
        params[f"p{{i}}"] = torch.randn(shape) if nd else torch.tensor(3, dtype=torch.int64)
    for bits in (8, 4, 2):
        assert SLQChannel(bits).simulate_bandwidth(params, 1e12) == ref.quant.SLQChannel(bits).simulate_bandwidth(params, 1e12)
        assert USLQChannel(bits).to_json() == ref.quant.USLQChannel(bits).to_json()
    ours, theirs = IdentityChannel(no_compute_time=True), ref.channel.IdentityChannel(no_compute_time=True)
    b_ours, _ = ours.on_server_send(params)
    b_theirs, _ = theirs.on_server_send(params)
    assert b_ours.size == b_theirs.size
    for name, p in params.items():
        assert b_ours.params[name].data == b_theirs.params[name].data
    back, _ = theirs.on_client_receive(b_ours)                 # reference decodes ours
    back2, _ = ours.on_client_receive(b_theirs)                # ours decodes the reference's
    for name, p in params.items():
        assert torch.equal(back[name], p) and torch.equal(back2[name], p)
    assert model.get_parameter_info(params) == ref.model.get_parameter_info(params)
# adfl_amd.compression: the reference's hot-path functions under the same names and parameter names
import inspect
from adfl_amd import compression
for fn in ("quantize_tensor", "dequantize_tensor", "pack_4bit", "unpack_4bit"):
    assert list(inspect.signature(getattr(compression, fn)).parameters) == \
        list(inspect.signature(getattr(ref.compression, fn)).parameters), fn
print("dropin ok")
"""


def test_dropin_with_reference_loaded():
    code = CODE.format(golden=os.path.join(HERE, "golden"), pkg=os.path.join(REPO, "ad-federatedlearning_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "dropin ok" in r.stdout
