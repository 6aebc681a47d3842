"""CPU: the binade-integer model behind the tile-parallel reference-order L2 norm (csrc/torch_norm_lb.h).

tools/torch_norm_proto.c restates, in plain C, what k_norm_torch does per tile: a run of steps adds the
integer sum of R(x^2 / u) in the accumulator's binade, with ties, crossings and non-finite values falling
back to fmaf. It checks the model against torch's sequential 8-chain loop (the oracle's
oracle_torch_l2_norm order) on 402 cases — random, integer and bf16-rounded data full of ties, constants,
2^+-60 scales, subnormal and overflowing squares, NaN / inf — both with the exact grid and with the
kernel's fp64-prefix predictor. Compiled and run here with gcc."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_binade_integer_model_is_bit_identical(tmp_path):
    exe = tmp_path / "torch_norm_proto"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(REPO, "tools", "torch_norm_proto.c"), "-lm"],
                   check=True)
    r = subprocess.run([str(exe), str(1 << 20)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "all bit-identical to the sequential chain (0 bad)" in r.stdout
