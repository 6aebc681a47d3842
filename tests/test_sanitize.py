"""CPU: the native host code under sanitizers (tools/sanitize/run.sh) — the staging-copy pool with ASan +
UBSan and with TSan (concurrent callers), the oracle's C with ASan + UBSan, and tests/test_hostcopy.py
against an ASan build of the pool. No GPU: the HIP kernels are not part of it (GPU ASan is not available)."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_code_is_sanitizer_clean(tmp_path):
    env = dict(os.environ, SAN_OUT=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "sanitize", "run.sh")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "0 mismatches" in r.stdout and "sanitizers: clean" in r.stdout
