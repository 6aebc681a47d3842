"""CPU: the channel's process-wide glibc tuning (hostcopy.keep_host_heap) is bounded by its working set.

A fresh process runs 50 rounds of a C3-sized host decode's allocation pattern — 256 owned fp32 outputs of a
ResNet-18-like layout (11.7 M elements, 46.8 MB) allocated, filled by the native scatter, handed out and
dropped — with the heap settings the channel applies for that layout. Its RSS growth over the rounds stays
within 2x the working set, the thresholds are the sized ones (mmap: the largest output rounded up to a power
of two; trim: 2x the working set), they are only raised, and ADFL_KEEP_HOST_HEAP=0 leaves glibc untouched.
"""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ad-federatedlearning_amd"))
import numpy as np, torch
from adfl_amd import hostcopy

def rss():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) * 1024

rng = np.random.default_rng(0)
sizes = np.exp(rng.uniform(np.log(64), np.log(2_400_000), 256)).astype(np.int64)
sizes = (sizes * (11_689_512 / sizes.sum())).astype(np.int64) + 1
total, largest = int(sizes.sum()), int(sizes.max())
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
src = torch.randn(total)
ws = 4 * total
hostcopy.keep_host_heap(ws, 4 * largest)
hostcopy.keep_host_heap(ws // 4, 4 * largest // 4)   # a smaller layout later: never lowered
base = None
for r in range(50):
    outs = [torch.empty(int(n)) for n in sizes]
    hostcopy.scatter(src, outs, offs)
    del outs
    if r == 1:
        base = rss()
print(json.dumps({"ws": ws, "largest": 4 * largest, "growth": rss() - base, **hostcopy.heap_settings()}))
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    out = subprocess.run([sys.executable, "-c", _CHILD, REPO], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_heap_settings_are_sized_and_bounded():
    r = _run({})
    mmap = 128 << 10
    while mmap < min(r["largest"], 32 << 20):
        mmap <<= 1
    assert r["mmap"] == mmap and r["trim"] == min(2 * r["ws"], 1 << 30)
    assert r["growth"] <= 2 * r["ws"], r


def test_heap_opt_out_leaves_glibc_alone():
    r = _run({"ADFL_KEEP_HOST_HEAP": "0"})
    assert r["mmap"] == 0 and r["trim"] == 0
    assert r["growth"] <= 2 * r["ws"], r


@pytest.mark.parametrize("ws,largest,mmap", [(1000, 100, 128 << 10), (1 << 20, 300 << 10, 512 << 10),
                                              (10 << 30, 1 << 30, 32 << 20)])
def test_threshold_rounding(ws, largest, mmap):
    code = ("import os,sys; sys.path.insert(0, os.path.join(sys.argv[1], 'ad-federatedlearning_amd')); "
            "from adfl_amd import hostcopy; import json; "
            f"hostcopy.keep_host_heap({ws}, {largest}); print(json.dumps(hostcopy.heap_settings()))")
    out = subprocess.run([sys.executable, "-c", code, REPO], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["mmap"] == mmap and r["trim"] == min(2 * ws, 1 << 30)
