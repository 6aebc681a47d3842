"""cProfile of SLQChannel's host path on the C3 dict (where the host-side milliseconds go)."""
import cProfile
import os
import pstats
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd.Channel import SLQChannel  # noqa: E402

base, rem = divmod(11_689_512, 256)
params = {}
for i in range(256):
    params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0)) * 1e-3
    params[f"layer{i}.bias"] = torch.randn(64)
ch = SLQChannel(8)
for _ in range(3):
    qp, _ = ch.on_client_send(params)
    d, _ = ch.on_server_receive(qp)
for what, fn in (("encode", lambda: ch.on_client_send(params)), ("decode", lambda: ch.on_server_receive(qp))):
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        fn()
    pr.disable()
    print("=====", what, "(10 calls)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)
