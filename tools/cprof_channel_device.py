"""cProfile of SLQChannel on a device-resident ResNet-18-sized state dict (what tools/prof_channel_device.py
times): where the host-side time of a device round trip goes, by function."""
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ad-federatedlearning_amd"))
from adfl_amd.Channel import SLQChannel  # noqa: E402

RESNET18 = 11_689_512


def main():
    dev = torch.device("cuda", 0)
    base, rem = divmod(RESNET18, 256)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), device=dev) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, device=dev) * 1e-3
    ch = SLQChannel(8)
    for _ in range(3):
        ch.on_server_receive(ch.on_client_send(params)[0])
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        ch.on_server_receive(ch.on_client_send(params)[0])
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(s.getvalue())


if __name__ == "__main__":
    main()
