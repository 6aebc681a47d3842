"""cProfile of SLQChannel on a ResNet-18-sized state dict — device-resident (what tools/prof_channel_device.py
times), or with --host a CPU dict (ADFL's own call pattern): where the host-side time goes, by function."""
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
    dev = torch.device("cpu") if "--host" in sys.argv else torch.device("cuda", 0)
    base, rem = divmod(RESNET18, 256)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), device=dev) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, device=dev) * 1e-3
    ch = SLQChannel(8)
    for _ in range(3):
        ch.on_server_receive(ch.on_client_send(params)[0])
    qp = ch.on_client_send(params)[0]
    for what, fn in (("encode", lambda: ch.on_client_send(params)), ("decode", lambda: ch.on_server_receive(qp))):
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(10):
            fn()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(14)
        print("==", what)
        print(s.getvalue())


if __name__ == "__main__":
    main()
