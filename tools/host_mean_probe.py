"""receive_mean of K client updates of the C3 CPU dict (256 weights + 256 biases), host to host: the
synchronous server aggregate (Src/ADFL/Strategy/simple.py:83-89). Prints the minimum and median wall time over
`--steps` calls and a cProfile of a few more, per channel.

    python tools/host_mean_probe.py [--k 4] [--steps 10] [--channels SLQChannel,QSGDChannel]
"""
import argparse
import cProfile
import importlib
import os
import pstats
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
C = importlib.import_module("adfl_amd.Channel")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=4)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--channels", default="SLQChannel,QSGDChannel")
    a = p.parse_args()
    base, rem = divmod(11_689_512, 256)
    for name in a.channels.split(","):
        ch = getattr(C, name)(8)
        ups = []
        for k in range(a.k):
            g = torch.Generator().manual_seed(k)
            params = {}
            for i in range(256):
                params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
                params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
            ups.append(ch.on_client_send(params)[0])
        for _ in range(3):
            ch.receive_mean(ups)
        ts = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            ch.receive_mean(ups)
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"{name} K={a.k}: receive_mean min {min(ts):.3f} ms, median {statistics.median(ts):.3f} ms", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(5):
            ch.receive_mean(ups)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main()
