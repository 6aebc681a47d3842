"""SLQChannel / QSGDChannel on a device-resident ResNet-18-sized state dict (256 weights + 256 biases on
cuda:0): on_client_send + on_server_receive wall time (host-side cost of the per-tensor payload objects)."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "ad-federatedlearning_amd"))
from adfl_amd.Channel import QSGDChannel, SLQChannel  # noqa: E402

RESNET18 = 11_689_512


def main():
    dev = torch.device("cuda", 0)
    base, rem = divmod(RESNET18, 256)
    g = torch.Generator(device=dev).manual_seed(0)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), device=dev, generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, device=dev, generator=g) * 1e-3
    res = {}
    for name, ch in (("slq", SLQChannel(8)), ("qsgd", QSGDChannel(8))):
        enc, dec = [], []
        for it in range(13):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            qp, _ = ch.on_client_send(params)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            d, _ = ch.on_server_receive(qp)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if it >= 3:
                enc.append((t1 - t0) * 1e3)
                dec.append((t2 - t1) * 1e3)
        res[name] = {"encode_ms": round(min(enc), 3), "decode_ms": round(min(dec), 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
