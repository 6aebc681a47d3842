"""The bench line's host-to-host C3 dict leg (SLQChannel(8) on 256 weights + 256 biases, CPU in / CPU out) for a
trace (`--channel QSGDChannel` etc. for the other codecs): warm-up calls, then `--calls` encode + decode pairs with a hipDeviceSynchronize-free marker between them
(a 1-element H2D copy of a recognisable size), so the copies, kernels and HIP API calls of one call can be cut
out of a rocprofv3 trace:

    rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/hdt \
        -- python3 tools/host_dict_trace.py
    python3 tools/host_dict_trace_summary.py gpurun_out/hdt
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
import importlib  # noqa: E402
C = importlib.import_module("adfl_amd.Channel")

MARK_BYTES = 12345 * 4   # the marker copy's size (fp32 elements * 4)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--calls", type=int, default=6)
    p.add_argument("--channel", default="SLQChannel", help="SLQChannel, QSGDChannel, CNATChannel, ...")
    args = p.parse_args()
    base, rem = divmod(11_689_512, 256)
    g = torch.Generator().manual_seed(0)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
    ch = getattr(C, args.channel)(8)
    for _ in range(5):
        qp, _ = ch.on_client_send(params)
        ch.on_server_receive(qp)
    mark = torch.zeros(MARK_BYTES // 4).pin_memory()
    mark_dev = torch.empty(MARK_BYTES // 4, device="cuda:0")
    walls = []
    for _ in range(args.calls):
        mark_dev.copy_(mark, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        qp, _ = ch.on_client_send(params)
        t1 = time.perf_counter()
        mark_dev.copy_(mark, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ch.on_server_receive(qp)
        t3 = time.perf_counter()
        walls.append(((t1 - t0) * 1e3, (t3 - t2) * 1e3))
    for e, d in walls:
        print(f"encode {e:.3f} ms  decode {d:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
