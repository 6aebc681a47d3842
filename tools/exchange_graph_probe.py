"""Probe: can the RCCL peer exchange (encode -> all_gather_into_tensor -> fused decode-mean) be captured in
one HIP graph, and what does a replay cost against the eager call? World 1 over RCCL on one GPU, C3 bucket
layout (11.7 M fp32 in 256 tensors) and a flat 2^24 update.

    python tools/exchange_graph_probe.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)
from bench import free_port  # noqa: E402


def main():
    import recipes
    from adfl_amd import ops
    from adfl_amd.exchange import PeerExchange
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                            device_id=dev)
    res = {}
    for name, layout, n in (("c3_equal", ops.BucketLayout(recipes.bucket_sizes("equal")), None),
                            ("flat_2^24", None, 1 << 24)):
        n = layout.total if layout is not None else n
        ex = PeerExchange(n, bits=8, device=dev, layout=layout)
        x = torch.randn(n, device=dev) * 1e-3
        out = torch.empty(n, device=dev)
        want = ex.exchange_mean(x).clone()
        for _ in range(5):
            ex.exchange_mean(x, out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            ex.exchange_mean(x, out)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / 200 * 1e3
        r = {"eager_ms": round(eager, 4)}
        try:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                ex.exchange_mean(x, out)   # warm the capture stream
                with torch.cuda.graph(g):
                    ex.exchange_mean(x, out)
            torch.cuda.current_stream().wait_stream(side)
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
            r["graph_equal"] = bool(torch.equal(out, want))
            t0 = time.perf_counter()
            for _ in range(200):
                g.replay()
            torch.cuda.synchronize()
            r["graph_ms"] = round((time.perf_counter() - t0) / 200 * 1e3, 4)
        except Exception as e:  # noqa: BLE001
            r["graph_error"] = f"{type(e).__name__}: {e}"[:300]
        res[name] = r
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
