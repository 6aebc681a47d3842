"""C5 int4 round trip (2^30 fp32) per kernel under different device allocation orders of x / packed / out.

The same kernels measured 0.78 ms (quantize+pack) in tools/microbench_c5.hip (hipMalloc'd buffers) and
0.88 ms in tools/bench_configs.py --mode c5_int4 (torch's caching allocator). This runs the bench's
timing loop over several placements in one process to find which placement the difference follows.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ad-federatedlearning_amd"))
from adfl_amd import _lib, ops  # noqa: E402


def run(name, x, packed, out, lib, sh, steps=15):
    n = x.numel()
    scale = torch.empty(1, device=x.device)
    ws = ops.new_workspace(x.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    seg = [[], [], []]
    for s in range(steps + 3):
        ev[0].record()
        _lib.check(lib.adfl_slq_absmax(x.data_ptr(), n, ws.data_ptr(), ws.numel(), sh))
        ev[1].record()
        _lib.check(lib.adfl_slq_quantize_int4(x.data_ptr(), n, 4, ws.data_ptr(), packed.data_ptr(), scale.data_ptr(), sh))
        ev[2].record()
        _lib.check(lib.adfl_slq_dequantize_int4(packed.data_ptr(), n, scale.data_ptr(), out.data_ptr(), sh))
        ev[3].record()
        torch.cuda.synchronize()
        if s >= 3:
            for i in range(3):
                seg[i].append(ev[i].elapsed_time(ev[i + 1]))
    med = [sorted(v)[len(v) // 2] for v in seg]
    base = min(x.data_ptr(), packed.data_ptr(), out.data_ptr())
    print(json.dumps({"placement": name, "absmax": round(med[0], 4), "quantize_int4": round(med[1], 4),
                      "dequantize_int4": round(med[2], 4),
                      "x_off_MiB": (x.data_ptr() - base) / 2**20, "packed_off_MiB": (packed.data_ptr() - base) / 2**20,
                      "out_off_MiB": (out.data_ptr() - base) / 2**20}), flush=True)


def main():
    n = 1 << 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    sh = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)

    # A: as tools/bench_configs.py (randn's output freed by the multiply; packed carved from it)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    packed = torch.empty((n + 1) // 2, dtype=torch.uint8, device=dev)
    out = torch.empty(n, device=dev)
    run("A bench order", x, packed, out, lib, sh)
    ref = packed.clone()
    xs = x.clone()
    del x, packed, out
    torch.cuda.empty_cache()

    # B: packed first, then x, then out (fresh allocations only)
    packed = torch.empty((n + 1) // 2, dtype=torch.uint8, device=dev)
    x = xs.clone()
    out = torch.empty(n, device=dev)
    del xs
    torch.cuda.empty_cache()
    run("B packed first", x, packed, out, lib, sh)
    assert torch.equal(packed, ref)

    # C: packed in its own 4 GiB allocation's head, x and out fresh
    big = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    pk = big[: (n + 1) // 2]
    run("C packed in own 4 GiB block", x, pk, out, lib, sh)
    assert torch.equal(pk, ref)

    # D: packed in the middle of a 4 GiB block (2 GiB offset)
    pk = big[2 << 30: (2 << 30) + (n + 1) // 2]
    run("D packed at +2 GiB of own block", x, pk, out, lib, sh)
    del big, pk
    torch.cuda.empty_cache()

    # E: bench order again (reproducibility of A)
    x2 = x.clone() * 1.0
    del x
    packed = torch.empty((n + 1) // 2, dtype=torch.uint8, device=dev)
    run("E bench-like again", x2, packed, out, lib, sh)


if __name__ == "__main__":
    main()
