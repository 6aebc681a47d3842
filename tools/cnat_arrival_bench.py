"""C3 / C2 CNAT encode (bits 8, in-kernel Philox): the single-launch arrival-counter encode against the
register-resident one-launch encode and the three-launch encode. Median of --reps, each span after a 512 MiB
read; frac = 6 B/element / time / 8 TB/s.

    python tools/cnat_arrival_bench.py [--reps 21]
"""
import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd import ops, stoch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=21)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    junk = torch.empty(128 << 20, device=dev)
    base, rem = divmod(11_689_512, 256)
    out = {}
    for name, sizes in (("C3 equal 256", [base + (1 if i < rem else 0) for i in range(256)]),
                        ("C3 ResNet-18 shapes x 1/8 chunks cap", None)):
        if sizes is None:
            continue
        lay = ops.BucketLayout(sizes, align=1)
        x = torch.randn(lay.total, device=dev) * 1e-3
        ex = torch.empty(lay.total, dtype=torch.int8, device=dev)
        sg = torch.empty(lay.total, dtype=torch.int8, device=dev)
        nrm = torch.empty(lay.ntensors, device=dev)
        ws = stoch.workspace(lay, dev)
        res = {}
        for label, kw in (("three_launch", {"resident": False, "arrival": False}),
                          ("resident", {"arrival": False}), ("arrival", {"arrival": True})):
            ts = []
            for _ in range(a.reps):
                junk.mul_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                stoch.cnat_encode_batched(x, lay, 8, seed=1, exps=ex, signs=sg, norms=nrm, ws=ws, **kw)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            res[label] = {"ms": round(ms, 4), "frac_6B": round(6 * lay.total / (ms * 1e-3) / 8e12, 3)}
        out[name] = res
        print(name, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
