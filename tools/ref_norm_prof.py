"""Driver for rocprofv3 kernel traces of stoch.reference_norms: C2 (2^28 fp32) and C3 (256 equal tensors),
`--reps` launches each, so the per-kernel split of the phased norm shows in the stats.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python tools/ref_norm_prof.py [--dtype f32]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd import ops, stoch  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}

p = argparse.ArgumentParser()
p.add_argument("--reps", type=int, default=5)
p.add_argument("--dtype", default="f32")
p.add_argument("--cfg", default="c2,c3")
p.add_argument("--reps-only", action="store_true")
a = p.parse_args()
dev = torch.device("cuda", 0)
base, rem = divmod(11_689_512, 256)
cfgs = {"c2": ops.BucketLayout([1 << 28], align=1),
        "c3": ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)], align=1)}
g = torch.Generator(device=dev).manual_seed(0)
for name in a.cfg.split(","):
    lay = cfgs[name]
    x = (torch.randn(lay.total, device=dev, generator=g) * 1e-3).to(DT[a.dtype])
    for _ in range(a.reps):
        stoch.reference_norms(x, lay)
    torch.cuda.synchronize()
    print(name, "done", flush=True)
