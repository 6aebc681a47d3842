"""Driver for rocprofv3 kernel traces of stoch.reference_norms: C2 (2^28 fp32), C3 (256 equal tensors) and
C3 log-uniform (c3lu),
`--reps` launches each, so the per-kernel split of the phased norm shows in the stats.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python tools/ref_norm_prof.py [--dtype f32]
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from adfl_amd import ops, stoch  # noqa: E402
import recipes  # noqa: E402

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
        "c3": ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)], align=1),
        # C3's log-uniform layout (sizes in [64, 2.4 M] scaled to sum 11,689,512; tests/golden/recipes.py)
        "c3lu": ops.BucketLayout(recipes.bucket_sizes("loguniform"), align=64),
        # the unscaled draw rounds 4-5 quoted as "C3 log-uniform" (seed 33; 47.7 M elements, up to 2.37 M per tensor)
        "c3lu_raw": ops.BucketLayout(np.exp(np.random.default_rng(33).uniform(np.log(64), np.log(2_400_000), 256))
                                     .astype(np.int64).tolist(), align=64)}
g = torch.Generator(device=dev).manual_seed(0)
for name in a.cfg.split(","):
    lay = cfgs[name]
    x = (torch.randn(lay.total, device=dev, generator=g) * 1e-3).to(DT[a.dtype])
    for _ in range(a.reps):
        stoch.reference_norms(x, lay)
    torch.cuda.synchronize()
    print(name, "done", flush=True)
