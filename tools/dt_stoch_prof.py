"""Driver for kernel traces / SQ counters of the fp16 / bf16 / fp64 stochastic encodes (csrc/stoch_dtype.hip) on
C3's equal layout (256 x 45,662 elements), `--reps` launches of each (codec, dtype):

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -- python3 tools/dt_stoch_prof.py [--codecs cnat,qsgd]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd import ops, stoch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--reps", type=int, default=5)
p.add_argument("--codecs", default="cnat,qsgd")
p.add_argument("--dtypes", default="f16,bf16,f64")
a = p.parse_args()
DT = {"f16": torch.float16, "bf16": torch.bfloat16, "f64": torch.float64}
dev = torch.device("cuda", 0)
base, rem = divmod(11_689_512, 256)
lay = ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)], align=1)
g = torch.Generator(device=dev).manual_seed(0)
x32 = torch.randn(lay.total, device=dev, generator=g) * 1e-3
lv = torch.empty(lay.total, dtype=torch.uint8, device=dev)
sg = torch.empty(lay.total, dtype=torch.int8, device=dev)
for dn in a.dtypes.split(","):
    x = x32.to(DT[dn])
    for codec in a.codecs.split(","):
        for _ in range(a.reps):
            stoch.encode_batched_dt(codec, x, lay, 8, seed=7, counter=0,
                                    levels=lv.view(torch.int8) if codec == "cnat" else lv, signs=sg)
        torch.cuda.synchronize()
        print(dn, codec, "done", flush=True)
