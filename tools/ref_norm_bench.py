"""Device time of the reference-order L2 norm (stoch.reference_norms, csrc/torch_norm.hip) on C2 / C3 for each
dtype, against the fp64 norm (fp32), and the QSGD / CNAT encodes with either norm.

    python tools/ref_norm_bench.py [--reps 21] [--dtypes f32,bf16,f16,f64]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from adfl_amd import ops, stoch  # noqa: E402
import recipes  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=21)
    p.add_argument("--dtypes", default="f32,bf16,f16,f64")
    p.add_argument("--cfgs", default="", help="comma-separated substrings of the config names to run (default all)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    junk = torch.empty(128 << 20, device=dev)
    base, rem = divmod(11_689_512, 256)
    rng = np.random.default_rng(33)
    logu = np.exp(rng.uniform(np.log(64), np.log(2_400_000), 256)).astype(np.int64)
    cfgs = {"C2 flat 2^28": ops.BucketLayout([1 << 28], align=1),
            "C3 equal 256": ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)], align=1),
            "C3 log-uniform 256": ops.BucketLayout(recipes.bucket_sizes("loguniform"), align=64),
            "C3 log-uniform unscaled 256": ops.BucketLayout(logu.tolist(), align=64)}
    g = torch.Generator(device=dev).manual_seed(0)

    def timed(fn):
        ts = []
        for _ in range(a.reps):
            junk.mul_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return round(statistics.median(ts), 4)

    res = {}
    for name, lay in cfgs.items():
        if a.cfgs and not any(k in name for k in a.cfgs.split(",")):
            continue
        x32 = torch.randn(lay.total, device=dev, generator=g) * 1e-3
        for dn in a.dtypes.split(","):
            x = x32.to(DT[dn])
            out = {}
            n64 = torch.empty(lay.ntensors, dtype=torch.float64, device=dev)
            out["reference_norms_ms"] = timed(lambda: stoch.reference_norms(x, lay, out64=n64))
            if dn == "f32":
                nrm = torch.empty(lay.ntensors, device=dev)
                ws = stoch.workspace(lay, dev)
                out["default_fp64_norm_ms"] = timed(lambda: stoch.norms_batched(x, lay, stoch.NORM_L2, norms=nrm, ws=ws))
                qs = torch.empty(lay.total, dtype=torch.uint8, device=dev)
                sg = torch.empty(lay.total, dtype=torch.int8, device=dev)
                for tn in (False, True):
                    k = "reference" if tn else "fp64"
                    out[f"qsgd_encode_{k}_norm_ms"] = timed(lambda: stoch.qsgd_encode_batched(
                        x, lay, 8, seed=1, levels=qs, signs=sg, norms=nrm, ws=ws, torch_norm=tn))
                    out[f"cnat_encode_{k}_norm_ms"] = timed(lambda: stoch.cnat_encode_batched(
                        x, lay, 8, seed=1, exps=qs.view(torch.int8), signs=sg, norms=nrm, ws=ws, torch_norm=tn))
            res[f"{name} {dn}"] = out
            print(name, dn, json.dumps(out), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
