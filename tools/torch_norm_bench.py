"""Cost of the reference-order L2 norm against the default (fp64) one on C2 and C3, device-resident.

Times (median of --reps, each after a 512 MiB read so x comes from HBM) of:
  norm      norms_batched NORM_L2 (default) | torch_norms (look-back) | NORM_L2_TORCH (one block per tensor, in order)
  encode    qsgd_encode_batched / cnat_encode_batched with torch_norm False | True (bits 8, in-kernel Philox)

    python tools/torch_norm_bench.py [--reps 21] [--no-seq]
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
    p.add_argument("--no-seq", action="store_true", help="skip the sequential kernel (slow on C2)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    junk = torch.empty(128 << 20, device=dev)
    base, rem = divmod(11_689_512, 256)
    cfgs = {"C2 flat 2^28": ops.BucketLayout([1 << 28], align=1),
            "C3 equal 256": ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)], align=1)}
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, lay in cfgs.items():
        x = torch.randn(lay.total, device=dev, generator=g) * 1e-3
        out = {}

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

        ws = stoch.workspace(lay, dev)
        nrm = torch.empty(lay.ntensors, device=dev)
        out["norm_default_ms"] = timed(lambda: stoch.norms_batched(x, lay, stoch.NORM_L2, norms=nrm, ws=ws))
        out["norm_torch_lookback_ms"] = timed(lambda: stoch.torch_norms(x, lay, norms=nrm))
        key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
        scr = stoch._TORCH_NORM_SCRATCH[key]
        scr[32:64].zero_()
        stoch.torch_norms(x, lay, norms=nrm)
        cnt = scr[24:64].cpu().view(torch.int64).tolist()
        out["lookback_error_retries_sequential_notfound_bad"] = cnt
        ref = stoch.norms_batched(x, lay, stoch.NORM_L2_TORCH)[0].clone()
        got = stoch.torch_norms(x, lay)
        out["lookback_equals_sequential"] = bool(torch.equal(ref.view(torch.int32), got.view(torch.int32)))
        if not a.no_seq or lay.ntensors > 1:
            out["norm_torch_sequential_ms"] = timed(lambda: stoch.norms_batched(x, lay, stoch.NORM_L2_TORCH, norms=nrm))
        lv = torch.empty(lay.total, dtype=torch.uint8, device=dev)
        sg = torch.empty(lay.total, dtype=torch.int8, device=dev)
        ex = torch.empty(lay.total, dtype=torch.int8, device=dev)
        for tn in (False, True):
            k = "torch" if tn else "default"
            out[f"qsgd_encode_{k}_ms"] = timed(lambda: stoch.qsgd_encode_batched(
                x, lay, 8, seed=1, levels=lv, signs=sg, norms=nrm, ws=ws, torch_norm=tn))
            out[f"cnat_encode_{k}_ms"] = timed(lambda: stoch.cnat_encode_batched(
                x, lay, 8, seed=1, exps=ex, signs=sg, norms=nrm, ws=ws, torch_norm=tn))
        # the quantize alone, given the norms (the part of a torch_norm=True QSGD encode after the norm)
        tn = stoch.torch_norms(x, lay)
        out["qsgd_quantize_given_norms_ms"] = timed(lambda: stoch.qsgd_quantize_batched(
            x, lay, 8, tn, seed=1, levels=lv, signs=sg))
        for c in ("qsgd", "cnat"):
            out[f"{c}_torch_over_default"] = round(out[f"{c}_encode_torch_ms"] / out[f"{c}_encode_default_ms"], 4)
        res[name] = out
        print(name, json.dumps(out), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
