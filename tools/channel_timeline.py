"""Wall-clock timeline of one SLQChannel host-to-host call on the C3 CPU dict (256 weights + 256 biases): each
internal phase wrapped with perf_counter stamps (no extra synchronisation), medians over the calls.

    python tools/channel_timeline.py [--calls 30]
"""
import argparse
import json
import os
import statistics
import sys
import time
from collections import defaultdict

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd import hostcopy  # noqa: E402
from adfl_amd.Channel import SLQChannel  # noqa: E402
from adfl_amd.Channel import quant  # noqa: E402

STAMPS = []


def wrap(obj, name, label):
    fn = getattr(obj, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            STAMPS.append((label, t0, time.perf_counter()))
    setattr(obj, name, w)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--calls", type=int, default=30)
    p.add_argument("--no-pipeline", action="store_true", help="quant._PIPELINE off (create all outputs, then scatter)")
    args = p.parse_args()
    if args.no_pipeline:
        quant._PIPELINE = False
    for obj, name, label in [(quant, "_stage_in", "stage_in (gather + H2D enqueue)"),
                             (quant.ops, "encode_batched", "encode kernel enqueue"),
                             (quant.ops, "decode_batched", "decode kernel enqueue"),
                             (quant._PendingD2H, "__init__", "D2H enqueue"),
                             (quant._PendingD2H, "finish", "wait D2H + scatter"),
                             (quant._PendingD2H, "finish_building", "create outputs + pipelined scatter"),
                             (hostcopy, "advise_huge", "advise_huge"),
                             (hostcopy.Pending, "wait", "native job wait"),
                             (quant, "_host_scales", "host scales (range landed, H2D enqueued)"),
                             (quant, "_encode_dict", "_encode_dict"),
                             (quant, "_decode_dict", "_decode_dict"),
                             (torch.cuda.Event, "synchronize", "event sync")]:
        wrap(obj, name, label)
    base, rem = divmod(11_689_512, 256)
    g = torch.Generator().manual_seed(0)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
    ch = SLQChannel(8)
    for _ in range(5):
        qp, _ = ch.on_client_send(params)
        ch.on_server_receive(qp)
    res = {}
    for what in ("encode", "decode"):
        per = defaultdict(list)
        totals, frees = [], []
        for _ in range(args.calls):
            STAMPS.clear()
            t0 = time.perf_counter()
            if what == "encode":
                r = ch.on_client_send(params)
            else:
                r = ch.on_server_receive(qp)
            t1 = time.perf_counter()
            if what == "encode":
                qp = r[0]
            del r   # the previous result's tensors are freed here (encode: the old payload), outside the call
            frees.append((time.perf_counter() - t1) * 1e3)
            totals.append((t1 - t0) * 1e3)
            seen = defaultdict(int)
            for label, a, b in STAMPS:
                k = f"{label} #{seen[label]}"
                seen[label] += 1
                per[k].append(((a - t0) * 1e3, (b - t0) * 1e3))
        order = sorted(range(len(totals)), key=lambda i: totals[i])
        q = len(order) // 4

        def phase_means(idx):
            acc = defaultdict(list)
            for i in idx:
                for k, v in per.items():
                    if i < len(v):
                        acc[k].append(v[i])
            return {k: (round(statistics.mean(x[0] for x in v), 3), round(statistics.mean(x[1] for x in v), 3))
                    for k, v in sorted(acc.items(), key=lambda kv: statistics.mean(x[0] for x in kv[1]))}
        res.setdefault("spread", {})[what] = {
            "p10_p50_p90_ms": [round(totals[order[len(order) // 10]], 3), round(statistics.median(totals), 3),
                               round(totals[order[(9 * len(order)) // 10]], 3)],
            "fastest_quarter_phases": phase_means(order[:q]), "slowest_quarter_phases": phase_means(order[-q:])}
        res[what] = {"total_ms_median": round(statistics.median(totals), 3), "total_ms_min": round(min(totals), 3),
                     "free_previous_result_ms_median": round(statistics.median(frees), 3),
                     "phases_ms (start, end)": {k: (round(statistics.median(x[0] for x in v), 3),
                                                    round(statistics.median(x[1] for x in v), 3))
                                                for k, v in sorted(per.items(), key=lambda kv: statistics.median(
                                                    x[0] for x in kv[1]))}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
