"""C5's exchange leg under a kernel trace: does chunk c's quantize overlap chunk c-1's all-gather?

Run (world 1 over RCCL on one GPU, the C5 shape: 2^30 fp32, bits 4, int4-packed, chunks 8):

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o trace -- \\
        python tools/exchange_trace.py --run
    python tools/exchange_trace.py --report DIR > overlap.json

--run      builds PeerExchange(2^30, bits=4, packed=True, chunks=8) on a one-rank "nccl" (RCCL) process group
           and runs `--iters` exchange_means (the first is warm-up); the encode issues quantize(c) on the
           compute stream and then the chunk's all_gather_into_tensor(async_op=True), which RCCL runs on its
           own stream after an event wait, so quantize(c+1) can start while chunk c is in flight.
--report   reads the trace's kernel and memory-copy CSVs: per exchange, the time intervals of the eight
           k_quantize_int4_flat launches and of every RCCL kernel / copy that moves a chunk, and how much of
           each all-gather interval overlaps a LATER chunk's quantize.

Reference shape: Examples/ray_ad.py:164-190, Src/ADFL/Client/async_peer.py:137-176.
"""

import argparse
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
    from adfl_amd.exchange import PeerExchange

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(args.numel, device=dev, generator=g) * 1e-3
    ex = PeerExchange(args.numel, bits=4, packed=True, chunks=args.chunks, device=dev)
    assert not ex.host_staged
    out = torch.empty(args.numel, device=dev)
    for _ in range(args.iters):
        ex.exchange_mean(x, out)
    torch.cuda.synchronize()
    print(json.dumps({"iters": args.iters, "chunks": len(ex.bounds), "row_bytes": ex.row_bytes[0]}))
    dist.destroy_process_group()


def _rows(d, pattern):
    out = []
    for path in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def report(d):
    kernels = _rows(d, "*kernel_trace.csv")
    copies = _rows(d, "*memory_copy_trace.csv")
    ev = []
    for r in kernels:
        name = r.get("Kernel_Name", "")
        kind = ("quantize" if "k_quantize_int4_flat" in name else
                "absmax" if "k_absmax_flat" in name else
                "mean" if "k_dequantize_mean" in name else
                "rccl" if ("nccl" in name.lower() or "rccl" in name.lower()) else
                "blit" if "rocclr" in name.lower() or "copyBuffer" in name else None)
        if kind:
            ev.append({"kind": kind, "name": name[:80], "start": int(r["Start_Timestamp"]),
                       "end": int(r["End_Timestamp"]), "queue": r.get("Queue_Id", r.get("Stream_Id", ""))})
    for r in copies:
        ev.append({"kind": "copy", "name": r.get("Direction", "copy"), "start": int(r["Start_Timestamp"]),
                   "end": int(r["End_Timestamp"]), "queue": ""})
    ev.sort(key=lambda e: e["start"])
    # exchanges: each starts with an absmax launch
    starts = [i for i, e in enumerate(ev) if e["kind"] == "absmax"]
    exchanges = []
    for k, i0 in enumerate(starts):
        i1 = starts[k + 1] if k + 1 < len(starts) else len(ev)
        seg = ev[i0:i1]
        t0 = seg[0]["start"]
        quant = [e for e in seg if e["kind"] == "quantize"]
        moves = [e for e in seg if e["kind"] in ("rccl", "blit", "copy")]
        ov = []
        for m in moves:
            later = [q for q in quant if q["start"] >= m["start"] - 1 or q["end"] > m["start"]]
            overlap = sum(max(0, min(m["end"], q["end"]) - max(m["start"], q["start"])) for q in later)
            ov.append({"kind": m["kind"], "name": m["name"], "start_us": round((m["start"] - t0) / 1e3, 1),
                       "dur_us": round((m["end"] - m["start"]) / 1e3, 1),
                       "overlap_with_quantize_us": round(overlap / 1e3, 1)})
        exchanges.append({
            "exchange": k, "span_us": round((seg[-1]["end"] - t0) / 1e3, 1),
            "quantize": [{"start_us": round((q["start"] - t0) / 1e3, 1), "dur_us": round((q["end"] - q["start"]) / 1e3, 1),
                          "queue": q["queue"]} for q in quant],
            "moves": ov,
            "moves_overlapping_a_quantize": sum(1 for o in ov if o["overlap_with_quantize_us"] > 0),
            "overlap_total_us": round(sum(o["overlap_with_quantize_us"] for o in ov), 1),
            "moves_total_us": round(sum(o["dur_us"] for o in ov), 1)})
    return {"source": d, "n_events": len(ev), "exchanges": exchanges}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--run", action="store_true")
    p.add_argument("--report")
    p.add_argument("--numel", type=int, default=1 << 30)
    p.add_argument("--chunks", type=int, default=8)
    p.add_argument("--iters", type=int, default=3)
    args = p.parse_args()
    if args.run:
        run(args)
    if args.report:
        print(json.dumps(report(args.report), indent=1))


if __name__ == "__main__":
    main()
