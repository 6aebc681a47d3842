"""Summarise a rocprofv3 csv trace of tools/host_dict_trace.py: each encode / decode call is the window between
two hipDeviceSynchronize calls of the driver; per window, when the copies and kernels ran (ms from the window's
start), how long the copy engine was busy per direction, and which HIP API calls the calling threads spent
their time in.

    python3 tools/host_dict_trace_summary.py gpurun_out/hdt [--show N]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def rows(root, suffix):
    out = []
    for p in glob.glob(os.path.join(root, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--show", type=int, default=2, help="print the full event list of the last N windows")
    a = ap.parse_args()
    api = rows(a.root, "hip_api_trace.csv")
    cps = rows(a.root, "memory_copy_trace.csv")
    ker = rows(a.root, "kernel_trace.csv")
    syncs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                   if r["Function"] == "hipDeviceSynchronize")
    wins = [(syncs[i][1], syncs[i + 1][0]) for i in range(len(syncs) - 1)]
    # the driver: 5 warm-up pairs without syncs, then per call: sync, encode, marker, sync, decode, marker
    wins = wins[-12:]
    labels = ["encode" if i % 2 == 0 else "decode" for i in range(len(wins))]
    if len(syncs) % 2 == 0:
        labels = labels  # the last window ends at the final sync
    summary = defaultdict(list)
    for wi, ((t0, t1), lab) in enumerate(zip(wins, labels)):
        ev = []
        busy = defaultdict(float)
        for r in cps:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if t0 <= s < t1:
                d = r.get("Direction", "?")
                nb = r.get("Bytes") or r.get("Size") or ""
                ev.append(((s - t0) / 1e6, (e - t0) / 1e6, f"copy {d} {nb}"))
                busy[d] += (e - s) / 1e6
        for r in ker:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if t0 <= s < t1:
                ev.append(((s - t0) / 1e6, (e - t0) / 1e6, "kernel " + r["Kernel_Name"][:60]))
                busy["kernel"] += (e - s) / 1e6
        calls = defaultdict(lambda: [0, 0.0])
        for r in api:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if t0 <= s < t1:
                c = calls[(r["Function"], r.get("Thread_Id", "?"))]
                c[0] += 1
                c[1] += (e - s) / 1e6
        ev.sort()
        span = (t1 - t0) / 1e6
        first = ev[0][0] if ev else 0.0
        last = max((x[1] for x in ev), default=0.0)
        summary[lab].append((span, first, last, dict(busy)))
        if wi >= len(wins) - 2 * a.show:
            print(f"--- {lab} window {wi}: {span:.3f} ms; device work from {first:.3f} to {last:.3f} ms")
            for s, e, what in ev:
                print(f"  {s:7.3f} {e:7.3f} {e - s:6.3f}  {what}")
            for (fn, tid), (n, ms) in sorted(calls.items(), key=lambda kv: -kv[1][1])[:14]:
                print(f"  api {fn:32s} thread {tid:>8s} x{n:3d} {ms:7.3f} ms")
    for lab, v in summary.items():
        v.sort()
        m = v[len(v) // 2]
        print(f"{lab}: median window {m[0]:.3f} ms, device work {m[1]:.3f}..{m[2]:.3f} ms, busy "
              + ", ".join(f"{k} {x:.3f}" for k, x in sorted(m[3].items())))


if __name__ == "__main__":
    main()
