"""Secondary measurements for BASELINE.json's other configs (one JSON line each).

bench.py measures the headline (C2). This tool measures the rest on the same codec:

  c3        ResNet-18-sized update: 11,689,512 fp32 in 256 tensors, per-tensor scales, bucketed
            (one launch per pass), device-resident; with and without an Infinity-Cache flush
  c5_int4   4 GiB fp32 gradient per GPU (2^30 elements), SLQ bits=4 with pack_4bit layout,
            device-resident round trip (13 B/element algorithmic)
  exchange  one simulated client per GPU: encode -> RCCL all-gather -> fused decode+mean
            (--packed --chunks 8 --elems 1073741824 for C5's int4 pipelined variant). torchrun N>1.
  pcie      the same 1 GiB round trip starting and ending in pinned host memory
            (H2D 4N, D2H N, H2D N, D2H 4N), the rate DESIGN.md reports next to the device-resident one
  stoch     QSGD / RQSGD / CNAT (bits=8) device-resident encode + decode on the C2 tensor (2^28 fp32) and on
            the C3 bucket, in-kernel Philox uniforms; algorithmic bytes: QSGD/RQSGD encode 10N (norm pass
            4N + quantize 4N read, 2N levels+signs write), CNAT encode 6N (one pass), every decode 6N;
            plus the reference's ATen op sequence timed on a 2^22-element host sample

    python tools/bench_configs.py --mode c3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_configs.py --mode exchange
"""

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))

from bench import GIB, HBM_PEAK_GBS, barrier, dist_setup, free_port, max_over_ranks, maybe_launch  # noqa: E402

RESNET18 = 11_689_512


def events(k):
    return [[torch.cuda.Event(enable_timing=True) for _ in range(k)] for _ in range(2)]


def timed(step, steps, warmup, world, nev):
    """Run `step(ev)` (ev: list of nev events to record, or None) warmup+steps times; return
    (max-over-ranks wall seconds for `steps`, per-step event lists)."""
    for _ in range(warmup):
        step(None)
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(nev)] for _ in range(steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(evs[k])
    torch.cuda.synchronize()
    barrier(world)
    return max_over_ranks(time.perf_counter() - t0, world), evs


def seg_ms(evs, i, j):
    return sum(e[i].elapsed_time(e[j]) for e in evs) / len(evs)


def c3_round_trip(lay, packed, args, world, rank, dev, lib, sh, junk, mode="auto"):
    """Device-resident encode + decode of one bucket (per-tensor scales), Infinity Cache warm and
    flushed. packed: the int4 nibble layout (PackedSLQChannel's kernels, 13 B/element). mode: the int8
    encode as ops.encode_batched picks it ("auto": resident when every tensor fits a block, else the
    two passes) or forced ("twopass")."""
    from adfl_amd import _lib
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(lay.total, device=dev, generator=g) * 1e-3
    q = torch.empty(lay.total // 2 if packed else lay.total, dtype=torch.int8, device=dev)
    scales = torch.empty(lay.ntensors, device=dev)
    partials = torch.empty(lay.nchunks, dtype=torch.int32, device=dev)
    out = torch.empty(lay.total, device=dev)
    chunks = lay.device_chunks(dev)
    work = lay.device_work(dev)
    bits = 4 if packed else 8
    n = int(lay.sizes.sum())
    nwork = 0 if mode == "twopass" else lay.nwork

    def enc():
        if packed:
            _lib.check(lib.adfl_slq_encode_batched_int4_work(x.data_ptr(), chunks.data_ptr(), lay.nchunks,
                                                             work.data_ptr(), lay.nwork, bits, q.data_ptr(),
                                                             scales.data_ptr(), partials.data_ptr(), sh))
        else:  # resident one-launch encode when every tensor fits a block (nwork > 0), else the two passes
            _lib.check(lib.adfl_slq_encode_batched_work(x.data_ptr(), chunks.data_ptr(), lay.nchunks, work.data_ptr(),
                                                        nwork, bits, q.data_ptr(), scales.data_ptr(),
                                                        partials.data_ptr(), sh))

    dec_fn = lib.adfl_slq_dequantize_batched_int4 if packed else lib.adfl_slq_dequantize_batched

    def dec():
        _lib.check(dec_fn(q.data_ptr(), chunks.data_ptr(), lay.nchunks, scales.data_ptr(), out.data_ptr(), sh))

    res = {"encode": "resident" if nwork else "twopass", "encode_launches": 1 if nwork else 2}
    resident = bool(lay.nwork if packed else nwork)
    # bytes per element the kernels that ran must move: the one-launch encode reads x
    # once (int8: 4 + 1, int4: 4 + 0.5), the two passes twice; decode 1 + 4 (int4: 0.5 + 4)
    enc_moved = (4.5 if packed else 5.0) if resident else (8.5 if packed else 9.0)
    dec_moved = 4.5 if packed else 5.0
    for flush in (False, True):
        def flush_cache():
            if flush:
                junk.amax()  # READS 512 MiB: the Infinity Cache (256 MiB) holds clean junk lines, nothing of
                             # the codec's buffers, and no dirty lines drain during the timed region

        def step_rt(ev):  # the round trip as one span: no event between the launches
            flush_cache()
            if ev is not None:
                ev[0].record()
            enc()
            dec()
            if ev is not None:
                ev[1].record()

        def step_split(ev):  # encode and decode apart (an event between them perturbs the span)
            flush_cache()
            if ev is not None:
                ev[0].record()
            enc()
            if ev is not None:
                ev[1].record()
            dec()
            if ev is not None:
                ev[2].record()
        _, evs = timed(step_rt, args.steps, args.warmup, world, 2)
        rt = seg_ms(evs, 0, 1)
        _, evs = timed(step_split, args.steps, args.warmup, world, 3)
        e, d = seg_ms(evs, 0, 1), seg_ms(evs, 1, 2)
        res["flushed" if flush else "cache_resident"] = {
            "round_trip_ms": round(rt, 4), "GiB_per_s": round(n * 4 / GIB / (rt * 1e-3), 1),
            "hbm_frac": round((13 if packed else 14) * n / (rt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "hbm_frac_moved": round((enc_moved + dec_moved) * n / (rt * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "encode_frac_moved": round(enc_moved * n / (e * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "encode_ms": round(e, 4), "decode_ms": round(d, 4), "split_round_trip_ms": round(e + d, 4)}
    return res


def mode_c3(args, world, rank, dev):
    """C3: ResNet-18's 11,689,512 parameters in 256 tensors. The headline layout is equal sizes; the
    log-uniform layout (sizes drawn in [64, 2.4 M] and scaled to the total: 64 .. 350,191 elements,
    tests/golden/recipes.py) and the packed int4 variant are
    reported beside it."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import recipes
    from adfl_amd import _lib, ops
    lib = _lib.load()
    sh = torch.cuda.current_stream(dev).cuda_stream
    junk = torch.zeros(128 << 20, dtype=torch.float32, device=dev)
    lay = ops.BucketLayout(recipes.bucket_sizes("equal"))
    res = c3_round_trip(lay, False, args, world, rank, dev, lib, sh, junk)
    lay_log = ops.BucketLayout(recipes.bucket_sizes("loguniform", 0))
    return {"metric": "C3 bucketed round trip, 11,689,512 fp32 in 256 tensors (per-tensor scales)", "unit": "GiB/s",
            "value": res["flushed"]["GiB_per_s"], "chunks": lay.nchunks, **res,
            "loguniform_layout": {"chunks": lay_log.nchunks,
                                  **c3_round_trip(lay_log, False, args, world, rank, dev, lib, sh, junk)},
            "int4_packed": c3_round_trip(lay, True, args, world, rank, dev, lib, sh, junk)}


def mode_c5_int4(args, world, rank, dev):
    from adfl_amd import _lib, ops
    lib = _lib.load()
    sh = torch.cuda.current_stream(dev).cuda_stream
    n = args.elems or (1 << 30)
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    packed = torch.empty((n + 1) // 2, dtype=torch.uint8, device=dev)
    scale = torch.empty(1, device=dev)
    ws = ops.new_workspace(dev)
    out = torch.empty(n, device=dev)

    def step(ev):
        if ev is not None:
            ev[0].record()
        _lib.check(lib.adfl_slq_absmax(x.data_ptr(), n, ws.data_ptr(), ws.numel(), sh))
        if ev is not None:
            ev[1].record()
        _lib.check(lib.adfl_slq_quantize_int4(x.data_ptr(), n, 4, ws.data_ptr(), packed.data_ptr(),
                                              scale.data_ptr(), sh))
        if ev is not None:
            ev[2].record()
        _lib.check(lib.adfl_slq_dequantize_int4(packed.data_ptr(), n, scale.data_ptr(), out.data_ptr(), sh))
        if ev is not None:
            ev[3].record()
    elapsed, evs = timed(step, args.steps, args.warmup, world, 4)
    ms = {k: round(seg_ms(evs, i, i + 1), 4) for i, k in enumerate(("absmax", "quantize_int4", "dequantize_int4"))}
    t = elapsed / args.steps
    return {"metric": "C5 int4 device-resident round trip, 4 GiB fp32 per GPU", "unit": "GiB/s",
            "value": round(world * n * 4 / GIB / t, 2), "n_gpus": world, "ms_per_step": round(t * 1e3, 4),
            "kernels_ms": ms, "hbm_frac": round(13 * n / (sum(ms.values()) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def mode_exchange(args, world, rank, dev):
    from adfl_amd.exchange import PeerExchange
    import torch.distributed as dist
    if world == 1 and not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                                device_id=dev)
    bits = 4 if args.packed else 8
    layout = None
    if args.layout != "flat":   # a whole C3 state dict per client, SLQChannel's per-tensor scales
        sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
        import recipes
        from adfl_amd import ops
        name = args.layout.split("_", 1)[1]
        layout = ops.BucketLayout(recipes.bucket_sizes(name) if name == "equal" else recipes.bucket_sizes(name, 0))
        n = layout.total
    else:
        n = args.elems or (1 << 28)
    ex = PeerExchange(n, bits=bits, packed=args.packed, chunks=args.chunks, device=dev, layout=layout,
                      side_stream=False if args.serial else None)
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(n, device=dev, generator=g) * 1e-3
    out = torch.empty(n, device=dev)

    if args.graph:   # the whole step captured once (PeerExchange.graph), replayed with one host call
        gx = ex.graph(x, out)

        def step(ev):
            gx.replay()
    else:
        def step(ev):
            ex.exchange_mean(x, out)
    elapsed, _ = timed(step, args.steps, args.warmup, world, 1)
    t = elapsed / args.steps
    moved = ex.bytes_per_rank * (world - 1)  # bytes each rank receives over xGMI
    what = (f"bucketed {args.layout} state dict, per-tensor scales, bits={bits}{' packed' if args.packed else ''}"
            if layout is not None else
            f"bits={bits}{' packed' if args.packed else ''}, chunks={args.chunks}"
            f"{', side stream' if ex.side_stream else ', in order'}") + (", HIP graph replay" if args.graph else "")
    return {"metric": f"peer exchange: SLQ encode + RCCL all-gather + fused decode-mean, {what}", "unit": "GiB/s",
            "value": round(world * n * 4 / GIB / t, 2), "n_gpus": world, "ms_per_step": round(t * 1e3, 4),
            "elements_per_rank": n, "bytes_per_rank_on_wire": ex.bytes_per_rank,
            "allgather_algbw_GBs": round(moved / t / 1e9, 1) if world > 1 else None}


def mode_pcie(args, world, rank, dev):
    from adfl_amd import _lib, ops
    lib = _lib.load()
    sh = torch.cuda.current_stream(dev).cuda_stream
    n = args.elems or (1 << 28)
    x_h = (torch.randn(n) * 1e-3).pin_memory()
    q_h = torch.empty(n, dtype=torch.int8).pin_memory()
    out_h = torch.empty(n).pin_memory()
    s_h = torch.empty(1).pin_memory()
    x = torch.empty(n, device=dev)
    q = torch.empty(n, dtype=torch.int8, device=dev)
    q2 = torch.empty(n, dtype=torch.int8, device=dev)
    s = torch.empty(1, device=dev)
    out = torch.empty(n, device=dev)
    ws = ops.new_workspace(dev)

    def step(ev):
        if ev is not None:
            ev[0].record()
        x.copy_(x_h, non_blocking=True)
        if ev is not None:
            ev[1].record()
        _lib.check(lib.adfl_slq_encode(x.data_ptr(), n, 8, q.data_ptr(), s.data_ptr(), ws.data_ptr(), ws.numel(), sh))
        if ev is not None:
            ev[2].record()
        q_h.copy_(q, non_blocking=True)
        s_h.copy_(s, non_blocking=True)
        q2.copy_(q_h, non_blocking=True)   # the payload comes back over the host "wire"
        if ev is not None:
            ev[3].record()
        _lib.check(lib.adfl_slq_dequantize(q2.data_ptr(), n, s.data_ptr(), out.data_ptr(), sh))
        if ev is not None:
            ev[4].record()
        out_h.copy_(out, non_blocking=True)
        if ev is not None:
            ev[5].record()
    elapsed, evs = timed(step, args.steps, args.warmup, world, 6)
    t = elapsed / args.steps
    segs = {k: round(seg_ms(evs, i, i + 1), 4) for i, k in
            enumerate(("h2d_x", "encode", "d2h_h2d_payload", "decode", "d2h_out"))}
    pcie_ms = segs["h2d_x"] + segs["d2h_h2d_payload"] + segs["d2h_out"]
    stream = _pcie_stream(lib, n, x_h, dev, args)
    del x, q, q2, out, x_h, q_h, out_h
    # The same 1 GiB as ADFL hands it over: a pageable CPU state dict through SLQChannel (host to host). The
    # channel stages in element ranges (gather || H2D, D2H || scatter) and allocates its outputs while the
    # D2H runs (Channel/quant.py); encode returns an owned qint8 tensor, decode an owned fp32 tensor.
    from adfl_amd.Channel import SLQChannel
    ch = SLQChannel(8)
    params = {"w": (torch.randn(n) * 1e-3).view(-1, 1024)}
    enc_t, dec_t = [], []
    for k in range(args.warmup + min(args.steps, 10)):
        t0 = time.perf_counter()
        qp, _ = ch.on_client_send(params)
        t1 = time.perf_counter()
        ch.on_server_receive(qp)
        t2 = time.perf_counter()
        if k >= args.warmup:
            enc_t.append(t1 - t0)
            dec_t.append(t2 - t1)
    enc_ms, dec_ms = min(enc_t) * 1e3, min(dec_t) * 1e3
    return {"metric": "PCIe-inclusive SLQ round trip, 1 GiB fp32 from and to pinned host memory", "unit": "GiB/s",
            "value": round(n * 4 / GIB / t, 2), "ms_per_step": round(t * 1e3, 4), "segments_ms": segs,
            "pcie_GBs": round(10 * n / (pcie_ms * 1e-3) / 1e9, 1),
            "stream_of_updates": stream,
            "channel_pageable_dict": {"encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
                                      "round_trip_GiB_per_s": round(n * 4 / GIB / ((enc_ms + dec_ms) * 1e-3), 2),
                                      "best_of": len(enc_t)}}


def _pcie_stream(lib, n, x_h, dev, args, updates: int = 8):
    """The same host-to-host round trip for a STREAM of 1 GiB updates (what a server decoding update after
    update sees): three copy streams and one compute stream ordered only by events, device and pinned
    buffers double-buffered. PCIe is full duplex, so update i+1's
    H2D of x runs under update i's D2H of the output; per update each direction carries 5N bytes."""
    from adfl_amd import _lib, ops
    # four streams (the box runs 4 hardware queues per process; more streams would share them): x in, the
    # payload's hop out and back in (sequential by nature), output out, compute
    streams = {k: torch.cuda.Stream(dev) for k in ("x_in", "q_path", "o_out", "comp")}
    streams["q_out"] = streams["q_in"] = streams["q_path"]
    xs = [torch.empty(n, device=dev) for _ in range(2)]
    qs = [torch.empty(n, dtype=torch.int8, device=dev) for _ in range(2)]
    q2s = [torch.empty(n, dtype=torch.int8, device=dev) for _ in range(2)]
    outs = [torch.empty(n, device=dev) for _ in range(2)]
    ss = [torch.empty(1, device=dev) for _ in range(2)]
    wss = [ops.new_workspace(dev) for _ in range(2)]
    q_hs = [torch.empty(n, dtype=torch.int8).pin_memory() for _ in range(2)]
    o_hs = [torch.empty(n).pin_memory() for _ in range(2)]
    ev = lambda: torch.cuda.Event()  # noqa: E731
    last = {}  # per buffer slot: events of the previous use, so a slot is reused only when free

    def issue(i):
        b = i % 2
        e_x, e_enc, e_qo, e_qi, e_dec, e_oo = ev(), ev(), ev(), ev(), ev(), ev()
        prev = last.get(b)
        with torch.cuda.stream(streams["x_in"]):
            if prev:
                streams["x_in"].wait_event(prev["enc"])          # x[b] free once its encode has read it
            xs[b].copy_(x_h, non_blocking=True)
            e_x.record()
        with torch.cuda.stream(streams["comp"]):
            streams["comp"].wait_event(e_x)
            if prev:
                streams["comp"].wait_event(prev["qo"])           # q[b] free once sent
            _lib.check(lib.adfl_slq_encode(xs[b].data_ptr(), n, 8, qs[b].data_ptr(), ss[b].data_ptr(),
                                           wss[b].data_ptr(), wss[b].numel(), streams["comp"].cuda_stream))
            e_enc.record()
        with torch.cuda.stream(streams["q_out"]):
            streams["q_out"].wait_event(e_enc)
            if prev:
                streams["q_out"].wait_event(prev["qi"])          # q_h[b] free once received
            q_hs[b].copy_(qs[b], non_blocking=True)
            e_qo.record()
        with torch.cuda.stream(streams["q_in"]):
            streams["q_in"].wait_event(e_qo)
            if prev:
                streams["q_in"].wait_event(prev["dec"])          # q2[b] free once decoded
            q2s[b].copy_(q_hs[b], non_blocking=True)
            e_qi.record()
        with torch.cuda.stream(streams["comp"]):
            streams["comp"].wait_event(e_qi)
            if prev:
                streams["comp"].wait_event(prev["oo"])           # out[b] free once sent
            _lib.check(lib.adfl_slq_dequantize(q2s[b].data_ptr(), n, ss[b].data_ptr(), outs[b].data_ptr(),
                                               streams["comp"].cuda_stream))
            e_dec.record()
        with torch.cuda.stream(streams["o_out"]):
            streams["o_out"].wait_event(e_dec)
            o_hs[b].copy_(outs[b], non_blocking=True)
            e_oo.record()
        last[b] = {"enc": e_enc, "qo": e_qo, "qi": e_qi, "dec": e_dec, "oo": e_oo}

    for i in range(2):  # warmup
        issue(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(updates):
        issue(i)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / updates
    ok = bool(torch.equal(o_hs[(updates - 1) % 2], o_hs[(updates - 2) % 2]))  # same input, same output
    # the duplex ceiling on this box: 1 GiB H2D and 1 GiB D2H at the same time, alone and together
    def copy_ms(h2d, d2h, reps=3):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if h2d:
                with torch.cuda.stream(streams["x_in"]):
                    xs[0].copy_(x_h, non_blocking=True)
            if d2h:
                with torch.cuda.stream(streams["o_out"]):
                    o_hs[0].copy_(outs[0], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t1)
        return round(best * 1e3, 3)
    duplex = {"h2d_1GiB_ms": copy_ms(True, False), "d2h_1GiB_ms": copy_ms(False, True),
              "both_at_once_ms": copy_ms(True, True)}
    return {"updates": updates, "ms_per_update": round(t * 1e3, 3), "GiB_per_s": round(n * 4 / GIB / t, 2),
            "pcie_GBs_per_direction": round(5 * n / t / 1e9, 1), "outputs_consistent": ok, "duplex_probe": duplex}


def mode_channel(args, world, rank, dev):
    """ADFL's own call pattern: a CPU state dict through SLQChannel.on_client_send / on_server_receive
    (what Src/ADFL/Client/worker.py:176 and Src/ADFL/Server/async_sc.py:209 do), against the reference's
    per-tensor ATen loop (quant.py:74-112) on the same host and dict."""
    from adfl_amd.Channel import SLQChannel
    base, rem = divmod(RESNET18, 256)
    g = torch.Generator().manual_seed(0)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
    ch = SLQChannel(bits=8)

    def ours():
        t0 = time.perf_counter()
        qp, _ = ch.on_client_send(params)
        t1 = time.perf_counter()
        d, _ = ch.on_server_receive(qp)
        return t1 - t0, time.perf_counter() - t1, qp, d

    def reference():  # quant.py:74-104 then :67-71,107-112 — the reference's loop, ATen CPU ops
        t0 = time.perf_counter()
        enc = {}
        for name, t in params.items():
            if t.ndim > 1:
                scale = torch.max(torch.abs(t)) / 127
                enc[name] = torch.quantize_per_tensor(t, float(scale), 0, dtype=torch.qint8)
            else:
                enc[name] = t
        t1 = time.perf_counter()
        dec = {name: (q.dequantize() if q.ndim > 1 else q.data) for name, q in enc.items()}
        return t1 - t0, time.perf_counter() - t1, enc, dec

    for _ in range(args.warmup):
        ours()
        reference()
    o = [ours()[:2] for _ in range(args.steps)]
    r = [reference()[:2] for _ in range(max(3, args.steps // 4))]
    _, _, qp, d = ours()
    _, _, enc, dec = reference()
    same = all(torch.equal(qp.params[k].data.int_repr(), enc[k].int_repr()) and torch.equal(d[k], dec[k])
               for k in params if params[k].ndim > 1)
    best = lambda xs, i: min(x[i] for x in xs) * 1e3  # noqa: E731
    gib = sum(t.numel() for t in params.values()) * 4 / GIB

    # synchronous server aggregate of K = 4 client updates (Src/ADFL/Strategy/simple.py:83-89): ours
    # receive_mean (one fused decode-mean launch) vs the reference's K decodes + simple_aggregate
    # (Src/ADFL/model.py:221-234) on the host
    ups = []
    for ci in range(4):
        gr = torch.Generator().manual_seed(10 + ci)
        ups.append(ch.on_client_send({k: torch.randn(v.shape, generator=gr) * 1e-3 for k, v in params.items()})[0])

    def ref_aggregate():
        t0 = time.perf_counter()
        dec = [{k: (p.data.dequantize() if p.data.ndim > 1 else p.data.data) for k, p in u.params.items()}
               for u in ups]
        agg = {k: torch.sum(torch.stack([d[k] for d in dec], dim=0), dim=0) / len(dec) for k in dec[0]}
        return time.perf_counter() - t0, agg

    for _ in range(args.warmup):
        ch.receive_mean(ups)
        ref_aggregate()
    om = min(ch.receive_mean(ups)[1] for _ in range(args.steps))
    rm = min(ref_aggregate()[0] for _ in range(max(3, args.steps // 4)))
    mine, want = ch.receive_mean(ups)[0], ref_aggregate()[1]
    agg_same = all(torch.equal(mine[k], want[k]) for k in want)
    return {"metric": "SLQChannel on a CPU ResNet-18-sized state dict (256 weights + 256 biases), host to host",
            "unit": "ms", "ours_encode_ms": round(best(o, 0), 3), "ours_decode_ms": round(best(o, 1), 3),
            "reference_encode_ms": round(best(r, 0), 3), "reference_decode_ms": round(best(r, 1), 3),
            "ours_GiB_s": round(gib / ((best(o, 0) + best(o, 1)) * 1e-3), 2),
            "reference_GiB_s": round(gib / ((best(r, 0) + best(r, 1)) * 1e-3), 2),
            "reference_threads": torch.get_num_threads(), "identical_output": same,
            "aggregate_k4": {"ours_receive_mean_ms": round(om * 1e3, 3),
                             "reference_decode_simple_aggregate_ms": round(rm * 1e3, 3),
                             "identical_output": agg_same}}


def _ref_stoch_cpu(codec, x, bits=8):
    """The reference's op sequence (quant.py:223-252 / 364-398 / 509-545) on a host tensor, in seconds."""
    s = 2 ** bits - 1
    t0 = time.perf_counter()
    if codec == "cnat":
        norm = torch.linalg.vector_norm(x, ord=2)
        signs = torch.sign(x).to(torch.int8)
        xa = torch.abs(x)
        lg = torch.log2(xa + torch.finfo(x.dtype).eps)
        f, c = torch.floor(lg), torch.ceil(lg)
        prob = (2 ** c - xa) / 2 ** f
        e = torch.where(torch.rand_like(prob) < prob, f, c).clamp_(-128, 127)
        e[x == 0] = -128
        e = e.to(torch.int8)
        t1 = time.perf_counter()
        _ = norm.item() * signs.float() * (2 ** e.float())
    else:
        norm = torch.linalg.vector_norm(x, ord=2 if codec == "qsgd" else float("inf"))
        scaled = s * torch.abs(x) / norm
        lo = torch.floor(scaled)
        q = (lo + (torch.rand_like(scaled) < scaled - lo).float()).to(torch.uint8)
        signs = torch.sign(x).to(torch.int8)
        if codec == "rqsgd":
            mf = torch.linalg.vector_norm(x, ord=-float("inf")).item()
        t1 = time.perf_counter()
        r = norm.item() * signs.float() * q.float() / s
        if codec == "rqsgd":
            z = q == 0
            r[z] = mf * signs[z].float()
    return t1 - t0, time.perf_counter() - t1


def mode_channel_stoch(args, world, rank, dev):
    """The stochastic channels on ADFL's call pattern: the C3 CPU state dict through QSGDChannel /
    RQSGDChannel / CNATChannel(8).on_client_send + on_server_receive, against the reference's per-tensor op
    sequence (quant.py:223-252, 364-398, 509-545; restated in _ref_stoch_cpu) on the same host and dict.
    Outputs are not compared here (the uniforms differ by design; tests/test_gpu_stoch.py pins parity)."""
    from adfl_amd.Channel import CNATChannel, QSGDChannel, RQSGDChannel
    base, rem = divmod(RESNET18, 256)
    g = torch.Generator().manual_seed(0)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
    weights = [t for t in params.values() if t.ndim > 1]
    gib = sum(t.numel() for t in params.values()) * 4 / GIB
    res = {"metric": "stochastic channels on a CPU ResNet-18-sized state dict (256 weights + 256 biases), host "
                     "to host", "unit": "ms", "reference_threads": torch.get_num_threads()}
    for name, cls in (("qsgd", QSGDChannel), ("rqsgd", RQSGDChannel), ("cnat", CNATChannel)):
        ch = cls(8)

        def ours():
            t0 = time.perf_counter()
            qp, _ = ch.on_client_send(params)
            t1 = time.perf_counter()
            ch.on_server_receive(qp)
            return t1 - t0, time.perf_counter() - t1

        def reference():
            e = d = 0.0
            for t in weights:
                a, b = _ref_stoch_cpu(name, t)
                e += a
                d += b
            return e, d

        for _ in range(args.warmup):
            ours()
        reference()
        o = [ours() for _ in range(args.steps)]
        r = [reference() for _ in range(3)]
        best = lambda xs, i: min(x[i] for x in xs) * 1e3  # noqa: E731
        res[name] = {"ours_encode_ms": round(best(o, 0), 3), "ours_decode_ms": round(best(o, 1), 3),
                     "reference_encode_ms": round(best(r, 0), 3), "reference_decode_ms": round(best(r, 1), 3),
                     "ours_GiB_s": round(gib / ((best(o, 0) + best(o, 1)) * 1e-3), 2),
                     "reference_GiB_s": round(gib / ((best(r, 0) + best(r, 1)) * 1e-3), 3)}
        res[name]["aggregate_k4"] = _stoch_aggregate_k4(name, ch, params, args)
    return res


def _stoch_aggregate_k4(codec, ch, params, args):
    """Synchronous server aggregate of K = 4 updates (Src/ADFL/Strategy/simple.py:83-89): receive_mean (one
    decode-mean launch) against the reference's per-tensor decode ops (quant.py:243-252 / 385-398 / 537-545)
    + simple_aggregate (Src/ADFL/model.py:221-234) on the host, over the same payloads; the output is checked
    against simple_aggregate of the channel's own decodes (bit-identical for K <= 4)."""
    s = float(2 ** ch.bits - 1)
    ups = []
    for ci in range(4):
        gr = torch.Generator().manual_seed(10 + ci)
        ups.append(ch.on_client_send({k: torch.randn(v.shape, generator=gr) * 1e-3 for k, v in params.items()})[0])

    def ref_decode(p):
        if p.data.ndim <= 1:
            return p.data.data
        norm, sf = float(p.scale), p.signs.float()
        if codec == "qsgd":
            return (norm * p.data.float()) / s * sf
        if codec == "rqsgd":
            r = ((norm * sf) * p.data.float()) / s
            z = p.data == 0
            r[z] = float(p.scale_2) * sf[z]
            return r
        return (norm * sf) * (2 ** p.data.float())

    def aggregate(dec):
        return {k: torch.sum(torch.stack([d[k] for d in dec], dim=0), dim=0) / len(dec) for k in dec[0]}

    def ref_aggregate():
        t0 = time.perf_counter()
        agg = aggregate([{k: ref_decode(p) for k, p in u.params.items()} for u in ups])
        return time.perf_counter() - t0, agg

    for _ in range(args.warmup):
        ch.receive_mean(ups)
        ref_aggregate()
    om = min(ch.receive_mean(ups)[1] for _ in range(args.steps))
    rm = min(ref_aggregate()[0] for _ in range(max(3, args.steps // 4)))
    mine = ch.receive_mean(ups)[0]
    want = aggregate([ch.on_server_receive(u)[0] for u in ups])
    return {"ours_receive_mean_ms": round(om * 1e3, 3), "reference_decode_simple_aggregate_ms": round(rm * 1e3, 3),
            "identical_to_own_decodes_aggregated": all(torch.equal(mine[k], want[k]) for k in want)}


def mode_stoch(args, world, rank, dev):
    """Stochastic codecs (QSGD / RQSGD / CNAT, bits = 8, in-kernel Philox) on C2 (one 2^28 tensor) and C3
    (256 tensors: one-launch resident encodes). Each timed span starts behind GPU work (a 512 MiB read that
    flushes the Infinity Cache, or a short spin when warm), so the Python enqueue cost stays off the span.
    encode_frac counts the algorithmic bytes of the multi-launch design (QSGD / RQSGD read x twice:
    10 B/element; CNAT 6), encode_frac_moved the bytes the kernels that ran must move (6 B/element for every
    codec when the resident encode runs)."""
    from adfl_amd import ops, stoch
    n_flat = args.elems or (1 << 28)
    base, rem = divmod(RESNET18, 256)
    workloads = {"c2_flat": [n_flat], "c3_bucket": [base + (1 if i < rem else 0) for i in range(256)]}
    junk = torch.ones(128 << 20, dtype=torch.float32, device=dev)
    res = {}
    for wname, sizes in workloads.items():
        lay = ops.BucketLayout(sizes, align=1)
        g = torch.Generator(device=dev).manual_seed(rank)
        x = torch.randn(lay.total, device=dev, generator=g) * 1e-3
        lv = torch.empty(lay.total, dtype=torch.uint8, device=dev)
        sg = torch.empty(lay.total, dtype=torch.int8, device=dev)
        nr = torch.empty(lay.ntensors, device=dev)
        mn = torch.empty(lay.ntensors, device=dev)
        out = torch.empty(lay.total, device=dev)
        ws = stoch.workspace(lay, dev)
        n = lay.total
        resident = lay.nwork > 0 and os.environ.get("ADFL_STOCH_RESIDENT", "1") != "0"
        for codec in ("qsgd", "rqsgd", "cnat"):
            for flush in (False, True):
                def step(ev, codec=codec, flush=flush):
                    if flush:
                        junk.amax()
                    else:
                        torch.cuda._sleep(100000)   # ~50 us of GPU spin: the host enqueues behind it
                    if ev is not None:
                        ev[0].record()
                    if codec == "qsgd":
                        stoch.qsgd_encode_batched(x, lay, 8, seed=7, counter=0, levels=lv, signs=sg, norms=nr, ws=ws)
                    elif codec == "rqsgd":
                        stoch.rqsgd_encode_batched(x, lay, 8, seed=7, counter=0, levels=lv, signs=sg, norms=nr,
                                                   mins=mn, ws=ws)
                    else:
                        stoch.cnat_encode_batched(x, lay, 8, seed=7, counter=0, exps=lv.view(torch.int8), signs=sg,
                                                  norms=nr, ws=ws)
                    if ev is not None:
                        ev[1].record()
                    if codec == "qsgd":
                        stoch.qsgd_decode_batched(lv, sg, nr, lay, 8, out=out)
                    elif codec == "rqsgd":
                        stoch.rqsgd_decode_batched(lv, sg, nr, mn, lay, 8, out=out)
                    else:
                        stoch.cnat_decode_batched(lv.view(torch.int8), sg, nr, lay, out=out)
                    if ev is not None:
                        ev[2].record()
                wall, evs = timed(step, args.steps, args.warmup, world, 3)
                enc, dec = seg_ms(evs, 0, 1), seg_ms(evs, 1, 2)
                enc_bytes = (6 if codec == "cnat" else 10) * n
                moved = 6 * n if (resident or codec == "cnat") else 10 * n
                res[f"{wname}_{codec}" + ("_flushed" if flush else "")] = {
                    "encode_ms": round(enc, 4), "decode_ms": round(dec, 4),
                    "encode_launches": 1 if resident else 3,
                    "encode_GBs": round(enc_bytes / enc / 1e6, 1), "decode_GBs": round(6 * n / dec / 1e6, 1),
                    "encode_frac": round(enc_bytes / enc / 1e6 / HBM_PEAK_GBS, 3),
                    "encode_frac_moved": round(moved / enc / 1e6 / HBM_PEAK_GBS, 3),
                    "decode_frac": round(6 * n / dec / 1e6 / HBM_PEAK_GBS, 3),
                    "round_trip_GiBs": round(4 * n / GIB / ((enc + dec) / 1e3), 1)}
    # fp16 / bf16 / fp64 C3 buckets (the *_dt kernels: the reference's arithmetic in each dtype), encode only
    # (decode is the fp32 kernels'); flushed
    lay = ops.BucketLayout(workloads["c3_bucket"], align=1)
    for dtype in (torch.float16, torch.bfloat16, torch.float64):
        xd = (torch.randn(lay.total, device=dev) * 1e-3).to(dtype)
        lvd = torch.empty(lay.total, dtype=torch.uint8, device=dev)
        sgd = torch.empty(lay.total, dtype=torch.int8, device=dev)
        wsd = stoch.workspace(lay, dev)
        for codec in ("qsgd", "cnat"):
            def step_dt(ev, codec=codec):
                junk.amax()
                if ev is not None:
                    ev[0].record()
                stoch.encode_batched_dt(codec, xd, lay, 8, seed=7, counter=0,
                                        levels=lvd.view(torch.int8) if codec == "cnat" else lvd, signs=sgd, ws=wsd)
                if ev is not None:
                    ev[1].record()
            _, evs = timed(step_dt, args.steps, args.warmup, world, 2)
            enc = seg_ms(evs, 0, 1)
            # QSGD: x read twice (norm pass, quantize) + 2 planes; CNAT: x once (exponents + partials) + 2 planes
            eb = ((1 if codec == "cnat" else 2) * xd.element_size() + 2) * lay.total
            res[f"c3_bucket_{str(dtype).replace('torch.', '')}_{codec}_flushed"] = {
                "encode_ms": round(enc, 4), "encode_GBs": round(eb / enc / 1e6, 1),
                "encode_frac": round(eb / enc / 1e6 / HBM_PEAK_GBS, 3)}
        del xd, lvd, sgd
    del junk
    # calibration on the same box: the SLQ flat round trip of bench.py's headline kernels
    from adfl_amd import _lib
    lib = _lib.load()
    sh = torch.cuda.current_stream(dev).cuda_stream
    x = torch.randn(n_flat, device=dev) * 1e-3
    q = torch.empty(n_flat, dtype=torch.int8, device=dev)
    sc = torch.empty(1, device=dev)
    wsl = ops.new_workspace(dev)
    outf = torch.empty(n_flat, device=dev)

    def slq_step(ev):
        if ev is not None:
            ev[0].record()
        lib.adfl_slq_encode(x.data_ptr(), n_flat, 8, q.data_ptr(), sc.data_ptr(), wsl.data_ptr(), wsl.numel(), sh)
        if ev is not None:
            ev[1].record()
        lib.adfl_slq_dequantize(q.data_ptr(), n_flat, sc.data_ptr(), outf.data_ptr(), sh)
        if ev is not None:
            ev[2].record()
    _, evs = timed(slq_step, args.steps, args.warmup, world, 3)
    res["c2_flat_slq_calibration"] = {"encode_ms": round(seg_ms(evs, 0, 1), 4), "decode_ms": round(seg_ms(evs, 1, 2), 4)}
    del x, q, outf
    if rank == 0 and not args.no_cpu:
        m = 1 << 22
        xs = torch.randn(m) * 1e-3
        torch.set_num_threads(os.cpu_count() if os.cpu_count() <= 16 else 16)
        for codec in ("qsgd", "rqsgd", "cnat"):
            best = min((_ref_stoch_cpu(codec, xs) for _ in range(3)), key=lambda t: t[0] + t[1])
            res[f"cpu_reference_{codec}"] = {"sample_elems": m, "threads": torch.get_num_threads(),
                                             "encode_ms": round(best[0] * 1e3, 2), "decode_ms": round(best[1] * 1e3, 2),
                                             "round_trip_GiBs": round(4 * m / GIB / (best[0] + best[1]), 3)}
    return {"mode": "stoch", "n_gpus": world, "steps": args.steps, **res}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--serial", action="store_true", help="exchange: no side stream (quantize + all-gather in order)")
    p.add_argument("--graph", action="store_true", help="exchange: time PeerExchange.graph replays")
    p.add_argument("--layout", choices=["flat", "c3_equal", "c3_loguniform"], default="flat",
                   help="exchange: one flat update per rank, or a C3 state dict with per-tensor scales")
    p.add_argument("--mode", choices=["c3", "c5_int4", "exchange", "pcie", "channel", "channel_stoch", "stoch"],
                   required=True)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--elems", type=int, default=0)
    p.add_argument("--packed", action="store_true")
    p.add_argument("--chunks", type=int, default=1)
    p.add_argument("--no-cpu", action="store_true", help="stoch: skip the host reference timing")
    args = p.parse_args()
    rc = maybe_launch(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world, rank, local = dist_setup(args)
    assert world == args.gpus, (world, args.gpus)
    dev = torch.device("cuda", local)
    line = {"c3": mode_c3, "c5_int4": mode_c5_int4, "exchange": mode_exchange, "pcie": mode_pcie,
            "channel": mode_channel, "channel_stoch": mode_channel_stoch, "stoch": mode_stoch}[args.mode](
        args, world, rank, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
