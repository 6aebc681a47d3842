"""One simulated client per GPU: quantized peer exchange over RCCL (BASELINE configs C4 and C5).

Reference shape: every decentralized peer sends its parameters to every other peer and then averages
what it holds, ``torch.stack([update.parameters[name] for update in updates]).mean(dim=0)``
(``Examples/ray_ad.py:164-190``; ``Src/ADFL/Client/async_peer.py:137-176``). In the reference that is
fp32 tensors pickled through Ray's object store. Here each rank is one client on its own MI355X:

    encode (SLQ, this rank's update)  ->  RCCL all-gather of the int8 / int4 payload over xGMI
                                      ->  fused decode + mean of the K payloads (one HIP launch)

Message layout (one row per chunk per rank, 16-byte aligned): ``payload | pad to 16 | fp32 scale | pad``.
The scale rides in the row, so one all-gather moves payloads and scales together. With a bucket layout (a
whole state dict, SLQChannel's per-tensor scales) the row is ``bucket payload | pad | T fp32 scales | pad``
and the mean is taken per tensor with each row's scale for that tensor; the bucket payload is int8, or
int4-packed with ``packed=True`` (PackedSLQChannel per tensor, compression.py:35-66).

The mean (``exact_self=True``, the default) is the reference's: the peers' decoded updates in rank order,
then the rank's OWN update exactly as it is (fp32, not quantized: async_peer.py:170-174 and
ray_ad.py:183-188 append the local parameters after the received ones), fp32 sum, then / K (the oracle's
``dequantize_mean_self``). ``exact_self=False`` averages the K decoded payloads, own row included, in rank
order (``dequantize_mean``), so every rank ends with the bit-identical mean.

Transport: RCCL (``nccl`` backend) all-gathers device rows directly over xGMI. With any other backend
(gloo) on a GPU — e.g. two simulated clients sharing one GPU, the reference's ``NUM_GPUS = 0.5`` packing
(``Examples/ray_ad.py:29``), which RCCL cannot form because it needs distinct devices per rank — each row
is staged through pinned host memory: D2H, gloo all-gather, H2D.

Streams (device ranks, chunks > 1). The absmax pass runs over the whole update on the caller's stream (the
scale needs the global max). Every chunk's quantize is then enqueued at once on a side HIP stream, one event recorded
after each; chunk c's all-gather is issued from a gather stream that waits on event c only, so RCCL's
stream starts chunk c as soon as its quantize retires, while chunk c+1's quantize runs on the side stream.
Enqueuing all the quantizes before any collective keeps the side stream busy back to back: issuing one
all-gather costs the host about as long as quantizing a C5 chunk (tools/exchange_trace.py measured
~100 us host gaps between the chunk quantizes when each quantize waited for the previous chunk's
all_gather call to return). The caller's stream waits for the side stream before encode_and_gather
returns, so later work there (the mean, or a write to x) is ordered after the quantizes. With one chunk
there is nothing to overlap, and the encode and the all-gather go on the caller's stream as issued.

The codec backend is injectable so the exchange protocol can be exercised by gloo on CPU in tests; the
product backend is the HIP codec (``HipCodec``) and there is no other.
"""

from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check


def _pad16(n: int) -> int:
    return (n + 15) // 16 * 16


class HipCodec:
    """The exchange's codec on the device: absmax over the full update, chunk quantize into a message
    row (payload + scale trailer), fused decode + mean over gathered rows."""

    def __init__(self, device: torch.device):
        self.device = device
        self.lib = _lib.load()
        self.ws = torch.empty(_lib.workspace_bytes(), dtype=torch.uint8, device=device)
        self._partials = None

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def absmax(self, x: torch.Tensor) -> None:
        check(self.lib.adfl_slq_absmax(x.data_ptr(), x.numel(), self.ws.data_ptr(), self.ws.numel(), self._stream()))

    def quantize(self, x: torch.Tensor, bits: int, packed: bool, row: torch.Tensor, payload_bytes: int) -> None:
        scale_ptr = row.data_ptr() + _pad16(payload_bytes)
        fn = self.lib.adfl_slq_quantize_int4 if packed else self.lib.adfl_slq_quantize
        check(fn(x.data_ptr(), x.numel(), bits, self.ws.data_ptr(), row.data_ptr(), scale_ptr, self._stream()))

    def encode_bucket(self, x: torch.Tensor, layout, bits: int, row: torch.Tensor, packed: bool = False) -> None:
        """A whole bucketed state dict into one message row: per-tensor SLQ payload (the layout's offsets;
        int4-packed with packed=True) | pad | one fp32 scale per tensor (ops.encode_batched[_int4]: one launch
        when every tensor fits a block)."""
        from . import ops
        pb = (layout.total + 1) // 2 if packed else layout.total
        soff = _pad16(pb)
        if self._partials is None or self._partials.numel() < layout.nchunks:
            self._partials = torch.empty(layout.nchunks, dtype=torch.int32, device=self.device)
        scales = row[soff:soff + 4 * layout.ntensors].view(torch.float32)
        if packed:
            ops.encode_batched_int4(x, layout, bits, packed=row[:pb], scales=scales, partials=self._partials)
        else:
            ops.encode_batched(x, layout, bits, q=row[:pb].view(torch.int8), scales=scales, partials=self._partials)

    def mean_bucket(self, rows: torch.Tensor, layout, out: torch.Tensor, self_row: int = -1,
                    self_x: Optional[torch.Tensor] = None, packed: bool = False) -> None:
        k, row_bytes = rows.shape
        xp = self_x.data_ptr() if self_row >= 0 else None
        pb = (layout.total + 1) // 2 if packed else layout.total
        fn = self.lib.adfl_slq_dequantize_mean_batched_int4 if packed else self.lib.adfl_slq_dequantize_mean_batched
        check(fn(rows.data_ptr(), row_bytes, k, layout.device_chunks(self.device).data_ptr(), layout.nchunks,
                 rows.data_ptr() + _pad16(pb), row_bytes // 4, self_row, xp, out.data_ptr(), self._stream()))

    def mean(self, rows: torch.Tensor, n: int, packed: bool, payload_bytes: int, out: torch.Tensor,
             self_row: int = -1, self_x: Optional[torch.Tensor] = None) -> None:
        k, row_bytes = rows.shape
        scales = rows.data_ptr() + _pad16(payload_bytes)
        fn = self.lib.adfl_slq_dequantize_mean_self_int4 if packed else self.lib.adfl_slq_dequantize_mean_self
        xp = self_x.data_ptr() if self_row >= 0 else None
        check(fn(rows.data_ptr(), row_bytes, k, n, scales, row_bytes // 4, self_row, xp, out.data_ptr(),
                 self._stream()))


class _StagedGather:
    """A pending host-staged all-gather: wait() finishes the gloo collective, then copies the gathered
    rows to the device on the current stream (ordered before the mean kernel)."""

    def __init__(self, work, host: torch.Tensor, dev: torch.Tensor):
        self.work, self.host, self.dev = work, host, dev

    def wait(self):
        self.work.wait()
        self.dev.copy_(self.host)
        return True


class PeerExchange:
    """Quantized all-gather + mean of one flat fp32 update per rank.

    numel   elements of each rank's update (same on every rank)
    bits    SLQ bit width (8: int8 payload; with packed=True the int4 nibble layout, compression.py:35-66)
    chunks  >1 splits quantize + all-gather into a pipeline (C5)
    side_stream  chunk quantizes on a side stream, each all-gather behind its chunk's event (default: when
            chunks > 1); False issues quantize and all-gather in order on the caller's stream
    layout  an ops.BucketLayout: the update is a bucketed state dict (numel = layout.total) encoded as
            SLQChannel encodes a state dict, one scale per tensor (quant.py:74-94), and averaged per tensor
            (ray_ad.py:164-190 averages every tensor). One chunk; int8, or int4 with packed=True (even tensor
            offsets, e.g. BucketLayout(align=2) or the default 64). Without it the whole update has one
            scale (BASELINE's C4 / C5: one flat gradient per client).
    """

    def __init__(self, numel: int, bits: int = 8, packed: bool = False, chunks: int = 1,
                 group: Optional[dist.ProcessGroup] = None, device: Optional[torch.device] = None, codec=None,
                 exact_self: bool = True, layout=None, side_stream: Optional[bool] = None):
        if numel < 1 or chunks < 1:
            raise ValueError("PeerExchange: numel and chunks must be >= 1")
        if layout is not None and (chunks != 1 or numel != layout.total):
            raise ValueError("PeerExchange: a bucket layout is exchanged in one chunk, numel = layout.total")
        if layout is not None and packed and (layout.align % 2 or (layout.offsets % 2).any()):
            raise ValueError("PeerExchange: an int4 bucket needs even tensor offsets")
        self.layout = layout
        self.side_stream = chunks > 1 if side_stream is None else side_stream
        self.numel, self.bits, self.packed, self.group = numel, bits, packed, group
        self.exact_self = exact_self
        self._x: Optional[torch.Tensor] = None
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.codec = HipCodec(device) if codec is None else codec
        # chunk boundaries: multiples of 32 elements keep every payload offset 16-byte aligned
        step = -(-numel // chunks)
        step = (step + 31) // 32 * 32
        self.bounds = [(c0, min(numel, c0 + step)) for c0 in range(0, numel, step)]
        self.payload = [self._payload_bytes(c1 - c0) for c0, c1 in self.bounds]
        trailer = 16 if layout is None else _pad16(4 * layout.ntensors)   # the scale(s) after the payload
        self.row_bytes = [_pad16(p) + trailer for p in self.payload]
        self.local = [torch.empty(rb, dtype=torch.uint8, device=device) for rb in self.row_bytes]
        self.gathered = [torch.empty(self.world, rb, dtype=torch.uint8, device=device) for rb in self.row_bytes]
        # device rows over a host-only backend (gloo): stage each row through pinned host memory. A group
        # made without an explicit backend reports a combined string ("cpu:gloo,cuda:nccl"): its CUDA
        # tensors go through RCCL, so any string naming nccl is device-direct
        self.host_staged = device.type == "cuda" and "nccl" not in str(dist.get_backend(group))
        if self.host_staged:
            self.local_host = [torch.empty(rb, dtype=torch.uint8, pin_memory=True) for rb in self.row_bytes]
            self.gathered_host = [torch.empty(self.world, rb, dtype=torch.uint8, pin_memory=True)
                                  for rb in self.row_bytes]
        if device.type == "cuda":
            self.quant_stream = torch.cuda.Stream(device)    # the chunk quantizes
            self.gather_stream = torch.cuda.Stream(device)   # issues each all-gather behind its chunk's event

    def _payload_bytes(self, n: int) -> int:
        return (n + 1) // 2 if self.packed else n

    @property
    def bytes_per_rank(self) -> int:
        """Bytes each rank contributes to the all-gather (payloads + scale trailers)."""
        return sum(self.row_bytes)

    def encode_and_gather(self, x: torch.Tensor) -> List:
        """Encode this rank's update chunk by chunk; each chunk's all-gather is issued as soon as it is
        quantized. Returns the pending collective works.

        With exact_self, `x` itself is this rank's term of the mean: it must stay unchanged until mean()
        returns (the peers received its quantized values as of this call), and is released there."""
        if x.numel() != self.numel or x.dtype != torch.float32:
            raise ValueError(f"PeerExchange: expected {self.numel} fp32 elements, got {x.numel()} {x.dtype}")
        x = x.reshape(-1)
        self._x = x
        if self.layout is None:
            self.codec.absmax(x)
        if self.device.type != "cuda" or not self.side_stream:
            # one chunk (nothing to overlap inside the exchange) or host tensors (the protocol tests' codec):
            # everything in order on the caller's stream, no stream or event traffic per step
            works = []
            for c in range(len(self.bounds)):
                self._encode(x, c)
                works.append(self._gather(c))
            return works
        main, qs, gs = torch.cuda.current_stream(self.device), self.quant_stream, self.gather_stream
        qs.wait_stream(main)             # the absmax partials (and x itself) are made on the caller's stream
        x.record_stream(qs)
        done = []
        with torch.cuda.stream(qs):
            for c in range(len(self.bounds)):
                self._encode(x, c)
                done.append(qs.record_event())
        works = []
        with torch.cuda.stream(gs):      # RCCL (or the staging copy) syncs with this stream: chunk c only
            for c, ev in enumerate(done):
                gs.wait_event(ev)
                works.append(self._gather(c))
        main.wait_stream(qs)
        return works

    def _chunk(self, x: torch.Tensor, c: int) -> torch.Tensor:
        c0, c1 = self.bounds[c]
        return x[c0:c1]

    def _encode(self, x: torch.Tensor, c: int) -> None:
        if self.layout is not None:
            self.codec.encode_bucket(x, self.layout, self.bits, self.local[c], self.packed)
        else:
            self.codec.quantize(self._chunk(x, c), self.bits, self.packed, self.local[c], self.payload[c])

    def _gather(self, c: int):
        """Issue chunk c's all-gather (async) from the current stream's position."""
        row, out = self.local[c], self.gathered[c]
        if self.host_staged:
            lh, gh = self.local_host[c], self.gathered_host[c]
            lh.copy_(row)  # blocking D2H: also orders after the previous step's H2D from gh
            w = dist.all_gather_into_tensor(gh.view(-1), lh, group=self.group, async_op=True)
            return _StagedGather(w, gh, out)
        return dist.all_gather_into_tensor(out.view(-1), row, group=self.group, async_op=True)

    def mean(self, works: List, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Wait for each chunk's all-gather and decode the K payloads into their fp32 mean (a `None` work
        is a chunk whose collective the caller has already waited on)."""
        if out is None:   # a bucket's gaps (alignment padding) are zero
            out = (torch.empty if self.layout is None else torch.zeros)(self.numel, dtype=torch.float32,
                                                                         device=self.device)
        self_row = self.rank if self.exact_self else -1
        if self_row >= 0 and self._x is None:
            raise RuntimeError("PeerExchange.mean: no pending encode_and_gather (exact_self needs its update)")
        for (c0, c1), rows, pb, w in zip(self.bounds, self.gathered, self.payload, works):
            if w is not None:
                w.wait()
            if self.layout is not None:
                self.codec.mean_bucket(rows, self.layout, out, self_row, self._x if self_row >= 0 else None,
                                       self.packed)
                continue
            self.codec.mean(rows, c1 - c0, self.packed, pb, out[c0:c1], self_row,
                            self._x[c0:c1] if self_row >= 0 else None)
        self._x = None   # the caller's update is not kept alive past the exchange (1-4 GiB at C4/C5)
        return out

    def exchange_mean(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """stack(all ranks' decoded updates).mean(0) (Examples/ray_ad.py:188), via quantized all-gather."""
        return self.mean(self.encode_and_gather(x), out)

    def graph(self, x: torch.Tensor, out: torch.Tensor) -> "ExchangeGraph":
        """Capture one whole exchange of the update in `x` into `out` — encode, RCCL all-gather(s), fused
        decode-mean, the side-stream chunk pipeline included — as a HIP graph. Each replay() re-runs it on
        x's contents at that time, with no Python and one launch call on the host: the C3 bucket at world 1
        measured 0.096 ms eager and 0.041 ms replayed (tools/exchange_graph_probe.py). Collective over the
        group: every rank must capture (and later replay) in the same order. RCCL (device-direct) groups
        only; x and out stay bound to the graph. With a bucket layout, out's gaps between tensors are zeroed
        here and never written again. Validated on hardware at world 1 only (tests/test_gpu_exchange.py:
        replays equal eager and the oracle): a one-GPU box cannot form a two-rank RCCL group, and the
        driver's 8-GPU runs use the eager exchange, so a capture across ranks has not yet been executed."""
        if self.device.type != "cuda" or self.host_staged:
            raise ValueError("PeerExchange.graph: needs device tensors over an RCCL group (host staging cannot "
                             "be captured)")
        if x.numel() != self.numel or x.dtype != torch.float32 or out.numel() != self.numel or \
                out.dtype != torch.float32 or not x.is_contiguous() or not out.is_contiguous():
            raise ValueError("PeerExchange.graph: x and out must be contiguous fp32 tensors of numel elements")
        if self.layout is not None:   # the mean never writes a bucket's gaps: zero them once, as mean(out=None) does
            out.zero_()
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(self.device)
        cap.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cap):
            self.exchange_mean(x, out)      # communicators and streams warmed outside the capture
            with torch.cuda.graph(g, stream=cap):
                self.exchange_mean(x, out)
                for s in (self.quant_stream, self.gather_stream):   # every forked stream rejoins the capture
                    cap.wait_stream(s)
        torch.cuda.current_stream(self.device).wait_stream(cap)
        return ExchangeGraph(g, x, out, self)


class ExchangeGraph:
    """A captured PeerExchange step (PeerExchange.graph): replay() enqueues it on the current stream's
    device; `x` is read and `out` written at replay time. It keeps the exchange (whose message rows, staging
    and streams the graph uses) alive as long as itself."""

    def __init__(self, graph: "torch.cuda.CUDAGraph", x: torch.Tensor, out: torch.Tensor, exchange: "PeerExchange"):
        self.g, self.x, self.out, self.exchange = graph, x, out, exchange

    def replay(self) -> torch.Tensor:
        self.g.replay()
        return self.out
