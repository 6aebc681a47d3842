"""Stochastic-rounding channels backed by the MI355X HIP codec — drop-in for
``Src/ADFL/Channel/quant.py:140-570`` (QSGD, UQSGD, RQSGD, URQSGD, CNAT, UCNAT).

Same names, constructor (``bits``; ``levels = 2**bits - 1``), six-method surface, ``to_json`` output,
``simulate_bandwidth`` formulas and payload layout as the reference:

* ``QuantParameter.data`` = levels (uint8; CNAT: int8 exponents), ``signs`` = int8 sign plane,
  ``scale`` = the norm as a Python float (``norm.item()``), ``scale_2`` = RQSGD's min|x|;
* all-zero tensors take the reference's norm == 0 branch: uint8 zeros, int8 ones, ``scale`` = the 0-dim
  fp32 tensor ``tensor(0.)`` (quant.py:227-228,368-369,513-514);
* ``ndim <= 1`` tensors pass through (same object) with ``signs = zeros(1, uint8)`` and scale 0;
* ``size`` counts only the level / exponent bytes, as the reference does (quant.py:218,359,504);
* decode returns owned, writable fp32 tensors.

What changes is where the arithmetic runs: the whole state dict is staged once into one flat bucket on
the GPU and encoded / decoded by a few HIP launches for all tensors together (include/adfl_stoch.h).

Randomness: the reference draws ``torch.rand_like`` from torch's CPU generator. Here each encode draws a
fresh 62-bit seed from that same generator (so ``torch.manual_seed`` reproduces a run) and the kernels
generate their uniforms from a Philox4x32-7 stream keyed by it. The uniforms are not the reference's
mt19937 draws, so individual rounding decisions differ from a reference run; their distribution is the
same (and with injected uniforms the codec is bit-identical: tests/test_gpu_stoch.py).

Norms: the L2 norm (QSGD, CNAT) is the reference's own, bit for bit: torch 2.10's CPU
``torch.linalg.vector_norm`` order in the tensor's dtype (fp32 / bf16 / fp16 / fp64; fp16's split over
``torch.get_num_threads()`` as the reference's call would make it), by csrc/torch_norm.hip. ADFL_STOCH_NORM=fp64
in the environment switches to the correctly rounded norm (fp64 accumulation of the squares: faster on very
large tensors, within torch's own summation error of the reference's). RQSGD's max / min norms are exact either
way. There is no CPU fallback: without the HIP library these raise.

fp16 / bf16 / fp64 tensors are encoded as the reference encodes them, in their own dtype's arithmetic (each
op rounded to the dtype; uniforms on torch.rand's grid for the dtype): one bucket per dtype through the
*_dt kernels (csrc/stoch_dtype.hip). Their payloads decode like fp32 ones (the reference decodes to fp32).
"""

import os
import time
from typing import Dict, List, Tuple

import torch

from .. import hostcopy, ops
from .. import stoch as sops
from ..model import CompressedParameters, Parameters, QuantParameter, QuantParameters, get_parameter_info
from .channel import Channel, IdentityChannel
from .quant import (_PendingD2H, _aggregate_entries, _hand_out, _serialized, _stage_in, _stage_rows, _staging,
                    device_mean_order_ok)

_CODECS = ("qsgd", "rqsgd", "cnat")


def reference_norm() -> bool:
    """The L2 norm mode of the QSGD / CNAT channels: True (default) = the reference's own norm, torch's CPU
    order bit for bit; ADFL_STOCH_NORM=fp64 = the correctly rounded norm (fp64 accumulation)."""
    mode = os.environ.get("ADFL_STOCH_NORM", "torch").lower()
    if mode not in ("torch", "fp64"):
        raise ValueError(f"ADFL_STOCH_NORM must be 'torch' (the reference's norm) or 'fp64', got {mode!r}")
    return mode == "torch"


def _require_codable(name: str, t: torch.Tensor, cls: str) -> None:
    """fp32 / fp16 / bf16 / fp64 tensors are encoded (each in its own dtype's arithmetic, as the reference
    computes them). Anything else fails as the reference's first op on it fails: torch.linalg.vector_norm
    raises for integer and bool tensors (quant.py:226,367,512)."""
    if t.dtype == torch.float32 or t.dtype in sops.DT_DTYPES:
        return
    if not (t.is_floating_point() or t.is_complex()):
        torch.linalg.vector_norm(t.reshape(-1)[:0])   # raises the reference's RuntimeError
    raise ValueError(f"{cls}: '{name}' is {t.dtype}; the HIP stochastic codecs take fp32 / fp16 / bf16 / fp64")


def _owned(parts: List[torch.Tensor], shapes: List[torch.Size]) -> List[torch.Tensor]:
    """Per-tensor copies: each payload tensor owns its bytes (it is pickled on its own; the staging
    buffers are reused by the next call)."""
    return [p.view(s).clone() for p, s in zip(parts, shapes)]


def _owned_dev(buf: torch.Tensor, lay, shapes: List[torch.Size]) -> List[torch.Tensor]:
    """_owned for a device dict: fresh tensors filled from the bucket by one launch (ops.bucket_scatter)."""
    outs = [torch.empty(s, dtype=buf.dtype, device=buf.device) for s in shapes]
    ops.bucket_scatter(buf, lay, outs, checked=False)
    return outs


def _owned_host(buf: torch.Tensor, offsets, shapes: List[torch.Size]) -> List[torch.Tensor]:
    """_owned for a host bucket: fresh tensors filled by one native parallel scatter."""
    outs = [torch.empty(s, dtype=buf.dtype) for s in shapes]
    hostcopy.advise_huge(outs)
    hostcopy.scatter(buf, outs, offsets)
    return outs


@_serialized
def _encode_stoch(params: Parameters, names: List[str], codec: str, bits: int, uniforms=None, seed=None,
                  torch_norm: bool = True):
    """Encode the ndim > 1 fp32 tensors `names` of `params` in one bucketed pass.

    Returns {name: (data, signs, scale, scale_2)} with CPU tensors for CPU inputs (device tensors for
    device inputs). `uniforms`: optional fp32 device plane over the compact bucket (tests)."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    lay = st.layout(tuple(int(t.numel()) for t in tensors))
    x_dev = _stage_in(tensors, lay, st, "x", torch.float32)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    ws = st.buf("stoch_ws", lay.nchunks * 16, torch.uint8)
    # staging buffers are cached by name: the level plane is always uint8 (CNAT views it as int8)
    planes = dict(levels=st.buf("s_levels", lay.total, torch.uint8), signs=st.buf("s_signs", lay.total, torch.int8))
    norms = st.buf("s_norms", lay.ntensors, torch.float32)
    mins = None
    if codec == "qsgd":
        lv, sg, norms = sops.qsgd_encode_batched(x_dev, lay, bits, uniforms=uniforms, seed=seed, counter=0,
                                                 levels=planes["levels"], signs=planes["signs"], norms=norms, ws=ws,
                                                 torch_norm=torch_norm)
    elif codec == "rqsgd":
        mins = st.buf("s_mins", lay.ntensors, torch.float32)
        lv, sg, norms, mins = sops.rqsgd_encode_batched(x_dev, lay, bits, uniforms=uniforms, seed=seed, counter=0,
                                                        levels=planes["levels"], signs=planes["signs"],
                                                        norms=norms, mins=mins, ws=ws)
    else:
        lv, sg, norms = sops.cnat_encode_batched(x_dev, lay, bits, uniforms=uniforms, seed=seed, counter=0,
                                                 exps=planes["levels"].view(torch.int8), signs=planes["signs"],
                                                 norms=norms, ws=ws, torch_norm=torch_norm)
    nm_host = st.buf("s_norms_host", 2 * lay.ntensors, torch.float32, pinned=True)
    nm_host[:lay.ntensors].copy_(norms, non_blocking=True)
    if mins is not None:
        nm_host[lay.ntensors:].copy_(mins, non_blocking=True)
    on_cpu = [not t.is_cuda for t in tensors]
    if all(on_cpu):
        # as SLQ's encode: both planes' D2H enqueued right behind the norms, the owned outputs allocated
        # while they run, each range scattered as it lands
        norms_ready = torch.cuda.Event()
        norms_ready.record(torch.cuda.current_stream(dev))
        pend_lv = _PendingD2H(lv.view(torch.uint8), lay, st, "s_levels")
        pend_sg = _PendingD2H(sg, lay, st, "s_signs")
        shapes = [t.shape for t in tensors]
        lv_parts = [torch.empty(s_, dtype=lv.dtype) for s_ in shapes]
        sg_parts = [torch.empty(s_, dtype=torch.int8) for s_ in shapes]
        hostcopy.advise_huge(lv_parts + sg_parts)
        norms_ready.synchronize()
        nm = nm_host.tolist()
        pend_lv.finish([t.view(torch.uint8) for t in lv_parts])
        pend_sg.finish(sg_parts)
        return _payloads(names, lv_parts, sg_parts, nm, lay.ntensors, codec)
    if any(on_cpu):
        lv_h = st.buf("s_levels_host", lay.total, torch.uint8, pinned=True).view(lv.dtype)
        sg_h = st.buf("s_signs_host", lay.total, torch.int8, pinned=True)
        lv_h.copy_(lv, non_blocking=True)
        sg_h.copy_(sg, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    nm = nm_host.tolist()
    sizes, shapes = lay.sizes.tolist(), [t.shape for t in tensors]
    split = lambda buf: [p[:n] for p, n in zip(torch.split(buf, lay.padded.tolist()), sizes)]  # noqa: E731
    lv_parts = _owned_host(lv_h, lay.offsets, shapes) if any(on_cpu) else None
    sg_parts = _owned_host(sg_h, lay.offsets, shapes) if any(on_cpu) else None
    if not any(on_cpu):   # device dict: one scatter launch per plane
        lv_dev, sg_dev = _owned_dev(lv, lay, shapes), _owned_dev(sg, lay, shapes)
    else:
        lv_dev = _owned(split(lv), shapes) if not all(on_cpu) else None
        sg_dev = _owned(split(sg), shapes) if not all(on_cpu) else None
    datas = [(lv_parts if cpu else lv_dev)[i] for i, cpu in enumerate(on_cpu)]
    signs = [(sg_parts if cpu else sg_dev)[i] for i, cpu in enumerate(on_cpu)]
    return _payloads(names, datas, signs, nm, lay.ntensors, codec)


# Philox block-counter base of each dtype bucket: one seed serves an fp32 bucket and every fp16 / bf16 / fp64
# bucket of the same call, and each draws from its own disjoint part of the stream (2^40 blocks = 2^42
# uniforms each), so no two buckets' rounding decisions share a uniform.
COUNTER_BASE = {torch.float32: 0, torch.float16: 1 << 40, torch.bfloat16: 2 << 40, torch.float64: 3 << 40}


@_serialized
def _encode_stoch_dt(params: Parameters, names: List[str], codec: str, bits: int, uniforms=None, seed=None,
                     torch_norm: bool = True):
    """Encode the ndim > 1 tensors `names` (all of one dtype: fp16 / bf16 / fp64) in one bucketed pass, in
    that dtype's arithmetic (adfl_stoch_encode_batched_dt). Same return as _encode_stoch; the norms are the
    dtype's values as Python floats (norm.item() of the reference's 0-dim norm tensor)."""
    st = _staging()
    dev = st.device
    tensors = [params[n] for n in names]
    dtype = tensors[0].dtype
    tag = str(dtype).replace("torch.", "")
    lay = st.layout(tuple(int(t.numel()) for t in tensors))
    x_dev = _stage_in(tensors, lay, st, "x_" + tag, dtype)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    ws = st.buf("stoch_ws", lay.nchunks * 16, torch.uint8)
    u = uniforms if uniforms is not None and uniforms.dtype == dtype else None
    levels = st.buf("s_levels", lay.total, torch.uint8).view(torch.int8 if codec == "cnat" else torch.uint8)
    signs = st.buf("s_signs", lay.total, torch.int8)
    if codec != "rqsgd" and torch_norm:  # the reference's norm in the dtype, then the given-norm quantize
        norms, _ = sops.reference_norms(x_dev, lay, out64=st.buf("s_norms64", lay.ntensors, torch.float64))
        lv, sg = sops.quantize_batched_dt(codec, x_dev, lay, bits, norms, uniforms=u, seed=seed,
                                          counter=COUNTER_BASE[dtype], levels=levels, signs=signs)
        mins = None
    else:
        lv, sg, norms, mins = sops.encode_batched_dt(codec, x_dev, lay, bits, uniforms=u, seed=seed,
                                                     counter=COUNTER_BASE[dtype], levels=levels, signs=signs, ws=ws)
    nm = torch.cat([norms, mins]) if mins is not None else norms
    on_cpu = [not t.is_cuda for t in tensors]
    shapes = [t.shape for t in tensors]
    if any(on_cpu):
        lv_h = st.buf("s_levels_host", lay.total, torch.uint8, pinned=True).view(lv.dtype)
        sg_h = st.buf("s_signs_host", lay.total, torch.int8, pinned=True)
        lv_h.copy_(lv, non_blocking=True)
        sg_h.copy_(sg, non_blocking=True)
    nm = nm.cpu().tolist()   # synchronises: the planes' D2H has landed too
    sizes = lay.sizes.tolist()
    split = lambda buf: [p[:n] for p, n in zip(torch.split(buf, lay.padded.tolist()), sizes)]  # noqa: E731
    lv_parts = _owned_host(lv_h, lay.offsets, shapes) if any(on_cpu) else None
    sg_parts = _owned_host(sg_h, lay.offsets, shapes) if any(on_cpu) else None
    if not any(on_cpu):   # device dict: one scatter launch per plane
        lv_dev, sg_dev = _owned_dev(lv, lay, shapes), _owned_dev(sg, lay, shapes)
    else:
        lv_dev = _owned(split(lv), shapes) if not all(on_cpu) else None
        sg_dev = _owned(split(sg), shapes) if not all(on_cpu) else None
    datas = [(lv_parts if cpu else lv_dev)[i] for i, cpu in enumerate(on_cpu)]
    signs = [(sg_parts if cpu else sg_dev)[i] for i, cpu in enumerate(on_cpu)]
    return _payloads(names, datas, signs, nm, lay.ntensors, codec, dtype)


def _payloads(names, datas, signs, nm, ntensors: int, codec: str, dtype: torch.dtype = torch.float32):
    """{name: (data, signs, scale, scale_2)} as the reference's _quantize_tensor returns them."""
    out = {}
    for i, name in enumerate(names):
        data, norm = datas[i], nm[i]
        if norm == 0.0:  # the reference's norm == 0 branch: uint8 zeros, the 0-dim norm tensor as scale
            scale = torch.tensor(0.0, dtype=dtype)
            data = data.view(torch.uint8)
            scale_2 = 0
        else:
            scale = norm
            scale_2 = nm[ntensors + i] if codec == "rqsgd" else 0
        out[name] = (data, signs[i], scale, scale_2)
    return out


@_serialized
def _decode_stoch(items: List[Tuple[str, QuantParameter]], codec: str, bits: int) -> Dict[str, torch.Tensor]:
    """Decode (levels, signs, norm[, min]) payloads of ndim > 1 tensors in one bucketed pass."""
    st = _staging()
    lay, out_dev = _decode_stoch_bucket(st, items, codec, bits)
    datas = [p.data for _, p in items]
    on_cpu = [not d.is_cuda for d in datas]
    # CPU payloads: the fp32 outputs (shaped like the level planes) made in one native call per range
    decoded = _hand_out(out_dev, lay, [d.shape for d in datas], on_cpu, st, "d_out", like=datas if all(on_cpu) else None)
    return {name: t for (name, _), t in zip(items, decoded)}


@_serialized
def _decode_add_stoch(items: List[Tuple[str, QuantParameter]], codec: str, bits: int,
                      targets: List[List[torch.Tensor]]) -> None:
    """Decode the payloads once into the device bucket and add it into every model (targets[k][j] += decode of
    item j, fp32 adds: add_parameters_inpace's mul_(1).add_(d, alpha=1), model.py:337-347)."""
    st = _staging()
    lay, out_dev = _decode_stoch_bucket(st, items, codec, bits)
    views = [out_dev[o:o + n].view(p.data.shape)
             for o, n, (_, p) in zip(lay.offsets.tolist(), lay.sizes.tolist(), items)]
    with torch.no_grad():
        for model in targets:
            torch._foreach_add_(model, views)
    # the next call's staging rewrites the pinned buffers this call's H2D read and the bucket it decoded into
    torch.cuda.current_stream(st.device).synchronize()


def _decode_stoch_bucket(st, items: List[Tuple[str, QuantParameter]], codec: str, bits: int):
    """Both planes staged as one bucket on the device and decoded by one launch: (layout, fp32 bucket)."""
    dev = st.device
    lay = st.layout(tuple(int(p.data.numel()) for _, p in items))
    lv_dev = _stage_in([p.data.view(torch.uint8) for _, p in items], lay, st, "d_levels", torch.uint8)
    sg_dev = _stage_in([p.signs.view(torch.int8) for _, p in items], lay, st, "d_signs", torch.int8)
    scales = [float(p.scale) for _, p in items]
    ntens = len(items)
    sc = torch.tensor(scales + ([float(p.scale_2) for _, p in items] if codec == "rqsgd" else []),
                      dtype=torch.float32).to(dev, non_blocking=True)
    out_dev = st.buf("d_out", lay.total, torch.float32)
    if codec == "qsgd":
        sops.qsgd_decode_batched(lv_dev, sg_dev, sc[:ntens], lay, bits, out=out_dev)
    elif codec == "rqsgd":
        sops.rqsgd_decode_batched(lv_dev, sg_dev, sc[:ntens], sc[ntens:], lay, bits, out=out_dev)
    else:
        sops.cnat_decode_batched(lv_dev.view(torch.int8), sg_dev, sc[:ntens], lay, out=out_dev)
    return lay, out_dev


@_serialized
def _decode_mean_stoch(all_c_params: List[QuantParameters], names: List[str], codec: str,
                       bits: int) -> List[torch.Tensor]:
    """simple_aggregate over K payloads of the entries `names` (every client's entry decodable by
    _decode_stoch, one shape): both byte planes of every client staged as device rows, one launch of
    adfl_stoch_dequantize_mean_batched, one owned fp32 tensor per entry (CPU when the payloads are)."""
    st = _staging()
    dev = st.device
    first = all_c_params[0].params
    lay = st.layout(tuple(int(first[n].data.numel()) for n in names))
    lv_rows = _stage_rows([[c.params[n].data for n in names] for c in all_c_params], lay, st, "sm_levels")
    sg_rows = _stage_rows([[c.params[n].signs for n in names] for c in all_c_params], lay, st, "sm_signs")
    norms = torch.tensor([[float(c.params[n].scale) for n in names] for c in all_c_params],
                         dtype=torch.float32).to(dev, non_blocking=True)
    mins = (torch.tensor([[float(c.params[n].scale_2) for n in names] for c in all_c_params],
                         dtype=torch.float32).to(dev, non_blocking=True) if codec == "rqsgd" else None)
    out_dev = sops.dequantize_mean_batched(codec, lv_rows, sg_rows, norms, lay, bits, mins=mins,
                                           out=st.buf("sm_out", lay.total, torch.float32))
    on_cpu = [not any(c.params[n].data.is_cuda for c in all_c_params) for n in names]
    return _hand_out(out_dev, lay, [first[n].data.shape for n in names], on_cpu, st, "sm_out")


class _StochChannel(Channel):
    """Shared body of the three bi-directional stochastic channels."""

    CODEC = "qsgd"
    NORM_BYTES = 4  # per quantized tensor: the norm (RQSGD: norm + minimum factor)

    def __init__(self, bits: int) -> None:
        """The reference's constructor (quant.py:145-147): the L2 norm is the reference's own (see the module
        docstring; ADFL_STOCH_NORM=fp64 selects the correctly rounded one instead)."""
        self.bits = bits
        self.levels = 2 ** bits - 1

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return self._send(params)

    def on_server_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return self._receive(c_params)

    def on_client_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return self._send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return self._receive(c_params)

    def to_json(self) -> Dict:
        return {"name": self.__class__.__name__, "bits": self.bits}

    def simulate_bandwidth(self, params: Parameters, mbps: float) -> float:
        """self.bits + 1 for weights and signs, 32 bits for biases, norms (quant.py:173-184,313-324,459-470)."""
        p_info = get_parameter_info(params)
        num_bytes = p_info.num_non_bias_w * (self.bits + 1) / 8
        num_bytes += p_info.num_bias_w * 4
        num_bytes += p_info.num_non_bias_t * self.NORM_BYTES
        transfer_time = num_bytes / (mbps * 1_000_000 / 8)
        time.sleep(transfer_time)
        return transfer_time

    def _send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        s_time = time.perf_counter()
        q_params = self._quantize_params(params, self.bits)
        return q_params, time.perf_counter() - s_time

    def _receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        assert isinstance(c_params, QuantParameters)
        s_time = time.perf_counter()
        items = [(name, p) for name, p in c_params.params.items() if p.data.ndim > 1 and p.data.numel() > 0]
        decoded = _decode_stoch(items, self.CODEC, self.bits) if items else {}
        params = {}
        for name, p in c_params.params.items():
            if name in decoded:
                params[name] = decoded[name]
            elif p.data.ndim > 1:  # empty tensor: the reference's scale == 0 branch
                params[name] = torch.zeros_like(p.data, dtype=torch.float32)
            else:
                params[name] = p.data.data  # passthrough
        return params, time.perf_counter() - s_time

    def receive_mean(self, all_c_params: List[CompressedParameters]) -> Tuple[Parameters, float]:
        """``simple_aggregate([self.on_server_receive(c)[0] for c in all_c_params])`` — a synchronous server
        decoding K client updates and averaging them (Src/ADFL/Strategy/simple.py:83-89 over
        Src/ADFL/model.py:221-234). Returns (aggregate, seconds).

        Entries encoded in every update are decoded and averaged on the device in one launch (each client's
        level and sign planes read once, no decoded copy materialised): summed in torch's CPU order for
        ``torch.sum(torch.stack(...), dim=0)`` (csrc/torch_sum_order.h), then / K, bit-identical to
        simple_aggregate of the decoded CPU tensors at every K (tests/golden/aggregate.npz: the reference's
        own payloads and aggregates at K = 5, 8, 16, 20). Everything else (biases, running statistics, empty
        tensors) is decoded and aggregated as the reference does, on the host."""
        if not all_c_params:
            raise AssertionError("receive_mean: no updates")   # simple_aggregate asserts len > 0
        for c in all_c_params:
            assert isinstance(c, QuantParameters)
        s_time = time.perf_counter()
        names = list(all_c_params[0].params.keys())
        fused = [n for n in names if all(n in c.params and self._fusable(c.params[n]) for c in all_c_params)
                 and len({tuple(c.params[n].data.shape) for c in all_c_params}) == 1] if device_mean_order_ok() else []
        out: Parameters = {}
        if fused:
            out.update(zip(fused, _decode_mean_stoch(all_c_params, fused, self.CODEC, self.bits)))
        rest = [n for n in names if n not in out]
        if rest:
            parts = [self._receive(QuantParameters({n: c.params[n] for n in rest}, 0))[0] for c in all_c_params]
            out.update(_aggregate_entries(rest, parts))
        return {n: out[n] for n in names}, time.perf_counter() - s_time

    def receive_add_(self, c_params: CompressedParameters, targets: List[Parameters]) -> float:
        """``on_client_receive(c_params)`` followed by ``add_parameters_inpace(t, decoded, 1, 1, False)`` for
        every ``t`` in ``targets`` — the client pool's ``add_to_model`` / ``add_to_model_all``
        (Src/ADFL/Client/pool.py:62-75) and QAFeL's hidden-state update (Src/ADFL/Server/qafel.py:176-179),
        bit-identical to them. Returns the seconds spent.

        Encoded tensors whose targets are all fp32 device tensors are decoded once, into device memory, and
        added into every model there (no decoded tensor crosses PCIe). Everything else takes the reference's
        route: decode, then ``mul_(1).add_(decoded, alpha=1)``."""
        assert isinstance(c_params, QuantParameters)
        for t in targets:
            assert set(t.keys()) == set(c_params.params.keys())  # add_parameters_inpace, model.py:340
        s_time = time.perf_counter()
        fused = [n for n, p in c_params.params.items()
                 if self._fusable(p) and all(t[n].is_cuda and t[n].dtype == torch.float32 for t in targets)]
        if fused and targets:
            dev = targets[0][fused[0]].device   # the staging's device (the current one) for the whole set
            if dev.index == torch.cuda.current_device() and all(t[n].device == dev for t in targets for n in fused):
                _decode_add_stoch([(n, c_params.params[n]) for n in fused], self.CODEC, self.bits,
                                  [[t[n] for n in fused] for t in targets])
            else:
                fused = []
        rest = QuantParameters({n: p for n, p in c_params.params.items() if n not in fused}, 0)
        if rest.params:
            decoded, _ = self.on_client_receive(rest)
            with torch.no_grad():
                for t in targets:
                    for n, d in decoded.items():
                        t[n].mul_(1).add_(d.to(t[n].device), alpha=1)
        return time.perf_counter() - s_time

    @staticmethod
    def _fusable(p: QuantParameter) -> bool:
        """An entry _receive decodes (_decode_stoch's inputs: byte planes of one size, a numeric norm)."""
        d, g = p.data, p.signs
        return (isinstance(d, torch.Tensor) and isinstance(g, torch.Tensor) and d.ndim > 1 and d.numel() > 0
                and d.element_size() == 1 and not d.is_quantized and not d.is_floating_point()
                and g.numel() == d.numel() and g.element_size() == 1 and not g.is_floating_point()
                and d.is_cuda == g.is_cuda)

    def _quantize_params(self, params: Parameters, bits: int, uniforms=None, seed=None) -> QuantParameters:
        """Biases and running metrics (ndim <= 1) are not quantized."""
        names = [name for name, p in params.items() if p.ndim > 1 and p.numel() > 0]
        for name in names:
            _require_codable(name, params[name], self.__class__.__name__)
        if uniforms is not None and {params[n].dtype for n in names} - {uniforms.dtype}:
            raise ValueError(f"{self.__class__.__name__}: injected uniforms ({uniforms.dtype}) cover one dtype bucket; "
                             f"this dict also holds {sorted(str(d) for d in {params[n].dtype for n in names})}")
        f32 = [n for n in names if params[n].dtype == torch.float32]
        tn = reference_norm()
        encoded = (_encode_stoch(params, f32, self.CODEC, bits, uniforms if uniforms is None or
                                 uniforms.dtype == torch.float32 else None, seed, tn) if f32 else {})
        for dtype in sops.DT_DTYPES:   # fp16 / bf16 / fp64: one bucket per dtype, in that dtype's arithmetic
            group = [n for n in names if params[n].dtype == dtype]
            if group:
                encoded.update(_encode_stoch_dt(params, group, self.CODEC, bits, uniforms, seed, tn))
        q_params = QuantParameters({}, 0)
        pass_signs = torch.zeros(1, dtype=torch.uint8)  # passthrough entries' unused signs, one per call
        for name, param in params.items():
            if name in encoded:
                data, signs, scale, scale_2 = encoded[name]
            elif param.ndim > 1:  # empty: vector_norm is 0 -> zero branch
                _require_codable(name, param, self.__class__.__name__)
                data = torch.zeros_like(param, dtype=torch.uint8)
                signs, scale, scale_2 = torch.ones_like(param, dtype=torch.int8), torch.tensor(0.0, dtype=param.dtype), 0
            else:
                data, signs, scale, scale_2 = param, pass_signs, 0, 0
            q_params.params[name] = QuantParameter(data=data, bits=bits, scale=scale, signs=signs, shape=param.shape,
                                                   dtype=param.dtype, q_dtype=data.dtype, scale_2=scale_2)
            q_params.size += data.nbytes
        return q_params


class QSGDChannel(_StochChannel):
    """Bi-directional QSGD (quant.py:140-252) on the MI355X HIP codec."""

    CODEC = "qsgd"


class RQSGDChannel(_StochChannel):
    """Bi-directional revised QSGD (quant.py:280-398): infinity norm, minimum factor for zero levels."""

    CODEC = "rqsgd"
    NORM_BYTES = 8


class CNATChannel(_StochChannel):
    """Bi-directional natural compression (quant.py:426-545): stochastic power-of-two exponents."""

    CODEC = "cnat"


class _Unidirectional:
    """Only client -> server is compressed; server -> client and the client's receive use the identity
    channel (quant.py:255-277,401-423,548-570)."""

    def on_server_send(self, params: Parameters) -> Tuple[CompressedParameters, float]:
        return IdentityChannel(no_compute_time=True).on_server_send(params)

    def on_client_receive(self, c_params: CompressedParameters) -> Tuple[Parameters, float]:
        return IdentityChannel(no_compute_time=True).on_client_receive(c_params)


class UQSGDChannel(_Unidirectional, QSGDChannel):
    """Uni-directional QSGD (quant.py:255-277)."""


class URQSGDChannel(_Unidirectional, RQSGDChannel):
    """Uni-directional RQSGD (quant.py:401-423)."""


class UCNATChannel(_Unidirectional, CNATChannel):
    """Uni-directional CNAT (quant.py:548-570)."""
