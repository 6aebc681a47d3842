"""Per-phase wall time of SLQChannel's host-to-host path on the C3 dict (256 weights + 256 biases, CPU
tensors): where the milliseconds of on_client_send / on_server_receive go. Each phase is synchronised
separately, so the phases add up to more than the real (overlapped) call.

    python tools/channel_breakdown.py
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ad-federatedlearning_amd"))
from adfl_amd import ops  # noqa: E402
from adfl_amd.Channel import SLQChannel  # noqa: E402
from adfl_amd.Channel.quant import _gather, _int8_view, _staging  # noqa: E402


def main():
    base, rem = divmod(11_689_512, 256)
    params = {}
    for i in range(256):
        params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0)) * 1e-3
        params[f"layer{i}.bias"] = torch.randn(64)
    names = [n for n, p in params.items() if p.ndim > 1]
    tensors = [params[n] for n in names]
    ch = SLQChannel(8)
    for _ in range(3):
        qp, _ = ch.on_client_send(params)
        ch.on_server_receive(qp)
    st = _staging()
    dev = st.device
    lay = st.layout(tuple(int(t.numel()) for t in tensors))
    res = {}

    def t(name, fn, reps=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / reps * 1e3, 3)

    host = st.buf("x_host", lay.total, torch.float32, pinned=True)
    devb = st.buf("x", lay.total, torch.float32)
    q = st.buf("q", lay.total, torch.int8)
    qh = st.buf("q_host", lay.total, torch.int8, pinned=True)
    t("encode.gather_cat_into_pinned", lambda: _gather(tensors, lay, host))
    t("encode.h2d", lambda: devb.copy_(host, non_blocking=True))
    t("encode.kernels", lambda: ops.encode_batched(devb, lay, 8, q=q))
    t("encode.d2h_payload", lambda: qh.copy_(q, non_blocking=True))
    parts = [p[:n].view(tt.shape) for p, n, tt in zip(torch.split(qh, lay.padded.tolist()), lay.sizes.tolist(), tensors)]
    t("encode.make_qint8_per_tensor", lambda: [torch._make_per_tensor_quantized_tensor(p, 0.01, 0) for p in parts])
    t("encode.total_on_client_send", lambda: ch.on_client_send(params))
    items = [(n, qp.params[n].data) for n in names]
    t("decode.int8_views", lambda: [_int8_view(x) for _, x in items])
    views = [_int8_view(x) for _, x in items]
    dq_host = st.buf("dq_host", lay.total, torch.int8, pinned=True)
    t("decode.gather_cat_into_pinned", lambda: _gather(views, lay, dq_host))
    dq = st.buf("dq", lay.total, torch.int8)
    t("decode.h2d_payload", lambda: dq.copy_(dq_host, non_blocking=True))
    s = torch.full((lay.ntensors,), 0.01, device=dev)
    out = torch.empty(lay.total, device=dev)
    t("decode.kernel", lambda: ops.decode_batched(dq, s, lay, out=out))
    oh = torch.empty(lay.total, pin_memory=True)
    t("decode.d2h_out", lambda: oh.copy_(out, non_blocking=True))
    t("decode.alloc_pinned_out", lambda: torch.empty(lay.total, pin_memory=True))
    t("decode.total_on_server_receive", lambda: ch.on_server_receive(qp))
    res["torch_threads"] = torch.get_num_threads()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
