"""Golden vectors for the aggregate step after the codec, made by EXECUTING the reference.

Run in the build container (the reference tree exists only there):

    python tests/golden/make_golden_aggregate.py

What is executed in place (``ref_loader``; torch 2.10.0+rocm7.0 on this container's x86-64 host, whose
CPU sum runs ATen's AVX2 kernel — ATen has no AVX-512 sum kernel, so an AVX-512 host such as the GPU
box's EPYC 9575F takes the same one):

* ``SLQChannel(bits)`` (``Src/ADFL/Channel/quant.py:15-112``) encodes each client's update and
  ``on_server_receive`` decodes it; ``simple_aggregate`` (``Src/ADFL/model.py:221-234``) averages the K
  decoded dicts — the synchronous server's aggregate (``Src/ADFL/Strategy/simple.py:83-89``) that
  ``SLQChannel.receive_mean`` fuses. K = 1..5, 7, 8, 10, 16, 17, 20, 33, 64 at bits 8 (``Src/main.py`` runs
  10, 16 and 20 clients), K = 3, 5, 8, 16, 20 at bits 4.
* The peer mean of ``Examples/ray_ad.py:183-188`` / ``Src/ADFL/Client/async_peer.py:170-174``
  (``torch.stack([received..., own]).mean(dim=0)``; those files import ray, so the expression itself is
  executed on the reference's decoded tensors) with the receiving client's own update exact and last, K = 2, 5, 8, 16, 20.
* ``QSGDChannel(8)``, ``RQSGDChannel(4)``, ``CNATChannel(8)``: each client encoded under
  ``torch.manual_seed(7000 + client)`` (the reference's ``torch.rand_like``), decoded, and
  ``simple_aggregate``-d at K = 5, 8, 16, 20. Their payloads are stored (the HIP channels draw other
  uniforms), so the GPU test feeds the reference's own payloads to ``receive_mean``.
* ``parameter_relative_mse`` / ``parameter_cosine_similarity`` (``Src/ADFL/model.py:256-323``) of each
  client's update against its SLQ decode, ``exclude_bias=True`` — the worker's q-error metrics
  (``Src/ADFL/Client/worker.py:186-189``).

Inputs are recipes (numpy PCG64, ``recipes.randn``) with their SHA-256 in the manifest; a few clients carry
special tensors (all zeros, a NaN, an inf). The tensor shapes cover every branch of torch's summation
order: n % 32 tails, 2 <= n < 8, n == 1.

Outputs (data only):
  tests/golden/aggregate.npz            expected aggregates / peer means per (channel, K, tensor),
                                        stochastic payloads (levels, signs) per (codec, client, tensor)
  tests/golden/aggregate_manifest.json  shapes, client recipes + SHA-256, K lists, payload scales
                                        (fp32 bits), q-error values (repr of the Python floats)
"""

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import recipes  # noqa: E402
from ref_loader import load_reference  # noqa: E402

# name -> shape; n = 432 (n % 32 = 16), 330 (10), 35 (3), 6 (2 <= n < 8), 1, 3, 9 (no full 32-group),
# 2064 (16), 1313 (1), 1024 (0)
SHAPES = {"conv.weight": (16, 3, 3, 3), "fc.weight": (10, 33), "mid.weight": (7, 5), "six.weight": (2, 3),
          "one.weight": (1, 1), "three.weight": (3, 1), "nine.weight": (1, 9), "big.weight": (16, 129),
          "rag.weight": (13, 101), "sq.weight": (32, 32)}
BIASES = {"fc.bias": (10,)}
K_SLQ = [1, 2, 3, 4, 5, 7, 8, 10, 16, 17, 20, 33, 64]
K_SLQ4 = [3, 5, 8, 16, 20]       # bits = 4 (PackedSLQChannel's decode)
K_PEER = [2, 5, 8, 16, 20]
K_STOCH = [5, 8, 16, 20]
STOCH = {"qsgd": ("QSGDChannel", 8), "rqsgd": ("RQSGDChannel", 4), "cnat": ("CNATChannel", 8)}
NCLIENTS = max(K_SLQ)


def client_arrays(c: int) -> dict:
    """Client c's update as numpy arrays (shared with the tests through this function's recipe)."""
    out = {}
    for i, (name, shape) in enumerate(SHAPES.items()):
        out[name] = recipes.randn(shape, 50_000 + 97 * c + i, 10.0 ** -(1 + (i + c) % 4))
    for i, (name, shape) in enumerate(BIASES.items()):
        out[name] = recipes.randn(shape, 90_000 + 97 * c + i, 0.1)
    # special tensors: all zeros (scale 0), a NaN (scale NaN), an inf (scale inf)
    if c == 2:
        out["mid.weight"] = np.zeros(SHAPES["mid.weight"], np.float32)
    if c == 6:
        out["fc.weight"].reshape(-1)[5] = np.nan
    if c == 9:
        out["six.weight"].reshape(-1)[1] = np.inf
    return out


def client_dict(c: int) -> dict:
    d = {n: torch.from_numpy(a.copy()) for n, a in client_arrays(c).items()}
    d["bn.num_batches_tracked"] = torch.tensor(3 + c, dtype=torch.int64)
    return d


def f32_bits(v) -> int:
    return int(np.array([float(v)], dtype=np.float32).view(np.uint32)[0])


def scale_record(v):
    if isinstance(v, torch.Tensor):
        assert v.ndim == 0 and v.dtype == torch.float32
        return {"tensor": True, "bits": f32_bits(v.item())}
    if isinstance(v, int):
        return {"int": v}
    return {"bits": f32_bits(v)}


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    arrays = {}
    manifest = {"shapes": {n: list(s) for n, s in SHAPES.items()}, "biases": {n: list(s) for n, s in BIASES.items()},
                "k_slq": K_SLQ, "k_slq4": K_SLQ4, "k_peer": K_PEER, "k_stoch": K_STOCH, "stoch": {k: list(v) for k, v in STOCH.items()},
                "clients": [], "q_error": {}, "stoch_scales": {},
                "torch": torch.__version__, "cpu_capability": torch.backends.cpu.get_cpu_capability()}
    clients = [client_dict(c) for c in range(NCLIENTS)]
    for c in range(NCLIENTS):
        manifest["clients"].append({n: recipes.sha256(t.numpy()) for n, t in clients[c].items() if t.ndim})

    for bits in (8, 4):
        ch = ref.quant.SLQChannel(bits=bits)
        decoded = []
        for c in range(NCLIENTS):
            qp, _ = ch.on_client_send(clients[c])
            dec, _ = ch.on_server_receive(qp)
            decoded.append(dec)
            x = {n: t for n, t in clients[c].items()}
            manifest["q_error"][f"slq{bits}_c{c}"] = {
                "mse": repr(ref.model.parameter_relative_mse(x, dec, exclude_bias=True)),
                "cos": repr(ref.model.parameter_cosine_similarity(x, dec, exclude_bias=True))}
        for k in (K_SLQ if bits == 8 else K_SLQ4):
            for n, t in ref.model.simple_aggregate(decoded[:k]).items():
                arrays[f"slq{bits}__k{k}__{n}"] = t.numpy()
        # the peer mean at receiving client k // 2: its own update exact and appended last (ray_ad.py:183-188)
        for k in K_PEER:
            me = k // 2
            for n in SHAPES:
                rows = [decoded[r][n] for r in range(k) if r != me] + [clients[me][n]]
                arrays[f"peer{bits}__k{k}__{n}"] = torch.stack(rows).mean(dim=0).numpy()

    for codec, (cls, bits) in STOCH.items():
        ch = getattr(ref.quant, cls)(bits)
        decoded = []
        for c in range(max(K_STOCH)):
            torch.manual_seed(7000 + c)
            qp, _ = ch.on_client_send(clients[c])
            for n in SHAPES:
                p = qp.params[n]
                arrays[f"{codec}__c{c}__{n}__q"] = p.data.numpy().view(np.uint8)
                arrays[f"{codec}__c{c}__{n}__signs"] = p.signs.numpy()
                manifest["stoch_scales"][f"{codec}__c{c}__{n}"] = {"scale": scale_record(p.scale),
                                                                   "scale_2": scale_record(p.scale_2)}
            dec, _ = ch.on_server_receive(qp)
            decoded.append(dec)
        for k in K_STOCH:
            for n, t in ref.model.simple_aggregate(decoded[:k]).items():
                arrays[f"{codec}__k{k}__{n}"] = t.numpy()

    np.savez_compressed(os.path.join(HERE, "aggregate.npz"), **arrays)
    with open(os.path.join(HERE, "aggregate_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(arrays)} arrays")


if __name__ == "__main__":
    main()
