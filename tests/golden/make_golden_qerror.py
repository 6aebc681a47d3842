"""Golden q-error metrics at model sizes, made by EXECUTING the reference.

Run in the build container (the reference tree exists only there):

    python tests/golden/make_golden_qerror.py

``tests/golden/aggregate_manifest.json`` already holds the reference's q-error metrics for small dicts
(every tensor below torch's 32,768-element grain, so every sum is single-threaded). This adds dicts where
torch's two-pass parallel sum and the cascade's larger level steps apply: per tensor above 32,768 elements
and over the concatenated vector of ``cosine_similarity``, at several thread counts.

Executed in place (``ref_loader``): ``SLQChannel(bits).on_client_send`` + ``on_server_receive``
(``Src/ADFL/Channel/quant.py:15-112``), then ``parameter_relative_mse`` / ``parameter_cosine_similarity``
with ``exclude_bias=True`` (``Src/ADFL/model.py:256-323``) — the worker's q-error metrics
(``Src/ADFL/Client/worker.py:186-189``) — under ``torch.set_num_threads(T)``.

Inputs are recipes (``recipes.randn``) with their SHA-256 in the manifest; outputs are the Python floats'
``repr``. Output (data only): tests/golden/qerror_manifest.json
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

THREADS = [1, 3, 8, 16]
BITS = [8, 4]


def resnet18_shapes():
    """torchvision's resnet18 state dict shapes, in its order (11,689,512 parameters; BN running stats and
    num_batches_tracked left out — the channel passes ndim <= 1 entries through either way)."""
    out = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    cin = 64
    for li, cout in enumerate((64, 128, 256, 512), start=1):
        for b in range(2):
            pre = f"layer{li}.{b}"
            c_in = cin if b == 0 else cout
            out += [(f"{pre}.conv1.weight", (cout, c_in, 3, 3)), (f"{pre}.bn1.weight", (cout,)),
                    (f"{pre}.bn1.bias", (cout,)), (f"{pre}.conv2.weight", (cout, cout, 3, 3)),
                    (f"{pre}.bn2.weight", (cout,)), (f"{pre}.bn2.bias", (cout,))]
            if b == 0 and li > 1:
                out += [(f"{pre}.downsample.0.weight", (cout, cin, 1, 1)), (f"{pre}.downsample.1.weight", (cout,)),
                        (f"{pre}.downsample.1.bias", (cout,))]
        cin = cout
    out += [("fc.weight", (1000, 512)), ("fc.bias", (1000,))]
    return out


# Tensors around the 32,768 grain and a large one (level power 5 per range at T = 1 above 2^24 elements).
EDGES = [("a.weight", (256, 127)), ("b.weight", (256, 128)), ("c.weight", (257, 128)), ("d.weight", (1, 7)),
         ("e.weight", (1000, 1000)), ("f.bias", (1000,)), ("g.weight", (4099, 4099))]


def dicts():
    return {
        "resnet18": [(n, s, 1e-2 if len(s) > 1 else 1e-1) for n, s in resnet18_shapes()],
        "edges": [(n, s, 10.0 ** -(1 + i % 3)) for i, (n, s) in enumerate(EDGES)],
    }


def build(spec, seed0):
    d = {}
    for i, (name, shape, mult) in enumerate(spec):
        d[name] = torch.from_numpy(recipes.randn(shape, seed0 + i, mult))
    return d


def main():
    ref = load_reference()
    man = {"torch": torch.__version__, "cpu_capability": torch.backends.cpu.get_cpu_capability(), "dicts": {}}
    for di, (name, spec) in enumerate(dicts().items()):
        seed0 = 120_000 + 1000 * di
        params = build(spec, seed0)
        entry = {"tensors": [[n, list(s), m] for n, s, m in spec], "seed0": seed0,
                 "sha256": {n: recipes.sha256(t.numpy()) for n, t in params.items()}, "metrics": {}}
        for bits in BITS:
            ch = ref.quant.SLQChannel(bits=bits)
            qp, _ = ch.on_client_send(params)
            dec, _ = ch.on_server_receive(qp)
            for t in THREADS:
                torch.set_num_threads(t)
                entry["metrics"][f"slq{bits}_t{t}"] = {
                    "mse": repr(ref.model.parameter_relative_mse(params, dec, exclude_bias=True)),
                    "cos": repr(ref.model.parameter_cosine_similarity(params, dec, exclude_bias=True))}
        man["dicts"][name] = entry
        print(name, json.dumps(entry["metrics"]))
    with open(os.path.join(HERE, "qerror_manifest.json"), "w") as f:
        json.dump(man, f, indent=1)


if __name__ == "__main__":
    main()
