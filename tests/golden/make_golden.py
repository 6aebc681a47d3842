"""Generate the golden vectors that pin the oracle and the HIP codec to the reference's own output.

Run in the build container (the reference tree exists only there):

    python tests/golden/make_golden.py

Every expected value below is produced by EXECUTING the reference codec in place
(``Src/ADFL/Channel/quant.py:61-112`` through ``ref_loader``) on torch 2.10.0+rocm7.0, quantized
engine x86 — the oracle version recorded in SURVEY.md §8c. The reference's own tests pin no values at
this boundary (``Src/ADFL/Channel/Tests/test_quant.py`` only prints), so these fixtures are the pin.

Outputs (data only — inputs and expected outputs; no reference source is stored):
  tests/golden/slq_small.npz     raw arrays for small cases
  tests/golden/int4.npz          pack_4bit / unpack_4bit vectors (Src/ADFL/compression.py:35-66)
  tests/golden/manifest.json     case list, scale bits, SHA-256 digests for recipe-defined large cases,
                                 passthrough metadata, simulate_bandwidth / to_json results
"""

import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import recipes  # noqa: E402
from ref_loader import load_reference  # noqa: E402


def f32_bits(v: float) -> int:
    return int(np.array([v], dtype=np.float32).view(np.uint32)[0])


def scale_bits_checked(scale) -> int:
    """Reference scale is a Python float holding an exact fp32 value (quant.py:100-104)."""
    s32 = np.float32(scale)
    assert (np.isnan(scale) and np.isnan(s32)) or float(s32) == float(scale), scale
    return f32_bits(scale)


def run_slq(ref, params: dict, bits: int):
    """Encode with the reference SLQChannel and decode back; returns (QuantParameters, decoded dict)."""
    ch = ref.quant.SLQChannel(bits=bits)
    qp, _ = ch.on_client_send(params)
    dec, _ = ch.on_server_receive(qp)
    return qp, dec


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    print("torch", torch.__version__, "engine", torch.backends.quantized.engine)
    arrays = {}
    manifest = {"torch": torch.__version__, "quant_engine": torch.backends.quantized.engine,
                "generator": "tests/golden/make_golden.py", "raw": [], "recipe": [], "edge": [],
                "bucket": [], "int4": [], "passthrough": {}, "bandwidth": [], "to_json": {}, "size": []}

    def add_raw(name, x: np.ndarray, bits: int, group: str = "raw"):
        t = torch.from_numpy(x.copy())
        qp, dec = run_slq(ref, {"w": t}, bits)
        p = qp.params["w"]
        q = p.data.int_repr().numpy()
        arrays[f"{name}__x"] = x
        arrays[f"{name}__q"] = q
        arrays[f"{name}__deq"] = dec["w"].numpy()
        manifest[group].append({"name": name, "bits": bits, "shape": list(x.shape),
                                "scale_bits": scale_bits_checked(p.scale), "size": qp.size})

    # ---- A. small random cases, stored raw -------------------------------------------------------
    for shape in [(2, 5), (7, 1), (1, 1), (33, 31), (3, 7, 5), (128, 129), (5, 4097), (1, 16), (1, 17)]:
        for bits in (8, 4, 2):
            x = recipes.randn(shape, 0, 1e-3)
            add_raw(f"randn_{'x'.join(map(str, shape))}_s0_b{bits}", x, bits)
    for seed, mult in [(1, 1.0), (2, 1e-30), (3, 1e20), (4, 1e-38), (5, 3e36)]:
        for bits in (8, 4):
            x = recipes.randn((31, 67), seed, mult)
            add_raw(f"randn_31x67_s{seed}_m{mult:g}_b{bits}", x, bits)
    add_raw("heavy_64x257_b8", recipes.heavy_tail((64, 257), 7, 1e-3), 8)
    # every other bit width SLQChannel accepts (q_max = 2**(bits-1)-1: bits=1 -> q_max 0, scale inf;
    # bits >= 9 -> q_max > 127, the int8 container clamps)
    for bits in (1, 3, 5, 6, 7, 9, 12, 16):
        add_raw(f"randn_33x31_s9_b{bits}", recipes.randn((33, 31), 9, 1e-3), bits)
    # C1: CPU 2-client small model, Examples/ray_async.py:63-70 ([10,3072] weight + [10] bias)
    add_raw("c1_fc_weight_b8", recipes.randn((10, 3072), 11, 0.02), 8)

    # ---- B. edge cases ----------------------------------------------------
    nan, inf = float("nan"), float("inf")
    edge = {
        "ties": np.array([[127, .5, 1.5, 2.5, -.5, -1.5, -2.5, 126.5, 3.5, -3.5, 0.0, -127]], np.float32),
        "zeros": np.zeros((4, 9), np.float32),
        "negzeros": np.full((3, 5), -0.0, np.float32),
        "onehot": np.pad(np.array([[5.0]], np.float32), ((0, 2), (3, 9))),
        "nan": recipes.randn((4, 33), 21, 1.0),
        "pinf": recipes.randn((4, 33), 22, 1.0),
        "ninf": recipes.randn((4, 33), 23, 1.0),
        "nan_and_inf": recipes.randn((2, 19), 24, 1.0),
        "denormal_all": recipes.randn((5, 13), 25, 1e-40),
        "denormal_some": recipes.randn((5, 13), 26, 1.0),
        "tiny": recipes.randn((5, 13), 27, 1e-38),
        "negzero_mix": np.array([[-0.0, 0.0, -1.0, 1.0, -0.0, 0.25, -0.25]], np.float32),
        "single": np.array([[-3.0]], np.float32),
        "near_max": np.array([[3.4028235e38, -3.4028235e38, 1e38, -2e38, 0.0, 1.0]], np.float32),
        "all_equal": np.full((3, 3), 0.7, np.float32),
        "halfway_scale": (np.arange(-40, 41, dtype=np.float32).reshape(1, -1) + 0.5),
    }
    edge["nan"][1, 7] = nan
    edge["pinf"][2, 30] = inf
    edge["ninf"][0, 0] = -inf
    edge["nan_and_inf"][0, 3] = inf
    edge["nan_and_inf"][1, 5] = nan
    edge["denormal_some"][3, 4:9] = np.float32(1e-41)
    for name, x in edge.items():
        for bits in (8, 4, 2):
            add_raw(f"edge_{name}_b{bits}", x, bits, group="edge")
    for name in ("ties", "zeros", "nan", "pinf", "ninf", "denormal_all", "tiny", "near_max"):
        for bits in (1, 16):
            add_raw(f"edge_{name}_b{bits}", edge[name], bits, group="edge")

    # ---- C. recipe-defined larger cases, stored as SHA-256 ---------------------------------------
    recipe_cases = [
        ({"kind": "randn", "shape": [1024, 1023], "seed": 0, "mult": 1e-3}, (8, 4, 2)),
        ({"kind": "randn", "shape": [4096, 1023], "seed": 1, "mult": 1e-3}, (8,)),
        ({"kind": "heavy_tail", "shape": [2048, 4096], "seed": 2, "mult": 1e-3}, (8,)),
        # C2: 1 GiB flat gradient (BASELINE.json configs[1]); shape [262144, 1024]
        ({"kind": "randn", "shape": [262144, 1024], "seed": 0, "mult": 1e-3}, (8, 4)),
    ]
    for rec, bit_list in recipe_cases:
        x = recipes.make(rec)
        for bits in bit_list:
            t0 = time.time()
            qp, dec = run_slq(ref, {"w": torch.from_numpy(x)}, bits)
            p = qp.params["w"]
            q = p.data.int_repr().numpy()
            manifest["recipe"].append({
                "recipe": rec, "bits": bits, "scale_bits": scale_bits_checked(p.scale),
                "q_sha256": recipes.sha256(q), "deq_sha256": recipes.sha256(dec["w"].numpy()),
                "q_sum": int(q.astype(np.int64).sum()), "q_abs_sum": int(np.abs(q.astype(np.int64)).sum()),
            })
            print(f"recipe {rec['shape']} b{bits}: {time.time() - t0:.2f}s")
        del x

    # ---- D. C3 bucketed update: 256 tensors, per-tensor scales -----------------------------------
    for layout in ("equal", "loguniform"):
        tensors = recipes.bucket_tensors(layout, 0, 1e-3)
        params = {k: torch.from_numpy(v) for k, v in tensors.items()}
        qp, dec = run_slq(ref, params, 8)
        names = list(params)
        q_cat = np.concatenate([qp.params[k].data.int_repr().numpy().reshape(-1) for k in names])
        d_cat = np.concatenate([dec[k].numpy().reshape(-1) for k in names])
        manifest["bucket"].append({
            "layout": layout, "seed": 0, "mult": 1e-3, "bits": 8, "sizes": recipes.bucket_sizes(layout, 0),
            "scale_bits": [scale_bits_checked(qp.params[k].scale) for k in names],
            "q_sha256": recipes.sha256(q_cat), "deq_sha256": recipes.sha256(d_cat), "size": qp.size})

    # ---- E. int4 nibble layout (Src/ADFL/compression.py:35-66) ------------------------------------
    def add_int4(name, q: np.ndarray):
        t = torch.from_numpy(q.copy())
        packed = ref.compression.pack_4bit(t).numpy()
        unpacked = ref.compression.unpack_4bit(bytearray(packed.tobytes()), torch.Size(q.shape)).numpy()
        arrays[f"int4_{name}__q"] = q
        arrays[f"int4_{name}__packed"] = packed
        arrays[f"int4_{name}__unpacked"] = unpacked
        manifest["int4"].append({"name": name, "shape": list(q.shape)})

    rng = np.random.default_rng(5)
    add_int4("range_even", rng.integers(-8, 8, size=(6, 10), dtype=np.int8))
    add_int4("range_odd", rng.integers(-8, 8, size=(3, 7), dtype=np.int8))
    add_int4("single", np.array([[-5]], np.int8))
    add_int4("out_of_range", np.array([[127, -128, 127, 8, -9, 100, -100, 7, -8]], np.int8))
    add_int4("full_byte_range", np.arange(-128, 128, dtype=np.int16).astype(np.int8).reshape(16, 16))
    for nm in ("randn_33x31_s0_b4", "edge_zeros_b4", "edge_nan_b4", "randn_5x4097_s0_b4"):
        add_int4("slq_" + nm, arrays[f"{nm}__q"])

    # ---- F. passthrough entries (quant.py:80-81) -------------------------------------------------
    bias = torch.from_numpy(recipes.randn((10,), 31, 1.0))
    nbt = torch.tensor(7, dtype=torch.int64)
    ivec = torch.arange(5, dtype=torch.int64)
    ch = ref.quant.SLQChannel(bits=8)
    qp, _ = ch.on_client_send({"bias": bias, "num_batches_tracked": nbt, "ivec": ivec})
    dec, _ = ch.on_server_receive(qp)
    manifest["passthrough"] = {
        name: {"scale": p.scale, "scale_type": type(p.scale).__name__, "same_object": p.data is src,
               "dtype": str(p.dtype), "q_dtype": str(p.q_dtype), "shape": list(p.shape), "bits": p.bits,
               "signs": p.signs.tolist(), "signs_dtype": str(p.signs.dtype),
               "decoded_same_object": dec[name] is src}
        for (name, p), src in zip(qp.params.items(), (bias, nbt, ivec))}
    manifest["passthrough"]["__size__"] = qp.size
    wq, _ = ch.on_client_send({"w": torch.ones(2, 3)})
    w = wq.params["w"]
    manifest["quant_meta"] = {"dtype": str(w.dtype), "q_dtype": str(w.q_dtype), "bits": w.bits,
                              "signs": w.signs.tolist(), "signs_dtype": str(w.signs.dtype),
                              "scale_type": type(w.scale).__name__, "data_dtype": str(w.data.dtype),
                              "scale_2": w.scale_2, "shape": list(w.shape)}

    # ---- G. simulate_bandwidth / to_json / size accounting (quant.py:40-58, channel.py:83-99) -----
    bw_params = {"non_bias": torch.from_numpy(recipes.randn((2, 5), 41, 1.0)),
                 "bias": torch.from_numpy(recipes.randn((10,), 42, 1.0)),
                 "conv": torch.from_numpy(recipes.randn((4, 3, 3, 3), 43, 1.0)),
                 "nbt": torch.tensor(3, dtype=torch.int64)}
    for bits in (8, 4, 2):
        for mbps in (1e9, 5e8):
            t = ref.quant.SLQChannel(bits=bits).simulate_bandwidth(bw_params, mbps)
            manifest["bandwidth"].append({"channel": "SLQChannel", "bits": bits, "mbps": mbps, "seconds": t})
            t = ref.quant.USLQChannel(bits=bits).simulate_bandwidth(bw_params, mbps)
            manifest["bandwidth"].append({"channel": "USLQChannel", "bits": bits, "mbps": mbps, "seconds": t})
    t = ref.channel.IdentityChannel(no_compute_time=True).simulate_bandwidth(bw_params, 1e9)
    manifest["bandwidth"].append({"channel": "IdentityChannel", "bits": None, "mbps": 1e9, "seconds": t})
    manifest["to_json"] = {
        "SLQChannel_8": ref.quant.SLQChannel(bits=8).to_json(),
        "USLQChannel_4": ref.quant.USLQChannel(bits=4).to_json(),
        "IdentityChannel": ref.channel.IdentityChannel(no_compute_time=False).to_json(),
    }
    qp, _ = ref.quant.SLQChannel(bits=8).on_client_send(bw_params)
    manifest["size"].append({"what": "SLQChannel(8) bw_params", "size": qp.size})
    bp, _ = ref.quant.USLQChannel(bits=8).on_server_send(bw_params)
    manifest["size"].append({"what": "USLQChannel(8).on_server_send bw_params", "size": bp.size,
                             "type": type(bp).__name__})

    np.savez_compressed(os.path.join(HERE, "slq_small.npz"),
                        **{k: v for k, v in arrays.items() if not k.startswith("int4_")})
    np.savez_compressed(os.path.join(HERE, "int4.npz"), **{k: v for k, v in arrays.items() if k.startswith("int4_")})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=False, default=str)
    print("wrote", len(arrays), "arrays;", len(manifest["recipe"]), "recipe cases")


if __name__ == "__main__":
    main()
