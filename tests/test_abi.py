"""CPU: the C-ABI library loads and exports every symbol include/*.h declares; argument checks
and host-side chunk planning work without a GPU (no kernel is launched by any call here)."""

import ctypes
import os
import re

import numpy as np
import pytest

from adfl_amd import _lib
from adfl_amd._build import LIB_PATH

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADER = os.path.join(INCLUDE, "adfl_slq.h")
HEADERS = sorted(os.path.join(INCLUDE, h) for h in os.listdir(INCLUDE) if h.endswith(".h"))


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(adfl_\w+)\s*\(", text, flags=re.M))
    return sorted(names)


def test_headers_present():
    assert [os.path.basename(h) for h in HEADERS] == ["adfl_host.h", "adfl_qerror.h", "adfl_slq.h", "adfl_stoch.h"]


def test_header_declares_the_binding_table():
    assert declared_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    raw = ctypes.CDLL(LIB_PATH)
    for name in declared_functions():
        assert hasattr(raw, name), name


def test_exports_via_nm():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (adfl_\w+)", out))
    assert exported == set(declared_functions())


def test_abi_version_and_constants():
    lib = _lib.load()
    assert lib.adfl_slq_abi_version() == _lib.ABI_VERSION
    assert lib.adfl_slq_workspace_bytes() >= (2048 + 1) * 4
    text = open(HEADER).read()
    assert f"#define ADFL_SLQ_ALIGN_ELEMS {_lib.ALIGN_ELEMS}" in text
    assert f"#define ADFL_SLQ_CHUNK_ELEMS {_lib.CHUNK_ELEMS}" in text
    assert ctypes.sizeof(_lib.Chunk) == 24


def test_reference_norm_short_bounds_per_dtype():
    """Host-only queries of the reference-order norm: the short-tensor bound per dtype (one block per tensor:
    fp32 / bf16 up to 2^19, fp16 up to 2^16, fp64 likewise, csrc/torch_norm.hip) — what a caller needs for
    `kinds` — and the scratch size."""
    lib = _lib.load()
    got = [lib.adfl_torch_norm_short_max_dt(d) for d in (_lib.DTYPE_F32, _lib.DTYPE_BF16, _lib.DTYPE_F16, _lib.DTYPE_F64)]
    assert got == [1 << 19, 1 << 19, 1 << 16, 1 << 16]
    assert lib.adfl_torch_norm_short_max_dt(-1) < 0 and lib.adfl_torch_norm_short_max_dt(9) < 0
    assert lib.adfl_torch_norm_short_max() == 1 << 16
    assert lib.adfl_torch_norm_scratch_bytes(100, 10) > 0 > lib.adfl_torch_norm_scratch_bytes(-1, 1)


@pytest.mark.parametrize("code,frag", [(0, "ok"), (-1, "invalid argument"), (-2, "bits"), (-3, "aligned"),
                                       (-4, "workspace")])
def test_strerror(code, frag):
    assert frag in _lib.load().adfl_slq_strerror(code).decode()


def test_argument_errors_return_codes_without_launching():
    lib = _lib.load()
    assert lib.adfl_slq_encode(None, 10, 8, None, None, None, 0, None) == -1
    assert lib.adfl_slq_encode(16, 10, 0, 16, 16, 16, 1 << 20, None) == -2       # bits checked first
    assert lib.adfl_slq_encode(16, 10, 17, 16, 16, 16, 1 << 20, None) == -2
    assert lib.adfl_slq_absmax(20, 10, 16, 1 << 20, None) == -3                  # misaligned x
    assert lib.adfl_slq_absmax(16, 10, 16, 16, None) == -4                       # workspace too small
    assert lib.adfl_slq_absmax(16, 0, 16, 1 << 20, None) == -1                   # empty
    assert lib.adfl_slq_absmax_value(None, 16, None) == -1
    assert lib.adfl_slq_absmax_value(20, 16, None) == -3                          # misaligned workspace
    assert lib.adfl_slq_dequantize(16, 10, 16, 20, None) == -3
    assert lib.adfl_slq_dequantize_mean(16, 8, 2, 10, 16, 1, 16, None) == -1    # row stride < n
    assert lib.adfl_slq_dequantize_mean(16, 24, 2, 10, 16, 1, 16, None) == -3   # row stride % 16
    assert lib.adfl_slq_encode_batched(16, 16, 0, 8, 16, 16, 16, None) == -1
    with pytest.raises(_lib.AdflError, match="bits"):
        _lib.check(-2)


def test_stochastic_argument_errors_return_codes_without_launching():
    lib = _lib.load()
    assert lib.adfl_stoch_workspace_bytes(100) == 1600
    # norms: bad mode, small workspace, misaligned x
    assert lib.adfl_stoch_norms_batched(16, 16, 1, 7, 16, 1 << 20, 16, 16, None) == -1
    assert lib.adfl_stoch_norms_batched(16, 16, 4, 0, 16, 63, 16, None, None) == -4
    assert lib.adfl_stoch_norms_batched(20, 16, 1, 0, 16, 1 << 20, 16, None, None) == -3
    assert lib.adfl_stoch_norms_batched(16, None, 1, 0, 16, 1 << 20, 16, None, None) == -1
    # quantize / encode: bits, null planes, misaligned uniforms
    assert lib.adfl_qsgd_quantize_batched(16, 16, 1, 0, 16, None, 0, 0, 16, 16, None) == -2
    assert lib.adfl_qsgd_quantize_batched(16, 16, 1, 8, 16, None, 0, 0, None, 16, None) == -1
    assert lib.adfl_qsgd_quantize_batched(16, 16, 1, 8, 16, 20, 0, 0, 16, 16, None) == -3
    assert lib.adfl_qsgd_encode_batched(16, 16, 1, 17, None, 0, 0, 16, 1 << 20, 16, 16, 16, None) == -2
    assert lib.adfl_rqsgd_encode_batched(16, 16, 1, 8, None, 0, 0, 16, 1 << 20, 16, 16, 16, None, None) == -1
    assert lib.adfl_cnat_encode_batched(16, 16, 1, 8, None, 0, 0, 16, 8, 16, 16, 16, None) == -4
    assert lib.adfl_cnat_encode_batched(16, 16, 0, 8, None, 0, 0, 16, 1 << 20, 16, 16, 16, None) == -1
    # decoders
    assert lib.adfl_qsgd_dequantize_batched(16, 16, 16, 1, 8, 16, 20, None) == -3
    assert lib.adfl_rqsgd_dequantize_batched(16, 16, 16, 1, 8, 16, None, 16, None) == -1
    assert lib.adfl_cnat_dequantize_batched(16, 16, 16, 1, None, 16, None) == -1
    assert lib.adfl_philox_uniforms(16, 0, 0, 1, 0, None) == -1
    # fused decode + accumulate
    assert lib.adfl_slq_dequantize_add_batched(16, 16, 1, 16, 16, 1, 0, None) == -1
    assert lib.adfl_slq_dequantize_add_batched(16, 16, 1, 16, None, 1, 1, None) == -1
    assert lib.adfl_slq_dequantize_add_batched(20, 16, 1, 16, 16, 1, 1, None) == -3


def test_dtype_and_bucket_mean_argument_errors_return_codes_without_launching():
    """The fp16 / bf16 / fp64 stochastic entries and the bucketed peer means check their arguments before
    any HIP call (so this runs without a GPU)."""
    lib = _lib.load()
    F16, F64, QSGD, CNAT = _lib.DTYPE_F16, _lib.DTYPE_F64, _lib.CODEC_QSGD, _lib.CODEC_CNAT
    # dtype / codec / bits / planes / alignment
    assert lib.adfl_stoch_quantize_batched_dt(QSGD, 0, 16, 16, 1, 8, 16, None, 0, 0, 16, 16, None) == -1   # fp32 here
    assert lib.adfl_stoch_quantize_batched_dt(9, F16, 16, 16, 1, 8, 16, None, 0, 0, 16, 16, None) == -1
    assert lib.adfl_stoch_quantize_batched_dt(QSGD, F16, 16, 16, 1, 0, 16, None, 0, 0, 16, 16, None) == -2
    assert lib.adfl_stoch_quantize_batched_dt(QSGD, F16, 16, 16, 1, 8, None, None, 0, 0, 16, 16, None) == -1
    assert lib.adfl_stoch_quantize_batched_dt(QSGD, F16, 20, 16, 1, 8, 16, None, 0, 0, 16, 16, None) == -3
    assert lib.adfl_stoch_quantize_batched_dt(CNAT, F64, 16, 16, 1, 8, 16, 24, 0, 0, 16, 16, None) == -3
    assert lib.adfl_stoch_quantize_batched_dt(CNAT, F64, 16, 16, 1, 8, 16, None, 0, 0, 16, 24, None) == -3
    assert lib.adfl_stoch_norms_batched_dt(F16, 16, 16, 4, 0, 16, 63, 16, None, None) == -4      # workspace
    assert lib.adfl_stoch_norms_batched_dt(F16, 16, 16, 1, 7, 16, 1 << 20, 16, None, None) == -1  # mode
    assert lib.adfl_stoch_norms_batched_dt(F16, 16, 16, 0, 0, 16, 1 << 20, 16, None, None) == -1  # no chunks
    assert lib.adfl_stoch_encode_batched_dt(_lib.CODEC_RQSGD, F16, 16, 16, 1, 8, None, 0, 0, 16, 1 << 20, 16, 16,
                                            16, None, None) == -1                                   # RQSGD needs mins
    assert lib.adfl_philox_uniforms_dt(7, 16, 10, 0, 1, 0, None) == -1
    assert lib.adfl_philox_uniforms_dt(F16, 16, 0, 0, 1, 0, None) == -1
    # bucketed peer means: row stride a 16-byte multiple, aligned rows / output, self row in range
    assert lib.adfl_slq_dequantize_mean_batched(16, 24, 2, 16, 1, 16, 1, -1, None, 16, None) == -3
    assert lib.adfl_slq_dequantize_mean_batched(16, 32, 2, 16, 1, 16, 1, 2, 16, 16, None) == -1
    assert lib.adfl_slq_dequantize_mean_batched_int4(16, 32, 2, 16, 1, 16, 1, 0, None, 16, None) == -1
    assert lib.adfl_slq_dequantize_mean_batched_int4(20, 32, 2, 16, 1, 16, 1, -1, None, 16, None) == -3
    assert lib.adfl_slq_dequantize_mean_batched_int4(16, 32, 0, 16, 1, 16, 1, -1, None, 16, None) == -1
    # stochastic server mean: codec, minima for RQSGD, K, strides, bits, alignment
    m = lib.adfl_stoch_dequantize_mean_batched
    assert m(9, 16, 16, 32, 2, 16, 1, 8, 16, None, 1, 16, None) == -1
    assert m(_lib.CODEC_RQSGD, 16, 16, 32, 2, 16, 1, 8, 16, None, 1, 16, None) == -1
    assert m(QSGD, 16, 16, 32, 0, 16, 1, 8, 16, None, 1, 16, None) == -1
    assert m(QSGD, 16, 16, 0, 2, 16, 1, 8, 16, None, 1, 16, None) == -1
    assert m(QSGD, 16, 16, 32, 2, 16, 1, 8, 16, None, 0, 16, None) == -1
    assert m(QSGD, 16, 16, 32, 2, 16, 1, 0, 16, None, 1, 16, None) == -2
    assert m(QSGD, 16, 16, 24, 2, 16, 1, 8, 16, None, 1, 16, None) == -3
    assert m(CNAT, 20, 16, 32, 2, 16, 1, 0, 16, None, 1, 16, None) == -3
    assert m(CNAT, 16, 16, 32, 2, 16, 1, 0, 16, None, 1, 24, None) == -3


def test_build_chunks_host_planning():
    lib = _lib.load()
    sizes = np.array([10, 8192, 8193, 64, 3 * 8192 + 5], np.int64)
    offsets = np.array([0, 64, 8256, 16512, 16576], np.int64)
    n = lib.adfl_slq_build_chunks(offsets.ctypes.data, sizes.ctypes.data, len(sizes), None, 0)
    assert n == 1 + 1 + 2 + 1 + 4
    chunks = (_lib.Chunk * n)()
    assert lib.adfl_slq_build_chunks(offsets.ctypes.data, sizes.ctypes.data, len(sizes), chunks, n) == n
    rows = [(c.start, c.len, c.tensor, c.first_chunk, c.nchunks) for c in chunks]
    assert rows[2] == (8256, 8192, 2, 2, 2) and rows[3] == (16448, 1, 2, 2, 2)
    assert rows[-1] == (16576 + 3 * 8192, 5, 4, 5, 4)
    covered = {t: sum(c.len for c in chunks if c.tensor == t) for t in range(len(sizes))}
    assert [covered[t] for t in range(len(sizes))] == sizes.tolist()
    # capacity too small, misaligned offset, empty tensor
    assert lib.adfl_slq_build_chunks(offsets.ctypes.data, sizes.ctypes.data, len(sizes), chunks, n - 1) == -1
    bad = offsets.copy()
    bad[1] = -1
    assert lib.adfl_slq_build_chunks(bad.ctypes.data, sizes.ctypes.data, len(sizes), None, 0) == -1
    bad[1] = 65  # unaligned offsets are valid (compact buckets)
    assert lib.adfl_slq_build_chunks(bad.ctypes.data, sizes.ctypes.data, len(sizes), None, 0) == n
    zero = sizes.copy()
    zero[0] = 0
    assert lib.adfl_slq_build_chunks(offsets.ctypes.data, zero.ctypes.data, len(sizes), None, 0) == -1


def test_philox_rounds_match_the_oracle():
    """The stochastic codecs' stream is Philox4x32-7 unless the library was built with ADFL_PHILOX_ROUNDS=10
    (csrc/philox.h); the oracle follows the same variable."""
    import stoch_oracle as so
    assert _lib.load().adfl_philox_rounds() == so.PHILOX_ROUNDS
