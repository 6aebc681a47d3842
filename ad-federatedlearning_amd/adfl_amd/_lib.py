"""ctypes binding of libadfl_slq.so (the C ABI declared in include/adfl_slq.h, adfl_stoch.h and adfl_host.h).

The product path has no CPU fallback: if the HIP library is missing this module raises at import
time, and every op checks the status code the library returns.
"""

import ctypes
import os

# torch must be loaded first: it brings its own libamdhip64 (SONAME libamdhip64.so.7). Loading our
# library first would pull in /opt/rocm's copy too, and two HIP runtimes in one process do not share
# devices, streams or allocations. With torch loaded, our DT_NEEDED resolves to torch's runtime.
import torch  # noqa: F401

from ._build import LIB_PATH

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
INT = ctypes.c_int

ALIGN_ELEMS = 64     # ADFL_SLQ_ALIGN_ELEMS
CHUNK_ELEMS = 8192   # ADFL_SLQ_CHUNK_ELEMS
RESIDENT_CHUNKS = 8  # ADFL_SLQ_RESIDENT_CHUNKS
ABI_VERSION = 2      # ADFL_SLQ_ABI_VERSION


class AdflError(RuntimeError):
    """A non-zero status from libadfl_slq (argument error or HIP launch error)."""


class Chunk(ctypes.Structure):
    """adfl_slq_chunk."""
    _fields_ = [("start", I64), ("len", I32), ("tensor", I32), ("first_chunk", I32), ("nchunks", I32)]


# name -> (restype, argtypes); the complete exported surface of include/adfl_slq.h + adfl_stoch.h + adfl_host.h
SIGNATURES = {
    "adfl_slq_abi_version": (INT, []),
    "adfl_slq_strerror": (ctypes.c_char_p, [INT]),
    "adfl_slq_workspace_bytes": (I64, []),
    "adfl_slq_absmax": (INT, [P, I64, P, I64, P]),
    "adfl_slq_absmax_value": (INT, [P, P, P]),
    "adfl_slq_quantize": (INT, [P, I64, INT, P, P, P, P]),
    "adfl_slq_encode": (INT, [P, I64, INT, P, P, P, I64, P]),
    "adfl_slq_dequantize": (INT, [P, I64, P, P, P]),
    "adfl_slq_build_chunks": (I64, [P, P, I32, P, I64]),
    "adfl_slq_encode_batched": (INT, [P, P, I64, INT, P, P, P, P]),
    "adfl_slq_build_encode_work": (I64, [P, I64, P, I64]),
    "adfl_slq_encode_batched_work": (INT, [P, P, I64, P, I64, INT, P, P, P, P]),
    "adfl_slq_dequantize_batched": (INT, [P, P, I64, P, P, P]),
    "adfl_slq_quantize_batched_range": (INT, [P, P, I64, I64, INT, P, P, P, P]),
    "adfl_slq_absmax_batched_range": (INT, [P, P, I64, I64, P, P]),
    "adfl_slq_qerror_batched": (INT, [P, P, P, I64, P, P, P]),
    "adfl_slq_qerror_batched_int4": (INT, [P, P, P, I64, P, P, P]),
    "adfl_slq_encode_batched_int4": (INT, [P, P, I64, INT, P, P, P, P]),
    "adfl_slq_encode_batched_int4_work": (INT, [P, P, I64, P, I64, INT, P, P, P, P]),
    "adfl_slq_dequantize_batched_int4": (INT, [P, P, I64, P, P, P]),
    "adfl_slq_quantize_int4": (INT, [P, I64, INT, P, P, P, P]),
    "adfl_slq_encode_int4": (INT, [P, I64, INT, P, P, P, I64, P]),
    "adfl_slq_dequantize_int4": (INT, [P, I64, P, P, P]),
    "adfl_pack_int4": (INT, [P, I64, P, P]),
    "adfl_unpack_int4": (INT, [P, I64, P, P]),
    "adfl_slq_dequantize_mean": (INT, [P, I64, I32, I64, P, I64, P, P]),
    "adfl_slq_dequantize_mean_int4": (INT, [P, I64, I32, I64, P, I64, P, P]),
    "adfl_slq_dequantize_mean_self": (INT, [P, I64, I32, I64, P, I64, I32, P, P, P]),
    "adfl_slq_dequantize_mean_self_int4": (INT, [P, I64, I32, I64, P, I64, I32, P, P, P]),
    "adfl_slq_dequantize_add_batched": (INT, [P, P, I64, P, P, I32, I32, P]),
    "adfl_slq_dequantize_mean_batched": (INT, [P, I64, I32, P, I64, P, I64, I32, P, P, P]),
    "adfl_slq_dequantize_mean_batched_int4": (INT, [P, I64, I32, P, I64, P, I64, I32, P, P, P]),
    # adfl_stoch.h
    "adfl_stoch_workspace_bytes": (I64, [I64]),
    "adfl_stoch_norms_batched": (INT, [P, P, I64, INT, P, I64, P, P, P]),
    "adfl_torch_norm_scratch_bytes": (I64, [I64, I64]),
    "adfl_torch_norm_short_max": (I64, []),
    "adfl_torch_norm_short_max_dt": (I64, [I32]),
    "adfl_torch_norms": (INT, [I32, P, P, I64, I64, I32, I32, P, I64, P, P, P]),
    "adfl_torch_norms_work": (INT, [I32, P, P, I64, P, I64, I32, I32, P, I64, P, P, P]),
    "adfl_qerror_ref_plan": (I64, [P, I32, I32, P, I64]),
    "adfl_qerror_ref_scratch_bytes": (I64, [P]),
    "adfl_qerror_ref": (INT, [P, P, P, P, P, P, I64, P, P]),
    "adfl_qsgd_quantize_batched": (INT, [P, P, I64, INT, P, P, U64, U64, P, P, P]),
    "adfl_qsgd_encode_batched": (INT, [P, P, I64, INT, P, U64, U64, P, I64, P, P, P, P]),
    "adfl_rqsgd_encode_batched": (INT, [P, P, I64, INT, P, U64, U64, P, I64, P, P, P, P, P]),
    "adfl_qsgd_dequantize_batched": (INT, [P, P, P, I64, INT, P, P, P]),
    "adfl_rqsgd_dequantize_batched": (INT, [P, P, P, I64, INT, P, P, P, P]),
    "adfl_cnat_encode_batched": (INT, [P, P, I64, INT, P, U64, U64, P, I64, P, P, P, P]),
    "adfl_cnat_dequantize_batched": (INT, [P, P, P, I64, P, P, P]),
    "adfl_stoch_dequantize_mean_batched": (INT, [I32, P, P, I64, I32, P, I64, INT, P, P, I64, P, P]),
    "adfl_bucket_gather": (INT, [P, P, I64, P, I32, P]),
    "adfl_bucket_scatter": (INT, [P, P, I64, P, I32, P]),
    "adfl_qsgd_encode_batched_work": (INT, [P, P, I64, P, I64, INT, P, U64, U64, P, I64, P, P, P, P]),
    "adfl_rqsgd_encode_batched_work": (INT, [P, P, I64, P, I64, INT, P, U64, U64, P, I64, P, P, P, P, P]),
    "adfl_cnat_encode_batched_work": (INT, [P, P, I64, P, I64, INT, P, U64, U64, P, I64, P, P, P, P]),
    "adfl_philox_uniforms": (INT, [P, I64, I64, U64, U64, P]),
    "adfl_stoch_norms_batched_dt": (INT, [I32, P, P, I64, INT, P, I64, P, P, P]),
    "adfl_stoch_quantize_batched_dt": (INT, [I32, I32, P, P, I64, INT, P, P, U64, U64, P, P, P]),
    "adfl_stoch_encode_batched_dt": (INT, [I32, I32, P, P, I64, INT, P, U64, U64, P, I64, P, P, P, P, P]),
    "adfl_philox_uniforms_dt": (INT, [I32, P, I64, I64, U64, U64, P]),
    # adfl_host.h
    "adfl_host_copy": (INT, [P, P, P, I64, I32]),
    "adfl_host_copy_ex": (INT, [P, P, P, I64, I32, I32]),
    "adfl_host_threads": (I32, []),
    "adfl_host_copy_submit": (I64, [P, P, P, I64, I32, I32, P, P]),
    "adfl_host_copy_wait": (INT, [I64]),
    "adfl_host_copy_done": (INT, [I64]),
    "adfl_host_bind": (INT, [P, I32]),
    "adfl_philox_rounds": (INT, []),
    "adfl_host_copy_submit_absmax": (I64, [P, P, P, I64, I32, I32, P, P, P]),
    "adfl_event_synchronize": (INT, [P]),
    "adfl_stage_events_create": (INT, [I32, P]),
    "adfl_stage_events_destroy": (INT, [P, I32]),
    "adfl_stage_d2h": (INT, [P, P, P, I32, P, P, P, P]),
    "adfl_stage_encode_range": (INT, [P, P, I64, I64, P, P, I64, I64, INT, P, P, P, I64, I64, P, P, P, P]),
    "adfl_stage_decode_range": (INT, [P, P, I64, I64, P, I64, I64, P, P, P, I64, I64, P, P, P, P]),
    "adfl_stage_stoch_decode_range": (INT, [I32, INT, P, P, P, P, I64, I64, P, I64, I64, P, P, P, P, I64, I64, P, P,
                                            P, P]),
}

NORM_L2, NORM_LINF, NORM_L2_TORCH = 0, 1, 2  # ADFL_NORM_*
CODEC_QSGD, CODEC_RQSGD, CODEC_CNAT = 0, 1, 2  # ADFL_CODEC_*
DTYPE_F32, DTYPE_F16, DTYPE_BF16, DTYPE_F64 = 0, 1, 2, 3  # ADFL_DTYPE_*

_lib = None


def load() -> ctypes.CDLL:
    """Load the in-tree HIP library once; raise loudly if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("ADFL_LIB_VARIANT") or LIB_PATH  # A/B builds of the same sources (tools/)
    if not os.path.exists(path):
        raise ImportError(f"adfl_amd: HIP codec library not found at {path}; "
                          "build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.adfl_slq_abi_version() != ABI_VERSION:
        raise ImportError(f"adfl_amd: ABI mismatch: library {lib.adfl_slq_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def check(status: int) -> None:
    if status != 0:
        raise AdflError(load().adfl_slq_strerror(status).decode())


def workspace_bytes() -> int:
    return int(load().adfl_slq_workspace_bytes())
