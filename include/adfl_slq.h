/*
 * adfl_slq.h — C ABI of the MI355X (gfx950) SLQ gradient codec: libadfl_slq.so.
 *
 * Drop-in boundary for ADFL's symmetric-linear-quantization channel. The reference codec is pure
 * Python over ATen CPU kernels; the entry points below are what its Channel plugin layer
 * (Src/ADFL/Channel/channel.py:10-45) binds through ctypes — see INTEGRATION.md. Each function names
 * the reference interface it replaces (file:line under the reference tree).
 *
 * Conventions
 *  - Every pointer named d_* is DEVICE memory (hipMalloc / torch CUDA allocator) on the current device.
 *    Pointers to fp32 / int8 element data must be 16-byte aligned (torch allocations are); element
 *    counts are int64 (a 4 GiB gradient overflows 32 bits).
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default stream). Every call is
 *    asynchronous on that stream, never synchronises, allocates nothing and is graph-capturable.
 *  - Return value: 0 on success; a positive hipError_t from a failed launch; a negative ADFL_E_* code
 *    for an argument error (nothing is launched then). adfl_slq_strerror() names either kind.
 *  - Bit-exact semantics (pinned by tests/golden): scale = fp32(absmax / (2^(bits-1)-1)), with absmax =
 *    max|x| (NaN propagates); inv = fp32(1/scale); q = NaN(x*inv) ? 127 : clamp(rne(fp32(x*inv)),
 *    -128, 127); dequantized value = fp32(scale * q).
 */
#ifndef ADFL_SLQ_H
#define ADFL_SLQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 5): adfl_stoch_norms_torch, adfl_stoch_torch_norm_scratch_bytes and adfl_stoch_torch_norm_walk_max
 * were replaced by adfl_torch_norms (adfl_stoch.h); the absmax / quantize kernels took new arguments. */
#define ADFL_SLQ_ABI_VERSION 2

enum {
  ADFL_OK = 0,
  ADFL_E_ARG = -1,       /* null pointer, negative count, bad tensor count */
  ADFL_E_BITS = -2,      /* bits outside [1, 16] */
  ADFL_E_ALIGN = -3,     /* a data pointer is not 16-byte aligned */
  ADFL_E_WORKSPACE = -4  /* workspace smaller than adfl_slq_workspace_bytes() */
};

/* Library / ABI identification. */
int adfl_slq_abi_version(void);
const char* adfl_slq_strerror(int status);

/* Bytes of device workspace the flat encode needs (per-block absmax partials). Constant. */
int64_t adfl_slq_workspace_bytes(void);

/* ---------------------------------------------------------------------------------------------
 * Flat (single tensor) codec — SLQChannel._quantize_tensor / _dequantize_tensor
 * (Src/ADFL/Channel/quant.py:97-104 and :107-112). n may be any value >= 1.
 * ------------------------------------------------------------------------------------------- */

/* Pass 1 of encode: max|x| partials into d_workspace (torch.max(torch.abs(t)), quant.py:100). */
int adfl_slq_absmax(const float* d_x, int64_t n, void* d_workspace, int64_t workspace_bytes, void* stream);

/* max|x| of pass 1 as one fp32 value into d_absmax[0] (torch.max(torch.abs(t)), quant.py:100; NaN
 * propagates): reduces the partials adfl_slq_absmax left in d_workspace, which stay valid for pass 2. */
int adfl_slq_absmax_value(const void* d_workspace, float* d_absmax, void* stream);

/* Pass 2 of encode: reduce the partials, scale = absmax/q_max (quant.py:99-100), write d_scale[0],
 * quantize x into d_q (torch.quantize_per_tensor(t, scale, 0, qint8), quant.py:102-103). */
int adfl_slq_quantize(const float* d_x, int64_t n, int bits, const void* d_workspace, int8_t* d_q,
                      float* d_scale, void* stream);

/* absmax + quantize (two launches): the whole of quant.py:97-104. */
int adfl_slq_encode(const float* d_x, int64_t n, int bits, int8_t* d_q, float* d_scale, void* d_workspace,
                    int64_t workspace_bytes, void* stream);

/* q.dequantize() (quant.py:110): d_out[i] = d_scale[0] * d_q[i]. */
int adfl_slq_dequantize(const int8_t* d_q, int64_t n, const float* d_scale, float* d_out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Bucketed (multi-tensor) codec — SLQChannel._quantize_params / _receive over a whole state dict
 * (quant.py:74-94, :67-71): one launch per pass for all tensors, per-tensor scales.
 *
 * Layout: tensor t owns elements [offset_t, offset_t + size_t) of the flat x / q / out buffers (the
 * base pointers 16-byte aligned). Offsets may be anything: tensors packed back to back (a compact
 * bucket, what the Channel uses) run their first elements up to a 16-element boundary element-wise;
 * offsets that are multiples of ADFL_SLQ_ALIGN_ELEMS never do. The work is described by a chunk table
 * built on the host by adfl_slq_build_chunks() and copied to the device once per layout.
 * ------------------------------------------------------------------------------------------- */
#define ADFL_SLQ_ALIGN_ELEMS 64
#define ADFL_SLQ_CHUNK_ELEMS 8192

typedef struct adfl_slq_chunk {
  int64_t start;        /* first element of the chunk in the flat buffer */
  int32_t len;          /* elements in the chunk, 1..ADFL_SLQ_CHUNK_ELEMS */
  int32_t tensor;       /* owning tensor index */
  int32_t first_chunk;  /* index of the owning tensor's first chunk */
  int32_t nchunks;      /* number of chunks of the owning tensor */
} adfl_slq_chunk;

/* Host-side: number of chunks for the given sizes (call with chunks == NULL), or fill `chunks`.
 * Returns the chunk count, or a negative ADFL_E_* code. */
int64_t adfl_slq_build_chunks(const int64_t* offsets, const int64_t* sizes, int32_t ntensors,
                              adfl_slq_chunk* chunks, int64_t capacity);

/* d_partials: int64 nchunks * 4 bytes of device scratch. d_scales: ntensors floats.
 * Two launches: per-chunk absmax partials, then per-chunk quantize (x read twice). */
int adfl_slq_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                            int8_t* d_q, float* d_scales, uint32_t* d_partials, void* stream);

/* One-launch encode (same output) for a bucket whose tensors ALL have at most ADFL_SLQ_RESIDENT_CHUNKS
 * chunks (<= 65,536 elements): one block holds a whole tensor in registers, so x is read once and there is
 * no second pass. Host-side: adfl_slq_build_encode_work() writes the first chunk of every tensor to `work`
 * and returns the count; it returns 0 if some tensor is larger (call with work == NULL to size). The list
 * is copied to the device once per layout, like the chunk table. adfl_slq_encode_batched_work() with
 * nwork == 0 is adfl_slq_encode_batched (the two-pass encode), so a caller can always go through it.
 * d_partials is used only by the two-pass encode. A work list entry naming a tensor with more than
 * ADFL_SLQ_RESIDENT_CHUNKS chunks (not one adfl_slq_build_encode_work made) gets a NaN scale and no payload. */
#define ADFL_SLQ_RESIDENT_CHUNKS 8
int64_t adfl_slq_build_encode_work(const adfl_slq_chunk* chunks, int64_t nchunks, int32_t* work, int64_t capacity);
int adfl_slq_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                 const int32_t* d_work, int64_t nwork, int bits, int8_t* d_q, float* d_scales,
                                 uint32_t* d_partials, void* stream);
int adfl_slq_dequantize_batched(const int8_t* d_q, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                const float* d_scales, float* d_out, void* stream);
/* The quantize pass of adfl_slq_encode_batched over chunks [chunk_begin, chunk_begin + count) of the FULL
 * chunk table d_chunks, from absmax partials the caller supplies: d_partials[c] for every chunk c of the
 * tensors involved, the per-chunk max|x| bits or the whole tensor's at its first chunk and 0 at the others
 * (the scale is fp32(max / (2^(bits-1)-1)) of their max, written by each tensor's first chunk). A host that
 * reduced every tensor's max|x| while staging it (SLQChannel's fused gather, quant.py:100) quantizes the
 * tensors one staging range completes while the next range is still being copied; same payload and scales
 * as adfl_slq_encode_batched. A dequantize of a chunk range is adfl_slq_dequantize_batched on d_chunks +
 * chunk_begin. */
int adfl_slq_quantize_batched_range(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t chunk_begin,
                                    int64_t count, int bits, const uint32_t* d_partials, int8_t* d_q,
                                    float* d_scales, void* stream);
/* The absmax pass of adfl_slq_encode_batched over chunks [chunk_begin, chunk_begin + count) of the FULL chunk
 * table: d_partials[c] = the max|x| bits of chunk c (torch.max(torch.abs(t)), quant.py:100, NaN winning) for
 * every c in the range, the partials adfl_slq_quantize_batched_range then reduces per tensor. */
int adfl_slq_absmax_batched_range(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t chunk_begin, int64_t count,
                                  uint32_t* d_partials, void* stream);

/* Quantization error of a bucket against its own payload without materialising the decode — the
 * metrics Src/ADFL/Client/worker.py:186-189 computes with parameter_relative_mse /
 * parameter_cosine_similarity (Src/ADFL/model.py:256-323). Per chunk, 4 fp64 sums into
 * d_partials[4*c .. 4*c+3]: sum (x-d)^2, sum x^2, sum x*d, sum d^2 with d = fp32(scale*q). */
int adfl_slq_qerror_batched(const float* d_x, const int8_t* d_q, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                            const float* d_scales, double* d_partials, void* stream);
/* Same against an int4-packed bucket (adfl_slq_encode_batched_int4's payload: even tensor offsets,
 * d = fp32(scale * (nibble - 8)), the value unpack_4bit + dequantize gives, compression.py:51-66). */
int adfl_slq_qerror_batched_int4(const float* d_x, const uint8_t* d_packed, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, const float* d_scales, double* d_partials, void* stream);

/* ---------------------------------------------------------------------------------------------
 * int4 packed variant — compression.py pack_4bit / unpack_4bit (Src/ADFL/compression.py:35-66)
 * fused with SLQ quantize / dequantize. Packed bytes = ceil(n/2); byte j = ((q[2j]+8)<<4) | (q[2j+1]+8)
 * in int8 wraparound arithmetic (high nibble = even element), a zero element padding odd n.
 * ------------------------------------------------------------------------------------------- */
int adfl_slq_quantize_int4(const float* d_x, int64_t n, int bits, const void* d_workspace, uint8_t* d_packed,
                           float* d_scale, void* stream);
int adfl_slq_encode_int4(const float* d_x, int64_t n, int bits, uint8_t* d_packed, float* d_scale,
                         void* d_workspace, int64_t workspace_bytes, void* stream);
int adfl_slq_dequantize_int4(const uint8_t* d_packed, int64_t n, const float* d_scale, float* d_out,
                             void* stream);
/* Bucketed int4 (PackedSLQChannel): every tensor offset in the chunk table must be EVEN; flat element e
 * then lives in packed byte e/2, so d_packed holds (total elements)/2 bytes, and an odd-sized tensor's
 * last byte pairs its last element with a zero pad exactly as pack_4bit does per tensor. */
int adfl_slq_encode_batched_int4(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                                 uint8_t* d_packed, float* d_scales, uint32_t* d_partials, void* stream);
/* One-launch int4 encode for a bucket whose tensors all fit a block (work list of
 * adfl_slq_build_encode_work; nwork == 0 is adfl_slq_encode_batched_int4). Same output. */
int adfl_slq_encode_batched_int4_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                      const int32_t* d_work, int64_t nwork, int bits, uint8_t* d_packed,
                                      float* d_scales, uint32_t* d_partials, void* stream);
int adfl_slq_dequantize_batched_int4(const uint8_t* d_packed, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                     const float* d_scales, float* d_out, void* stream);
int adfl_pack_int4(const int8_t* d_q, int64_t n, uint8_t* d_packed, void* stream);
int adfl_unpack_int4(const uint8_t* d_packed, int64_t n, int8_t* d_q, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Peer exchange epilogue — the mean over K gathered payloads that follows the all-gather
 * (Examples/ray_ad.py:188 `torch.stack(updates).mean(0)`, Src/ADFL/model.py:221-234 simple_aggregate):
 * d_out[i] = (sum_r d_scales[r] * q_r[i]) / K, summed in r order, fp32. The K payloads are rows of one
 * buffer: q_r = d_q + r * row_stride_bytes.
 * ------------------------------------------------------------------------------------------- */
int adfl_slq_dequantize_mean(const int8_t* d_q, int64_t row_stride_bytes, int32_t k, int64_t n,
                             const float* d_scales, int64_t scale_stride, float* d_out, void* stream);
/* Same over K int4-packed rows (ceil(n/2) bytes of payload each, layout of adfl_slq_quantize_int4). */
int adfl_slq_dequantize_mean_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k, int64_t n,
                                  const float* d_scales, int64_t scale_stride, float* d_out, void* stream);
/* The receiving peer's mean with its OWN update exact, as the reference forms it
 * (Src/ADFL/Client/async_peer.py:170-174, Examples/ray_ad.py:183-188: the local fp32 parameters are
 * appended after the received updates, then stack(...).mean(0)): row self_row is skipped, the other rows
 * are summed in r order, d_self_x (n fp32, 16-byte aligned) is added last, then / K.
 * self_row = -1 is adfl_slq_dequantize_mean. */
int adfl_slq_dequantize_mean_self(const int8_t* d_q, int64_t row_stride_bytes, int32_t k, int64_t n,
                                  const float* d_scales, int64_t scale_stride, int32_t self_row,
                                  const float* d_self_x, float* d_out, void* stream);
int adfl_slq_dequantize_mean_self_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k, int64_t n,
                                       const float* d_scales, int64_t scale_stride, int32_t self_row,
                                       const float* d_self_x, float* d_out, void* stream);

/* The same mean over K BUCKETED payloads with per-tensor scales: the decentralized exchange of a whole
 * state dict under SLQChannel's per-tensor codec (Examples/ray_ad.py:164-190 averages every tensor;
 * Src/ADFL/Channel/quant.py:74-94 gives each its own scale). Row r: payload d_q + r * row_stride_bytes in the
 * layout of d_chunks (an adfl_slq_encode_batched* payload), scales d_scales + r * scale_stride (one fp32 per
 * tensor). For tensor t, element i: (sum over r != self_row in r order of fp32(scale_r[t] * q_r[i]), then
 * + d_self_x[i] if self_row >= 0) / k, fp32 adds, correctly rounded division — adfl_slq_dequantize_mean_self
 * per tensor. d_out and d_self_x are flat buckets in the same layout; positions outside every tensor are
 * not written. row_stride_bytes: a multiple of 16, at least the bucket's extent. */
int adfl_slq_dequantize_mean_batched(const int8_t* d_q, int64_t row_stride_bytes, int32_t k,
                                     const adfl_slq_chunk* d_chunks, int64_t nchunks, const float* d_scales,
                                     int64_t scale_stride, int32_t self_row, const float* d_self_x, float* d_out,
                                     void* stream);
/* Same over K int4-packed bucket payloads (adfl_slq_encode_batched_int4's: every tensor offset in d_chunks
 * EVEN, flat element e in byte e/2 of the row, high nibble for even e): PackedSLQChannel per tensor
 * (Src/ADFL/compression.py:35-66 over quant.py:74-94). row_stride_bytes: a multiple of 16, at least
 * ceil(extent / 2). */
int adfl_slq_dequantize_mean_batched_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k,
                                          const adfl_slq_chunk* d_chunks, int64_t nchunks, const float* d_scales,
                                          int64_t scale_stride, int32_t self_row, const float* d_self_x,
                                          float* d_out, void* stream);

/* Fused decode + in-place accumulate into K models: for every model k and tensor t,
 *   model_k[t][i] = fp32(model_k[t][i] + fp32(scale_t * q[i]))
 * which is the receiver's on_client_receive followed by add_parameters_inpace(model, decoded, 1, 1)
 * (Src/ADFL/model.py:337-347) for each model: the client pool's add_to_model / add_to_model_all
 * (Src/ADFL/Client/pool.py:62-75) and QAFeL's hidden-state update (Src/ADFL/Server/qafel.py:176-179).
 * The payload is read once for all K models; each model is read and written once.
 *   d_q, d_chunks  a bucketed payload, any tensor offsets (offsets that are multiples of 4 elements, e.g. an
 *                  ADFL_SLQ_ALIGN_ELEMS-aligned bucket, take 16-byte accesses; others, e.g. a compact
 *                  bucket, are decoded element-wise with the same result); d_scales one fp32 per tensor
 *   d_targets      DEVICE array of ntargets * ntensors device pointers, d_targets[k * ntensors + t] = the
 *                  fp32 storage of tensor t of model k (contiguous, 16-byte aligned, sizes as the table) */
int adfl_slq_dequantize_add_batched(const int8_t* d_q, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                    const float* d_scales, float* const* d_targets, int32_t ntensors,
                                    int32_t ntargets, void* stream);

/* Device staging of a state dict as one bucket (the gather / scatter around every bucketed entry above when
 * the dict's tensors live on the device; the reference's per-tensor loop, quant.py:67-94, has one tensor per
 * op): every tensor's elements copied between its own storage and its slot of the bucket, one launch for the
 * whole dict. d_srcs / d_dsts[t] (a device array of nt pointers) is tensor t's first element, contiguous,
 * elem_bytes (1, 2, 4 or 8) per element; the bucket holds tensor t at its chunks' offsets (elements).
 * Bytes outside every chunk (an aligned bucket's pads) are neither read nor written. Any alignment. */
int adfl_bucket_gather(void* d_bucket, const adfl_slq_chunk* d_chunks, int64_t nchunks, const void* const* d_srcs,
                       int32_t elem_bytes, void* stream);
int adfl_bucket_scatter(const void* d_bucket, const adfl_slq_chunk* d_chunks, int64_t nchunks, void* const* d_dsts,
                        int32_t elem_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ADFL_SLQ_H */
