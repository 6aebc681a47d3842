/*
 * adfl_stoch.h — C ABI of the MI355X (gfx950) stochastic gradient codecs in libadfl_slq.so:
 * QSGD / RQSGD / CNAT (Src/ADFL/Channel/quant.py:140-570).
 *
 * Same conventions as adfl_slq.h (device pointers d_*, 16-byte aligned bases, int64 counts, void*
 * hipStream_t, asynchronous, no allocation, graph-capturable, 0 / hipError_t / ADFL_E_* returns) and the
 * same bucket description: an adfl_slq_chunk table from adfl_slq_build_chunks() over a flat buffer in
 * which tensor t owns elements [offset_t, offset_t + size_t). A single tensor is a one-entry table.
 *
 * Payload planes (what the reference's QuantParameter holds, quant.py:209-217,349-358,495-503):
 *   levels  uint8, one per element — QSGD/RQSGD quantization level l in [0, 2^bits - 1], or CNAT's
 *           int8 exponent in [-2^(bits-1), 2^(bits-1) - 1] (stored as its byte)
 *   signs   int8, one per element — torch.sign(x) in {-1, 0, 1} (NaN -> 0)
 *   norms   fp32, one per tensor — QSGD/CNAT: ||x||_2; RQSGD: max|x| (+ mins = min|x|)
 * Both planes are indexed like x (byte g of a plane belongs to element g of the bucket).
 *
 * Uniforms. Stochastic rounding compares u in [0, 1) with a per-element probability. d_uniforms == NULL
 * draws u from the counter-based Philox4x32-7 stream keyed by `seed`: element g of the bucket uses word
 * g % 4 of block (counter + g / 4), u = (word >> 8) * 2^-24. A caller that advances `counter` by
 * ceil(total / 4) per call never reuses a uniform. d_uniforms != NULL injects one fp32 uniform per
 * element (indexed like x) — with the reference's own uniforms the outputs are bit-identical to it.
 *
 * Norm: fp32 squares accumulated in fp64 per chunk and per tensor (fixed order: deterministic), rounded
 * once to fp32, correctly rounded sqrt. torch's fp32 vector_norm differs from it only by torch's own
 * accumulation error; every other output bit follows the reference exactly. For bit parity
 * with the reference's norm, compute it with ADFL_NORM_L2_TORCH and quantize with the given-norm entry.
 */
#ifndef ADFL_STOCH_H
#define ADFL_STOCH_H

#include <stdint.h>

#include "adfl_slq.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { ADFL_NORM_L2 = 0, ADFL_NORM_LINF = 1, ADFL_NORM_L2_TORCH = 2 };
enum { ADFL_CODEC_QSGD = 0, ADFL_CODEC_RQSGD = 1, ADFL_CODEC_CNAT = 2 };
enum { ADFL_DTYPE_F32 = 0, ADFL_DTYPE_F16 = 1, ADFL_DTYPE_BF16 = 2, ADFL_DTYPE_F64 = 3 };

/* Device workspace bytes the encode / norm calls need for a table of nchunks chunks (16 B per chunk). */
int64_t adfl_stoch_workspace_bytes(int64_t nchunks);

/* Per-tensor norms of a bucket (two launches: chunk partials, per-tensor finalize).
 *   ADFL_NORM_L2:   d_norms[t] = ||x_t||_2   (torch.linalg.vector_norm(x, ord=2), quant.py:226,512)
 *   ADFL_NORM_LINF: d_norms[t] = max|x_t|, d_mins[t] = min|x_t| (ord=inf / -inf, quant.py:367,380);
 *                   NaN anywhere in x_t makes both NaN. d_mins may be NULL for ADFL_NORM_L2.
 *   ADFL_NORM_L2_TORCH: ||x_t||_2 bit-identical to torch 2.10's CPU vector_norm (its fp32 reduction order:
 *                   8 FMA lane accumulators, lane sum, then the n % 8 tail: 4 rounded squares, then FMA),
 *                   i.e. the reference's own norm. One launch, no workspace (d_workspace may be NULL), but
 *                   sequential per tensor: about one element per cycle per tensor. */
int adfl_stoch_norms_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int mode,
                             void* d_workspace, int64_t workspace_bytes, float* d_norms, float* d_mins,
                             void* stream);

enum { ADFL_TORCH_NORM_SHORT = 1, ADFL_TORCH_NORM_LONG = 2 };

/* torch 2.10's CPU vector_norm(x, ord=2) — the reference's QSGD / CNAT norm (quant.py:226,512) — bit for bit
 * for fp32, bf16, fp16 and fp64 buckets (dtype ADFL_DTYPE_*: d_x holds elements of that type, indexed by the
 * chunk table), in phases with no cross-block waits (csrc/torch_norm.hip): per-tile fp64 sums, a per-chain
 * prefix that predicts each tile's binade, per-tile exact integer maps under the predicted binades, and one
 * block per tensor composing them, running the reference's fma only where an accumulator leaves its binade.
 * Orders restated: oracle/slq_oracle.c
 * oracle_torch_l2_norm{,_bf16,_f16,_f64}.
 *   threads: torch.get_num_threads() of the process whose norm is reproduced (fp16 tensors of >= 32768
 *            elements are summed in min(threads, ceil(n / 32768)) contiguous pieces: 1..512 for fp16 buckets;
 *            any value >= 1 for the other dtypes, which do not use it).
 *   kinds:   which tensors the bucket holds, so launches with nothing to do are skipped:
 *            ADFL_TORCH_NORM_SHORT (some of at most adfl_torch_norm_short_max_dt(dtype) elements: fp32, bf16
 *            and fp16 ones in one launch, one block per tensor) | ADFL_TORCH_NORM_LONG (some longer: the phased
 *            path); 0 = both.
 *   outputs: d_norms64[t] = the norm as a double (the dtype's value: exact for every dtype) and / or
 *            d_norms32[t] = (float) of it; either may be NULL, not both.
 * d_scratch: adfl_torch_norm_scratch_bytes(nchunks, ntensors) bytes, 256-byte aligned, no initialisation.
 * Up to nine launches, stream-ordered with no host waits (one for layouts of short fp32 / bf16 / fp16 tensors
 * only). */
int64_t adfl_torch_norm_scratch_bytes(int64_t nchunks, int64_t ntensors);
int64_t adfl_torch_norm_short_max(void);          /* fp16 / fp64: 65,536 */
int64_t adfl_torch_norm_short_max_dt(int32_t dtype); /* the short-tensor bound of a dtype (fp32, bf16: 2^19; fp16,
                                                        fp64: 2^16), or ADFL_E_ARG */
int adfl_torch_norms(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                     int64_t ntensors, int32_t kinds, int32_t threads, void* d_scratch, int64_t scratch_bytes,
                     double* d_norms64, float* d_norms32, void* stream);
/* The same with the caller's list of every tensor's first chunk (d_tfirst[t], ntensors int32 on the device; the
 * host has it from building the chunk table), which saves the launch that builds it; NULL: adfl_torch_norms. */
int adfl_torch_norms_work(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                          const int32_t* d_tfirst, int64_t ntensors, int32_t kinds, int32_t threads, void* d_scratch,
                          int64_t scratch_bytes, double* d_norms64, float* d_norms32, void* stream);

/* QSGD / RQSGD level quantization given per-tensor norms (quant.py:230-238 and :371-379), levels =
 * 2^bits - 1: scaled = fl(fl(levels*|x|) / norm); l = floor(scaled); q = u8(l + (u < scaled - l));
 * norm == 0 gives levels 0 and signs 1 (quant.py:227-228). One launch. */
int adfl_qsgd_quantize_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                               const float* d_norms, const float* d_uniforms, uint64_t seed, uint64_t counter,
                               uint8_t* d_levels, int8_t* d_signs, void* stream);

/* QSGDChannel._quantize_tensor over a bucket (quant.py:223-240): L2 norms + quantize (three launches). */
int adfl_qsgd_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                             const float* d_uniforms, uint64_t seed, uint64_t counter, void* d_workspace,
                             int64_t workspace_bytes, uint8_t* d_levels, int8_t* d_signs, float* d_norms,
                             void* stream);

/* RQSGDChannel._quantize_tensor (quant.py:364-382): max|x| norms, min|x| factors + quantize. */
int adfl_rqsgd_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                              const float* d_uniforms, uint64_t seed, uint64_t counter, void* d_workspace,
                              int64_t workspace_bytes, uint8_t* d_levels, int8_t* d_signs, float* d_norms,
                              float* d_mins, void* stream);

/* QSGDChannel._dequantize_tensor (quant.py:243-252): out = fl(fl(norm*l) / levels) * sign; 0 if norm == 0. */
int adfl_qsgd_dequantize_batched(const uint8_t* d_levels, const int8_t* d_signs, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, int bits, const float* d_norms, float* d_out, void* stream);

/* RQSGDChannel._dequantize_tensor (quant.py:385-398): out = fl(fl(norm*sign)*l) / levels, and
 * min*sign where l == 0; 0 if norm == 0. */
int adfl_rqsgd_dequantize_batched(const uint8_t* d_levels, const int8_t* d_signs, const adfl_slq_chunk* d_chunks,
                                  int64_t nchunks, int bits, const float* d_norms, const float* d_mins,
                                  float* d_out, void* stream);

/* CNATChannel._quantize_tensor (quant.py:509-534) in one pass over x (exponents, signs and the L2 norm
 * partials together), then a per-tensor finalize and the norm == 0 rewrite (levels 0, signs 1,
 * quant.py:513-514): three launches, x read once. d_exps holds each exponent's int8 byte. */
int adfl_cnat_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                             const float* d_uniforms, uint64_t seed, uint64_t counter, void* d_workspace,
                             int64_t workspace_bytes, int8_t* d_exps, int8_t* d_signs, float* d_norms,
                             void* stream);

/* CNATChannel._dequantize_tensor (quant.py:537-545): out = fl(fl(norm*sign) * 2^e); 0 if norm == 0. */
int adfl_cnat_dequantize_batched(const int8_t* d_exps, const int8_t* d_signs, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, const float* d_norms, float* d_out, void* stream);

/* simple_aggregate (Src/ADFL/model.py:221-234) of K clients' decodes, one launch: out[i] =
 * fp32(((0 + d_0[i]) + ... + d_{K-1}[i]) / K), d_r the codec's decode (above) of row r's level / exponent
 * and sign bytes (d_levels / d_signs + r * row_stride_bytes, each a bucket payload over d_chunks) under row
 * r's norms d_norms + r * norm_stride (RQSGD: d_mins likewise; +0 where a norm is 0). codec: ADFL_CODEC_*
 * (bits unused for CNAT). Bases 16-byte aligned, row_stride_bytes a multiple of 16. Bit-identical to torch's
 * CPU sum for K <= 4 (it adds rows in order from zero); from K = 5 torch regroups, within fp32 summation
 * error. */
int adfl_stoch_dequantize_mean_batched(int32_t codec, const uint8_t* d_levels, const int8_t* d_signs,
                                       int64_t row_stride_bytes, int32_t k, const adfl_slq_chunk* d_chunks,
                                       int64_t nchunks, int bits, const float* d_norms, const float* d_mins,
                                       int64_t norm_stride, float* d_out, void* stream);

/* One-launch encodes (same outputs, bit for bit) for a bucket whose tensors ALL have at most
 * ADFL_SLQ_RESIDENT_CHUNKS chunks: d_work / nwork is the work list of adfl_slq_build_encode_work (the first
 * chunk of every tensor; nwork == 0 when some tensor is larger). A 1024-thread block holds one whole tensor
 * in registers, reduces its norm and quantizes it: x read once, no workspace, no fix-up launch. With
 * nwork == 0 these run the multi-launch encodes above (which need the workspace). A work list entry naming a
 * tensor with more than ADFL_SLQ_RESIDENT_CHUNKS chunks gets a NaN norm and no payload. */
int adfl_qsgd_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                  const int32_t* d_work, int64_t nwork, int bits, const float* d_uniforms,
                                  uint64_t seed, uint64_t counter, void* d_workspace, int64_t workspace_bytes,
                                  uint8_t* d_levels, int8_t* d_signs, float* d_norms, void* stream);
int adfl_rqsgd_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                   const int32_t* d_work, int64_t nwork, int bits, const float* d_uniforms,
                                   uint64_t seed, uint64_t counter, void* d_workspace, int64_t workspace_bytes,
                                   uint8_t* d_levels, int8_t* d_signs, float* d_norms, float* d_mins, void* stream);
int adfl_cnat_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                  const int32_t* d_work, int64_t nwork, int bits, const float* d_uniforms,
                                  uint64_t seed, uint64_t counter, void* d_workspace, int64_t workspace_bytes,
                                  int8_t* d_exps, int8_t* d_signs, float* d_norms, void* stream);

/* The Philox uniforms the codecs draw: d_out[i] = u(start + i) of stream (seed, counter), i < n.
 * (Exposed for tests and for callers that want the uniforms a call used.) */
int adfl_philox_uniforms(float* d_out, int64_t n, int64_t start, uint64_t seed, uint64_t counter, void* stream);

/* The Philox4x32 round count this library was built with: 7 (the product) or 10 (an ADFL_PHILOX_ROUNDS=10
 * build; csrc/philox.h records why 7). */
int adfl_philox_rounds(void);

/* ---- fp16 / bf16 / fp64 tensors -------------------------------------------------------------------
 * The reference computes QSGD / RQSGD / CNAT in the tensor's own dtype (quant.py:223-240, :364-382,
 * :509-534): each op on fp16 / bf16 computes in fp32 and rounds to the dtype; fp64 ops are fp64. These
 * entries do the same on a bucket of one dtype (d_x: uint16 bit patterns for fp16 / bf16, doubles for fp64;
 * 16-byte aligned bases, the level / sign planes too). Uniforms are on torch.rand's grid for the dtype:
 * d_uniforms (NULL or a plane of the dtype indexed like x) or the Philox4x32-7 stream — fp16 / bf16:
 * element g takes word g % 4 of block
 * (counter + g / 4), u = (word >> 21) * 2^-11 (fp16) or (word >> 24) * 2^-8 (bf16); fp64: element g takes
 * words 2 (g % 2), 2 (g % 2) + 1 of block (counter + g / 2) as the high / low halves of 64 bits,
 * u = (bits >> 11) * 2^-53 (advance counter by ceil(total / 4), fp64 ceil(total / 2), per call).
 * Norms are fp64 values of the dtype's norm: fp16 / bf16 L2 = R(sqrt(fp32(sum of fp32 squares in fp64)));
 * fp64 L2 = sqrt(fp64 sum); LINF = max|x| / min|x|. CNAT's floor / ceil(log2) is the exact band rule of
 * cnat_log2_dt_table.h. Decode with the fp32 dequantize entries and fp32(norm) (the reference decodes to
 * fp32 with the Python-float norm as an fp32 scalar). Workspace: adfl_stoch_workspace_bytes(nchunks). */
int adfl_stoch_norms_batched_dt(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                int mode, void* d_workspace, int64_t workspace_bytes, double* d_norms, double* d_mins,
                                void* stream);
/* Levels (QSGD / RQSGD: codec's norm in d_norms) or CNAT exponents + signs; norm == 0 gives 0 / 1. */
int adfl_stoch_quantize_batched_dt(int32_t codec, int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks,
                                   int64_t nchunks, int bits, const double* d_norms, const void* d_uniforms,
                                   uint64_t seed, uint64_t counter, uint8_t* d_levels, int8_t* d_signs, void* stream);
/* norms (L2; RQSGD: LINF with d_mins) + quantize. CNAT reads x once (its exponents do not depend on the norm:
 * exponents, signs and chunk partials in one pass, then the norms and the norm == 0 fill). */
int adfl_stoch_encode_batched_dt(int32_t codec, int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, int bits, const void* d_uniforms, uint64_t seed, uint64_t counter,
                                 void* d_workspace, int64_t workspace_bytes, uint8_t* d_levels, int8_t* d_signs,
                                 double* d_norms, double* d_mins, void* stream);
/* The uniforms elements start .. start+n-1 draw from stream (seed, counter) in the dtype (tests). */
int adfl_philox_uniforms_dt(int32_t dtype, void* d_out, int64_t n, int64_t start, uint64_t seed, uint64_t counter,
                            void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ADFL_STOCH_H */
