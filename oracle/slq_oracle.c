/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement of ADFL's SLQ gradient codec.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
 * as the checker. The product path (ad-federatedlearning_amd/) never links or calls it.
 *
 * Parity pin: checked against tests/golden/ (vectors produced by executing the reference's
 * Src/ADFL/Channel/quant.py in place on torch 2.10.0+rocm7.0, quantized engine x86; generator
 * tests/golden/make_golden.py). The arithmetic itself lives in third-party ATen/fbgemm kernels
 * (torch 2.10.0, requirements.txt:1 pins no version): torch.max/abs, quantize_per_tensor and
 * Tensor.dequantize, called at Src/ADFL/Channel/quant.py:100-103,110. This file restates what those
 * calls compute, as established empirically against that torch build.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math: SSE scalar fp32 is IEEE).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* torch.max(torch.abs(t)) — Src/ADFL/Channel/quant.py:100. NaN propagates (torch.max semantics). */
float oracle_slq_absmax(const float* x, int64_t n) {
    float m = 0.0f;
    for (int64_t i = 0; i < n; ++i) {
        float a = fabsf(x[i]);
        if (isnan(a)) return a;
        if (a > m) m = a;
    }
    return m;
}

/* q_max = 2**(bits-1)-1; scale = fp32(absmax / q_max) — quant.py:99-100 (fp32 tensor / int). */
float oracle_slq_scale(float absmax, int bits) {
    int qmax = (1 << (bits - 1)) - 1;
    return absmax / (float)qmax;
}

/* torch.quantize_per_tensor(t, scale, 0, qint8) — quant.py:102-103.
 * Elementwise: inv = fp32(1/scale); y = fp32(x*inv); NaN -> 127; clamp to [-128,127];
 * round half to even. (Multiply-by-reciprocal, not divide: SURVEY.md §7 "Hard parts".) */
void oracle_slq_quantize(const float* x, int64_t n, float scale, int8_t* q) {
    float inv = 1.0f / scale;
    for (int64_t i = 0; i < n; ++i) {
        float y = x[i] * inv;
        if (isnan(y)) { q[i] = 127; continue; }
        if (y > 127.0f) y = 127.0f;
        if (y < -128.0f) y = -128.0f;
        q[i] = (int8_t)nearbyintf(y); /* default FE_TONEAREST = ties to even */
    }
}

/* SLQChannel._quantize_tensor (quant.py:97-104): returns the fp32 scale, writes the int8 payload. */
float oracle_slq_encode(const float* x, int64_t n, int bits, int8_t* q) {
    float scale = oracle_slq_scale(oracle_slq_absmax(x, n), bits);
    oracle_slq_quantize(x, n, scale, q);
    return scale;
}

/* q.dequantize() — quant.py:110: fp32(scale * float(q)), zero point 0. */
void oracle_slq_dequantize(const int8_t* q, int64_t n, float scale, float* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = scale * (float)q[i];
}

/* Multi-tensor form of SLQChannel._quantize_params (quant.py:74-94) over a flat buffer: tensor t owns
 * elements [offsets[t], offsets[t] + sizes[t]) of x and of q. */
void oracle_slq_encode_batched(const float* x, const int64_t* offsets, const int64_t* sizes, int32_t ntensors,
                               int bits, int8_t* q, float* scales) {
    for (int32_t t = 0; t < ntensors; ++t)
        scales[t] = oracle_slq_encode(x + offsets[t], sizes[t], bits, q + offsets[t]);
}

void oracle_slq_dequantize_batched(const int8_t* q, const int64_t* offsets, const int64_t* sizes, int32_t ntensors,
                                   const float* scales, float* out) {
    for (int32_t t = 0; t < ntensors; ++t)
        oracle_slq_dequantize(q + offsets[t], sizes[t], scales[t], out + offsets[t]);
}

/* pack_4bit — Src/ADFL/compression.py:35-48. Flatten; pad one 0 if odd; q+8 in int8 arithmetic
 * (wraps); byte = (hi << 4) | lo with hi = even element, lo = odd element, int8 wraparound, the low
 * operand NOT masked to a nibble (out-of-range values alias, e.g. 127 packs as nibbles (7,-1)). */
int64_t oracle_pack_int4(const int8_t* q, int64_t n, uint8_t* packed) {
    int64_t np = (n + 1) / 2;
    for (int64_t j = 0; j < np; ++j) {
        int64_t i0 = 2 * j, i1 = 2 * j + 1;
        uint8_t hi = (uint8_t)(q[i0] + 8);
        uint8_t lo = (uint8_t)((i1 < n ? q[i1] : 0) + 8);
        packed[j] = (uint8_t)((uint8_t)(hi << 4) | lo);
    }
    return np;
}

/* unpack_4bit — Src/ADFL/compression.py:51-66: high = ((b>>4)&0xF)-8, low = (b&0xF)-8, truncated to n. */
void oracle_unpack_int4(const uint8_t* packed, int64_t n, int8_t* q) {
    for (int64_t i = 0; i < n; ++i) {
        uint8_t b = packed[i / 2];
        q[i] = (int8_t)((i & 1) ? ((b & 0xF) - 8) : (((b >> 4) & 0xF) - 8));
    }
}

/* int4 end-to-end as the composition the reference's functions define: dequantize(unpack(pack(q))). */
void oracle_slq_dequantize_int4(const uint8_t* packed, int64_t n, float scale, float* out) {
    for (int64_t i = 0; i < n; ++i) {
        uint8_t b = packed[i / 2];
        int v = (i & 1) ? ((b & 0xF) - 8) : (((b >> 4) & 0xF) - 8);
        out[i] = scale * (float)v;
    }
}

/* torch 2.10's CPU summation order of torch.sum(torch.stack(rows), dim=0) — simple_aggregate
 * (Src/ADFL/model.py:229-231) and stack(...).mean(0) (Examples/ray_ad.py:188; CPU mean = that sum / K) —
 * restated from aten/src/ATen/native/cpu/SumKernel.cpp (cascade_sum, the AVX2 kernel: 8-float vectors) and
 * pinned against torch itself and the reference's simple_aggregate executed in place
 * (tests/golden/aggregate.npz, tests/test_sum_order_golden.py). d[s * stride] is row s's value of one
 * element; j is the element's index in its n-element tensor.
 *   SEQ   j < (n >= 8 ? n & ~31 : n & ~3): rows in order into a 4-level cascade (fold every 16 rows);
 *   ILP4  other columns, and n == 1 with K < 8: 4 interleaved partials (rows 4g+p), leftover rows into
 *         partial 0, then p0 + p1 + p2 + p3;
 *   INNER n == 1 with K >= 8: vectorized_inner_sum (8 lanes, each an ILP4 sum over its vectors). */
static float cascade_f(const float* d, int64_t count, int64_t stride) {
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    for (int64_t i = 0; i < count;) {
        a0 = a0 + d[i * stride];
        ++i;
        if ((i & 15) == 0) {
            a1 = a1 + a0; a0 = 0.0f;
            if ((i & 0xF0) == 0) {
                a2 = a2 + a1; a1 = 0.0f;
                if ((i & 0xF00) == 0) { a3 = a3 + a2; a2 = 0.0f; }
            }
        }
    }
    a0 = a0 + a1;
    a0 = a0 + a2;
    return a0 + a3;
}

static float ilp4_f(const float* d, int64_t count, int64_t stride) {
    const int64_t g = count / 4;
    float p0 = cascade_f(d, g, 4 * stride);
    const float p1 = cascade_f(d + stride, g, 4 * stride);
    const float p2 = cascade_f(d + 2 * stride, g, 4 * stride);
    const float p3 = cascade_f(d + 3 * stride, g, 4 * stride);
    for (int64_t i = 4 * g; i < count; ++i) p0 = p0 + d[i * stride];
    p0 = p0 + p1;
    p0 = p0 + p2;
    return p0 + p3;
}

float oracle_torch_sum_col(const float* d, int32_t k, int64_t j, int64_t n) {
    if (n == 1) {
        if (k < 8) return ilp4_f(d, k, 1);
        const int64_t v = k / 8;
        float acc = 0.0f;
        for (int64_t i = 8 * v; i < k; ++i) acc = acc + d[i];
        for (int l = 0; l < 8; ++l) acc = acc + ilp4_f(d + l, v, 8);
        return acc;
    }
    const int64_t seq_end = n >= 8 ? (n & ~(int64_t)31) : (n & ~(int64_t)3);
    return j < seq_end ? cascade_f(d, k, 1) : ilp4_f(d, k, 1);
}

/* torch.stack(rows).sum(0) / K for a row-major [k, n] fp32 matrix (one tensor per row). */
void oracle_torch_mean_rows(const float* rows, int32_t k, int64_t n, float* out) {
    float* col = (float*)malloc(sizeof(float) * (size_t)k);
    for (int64_t i = 0; i < n; ++i) {
        for (int32_t r = 0; r < k; ++r) col[r] = rows[(int64_t)r * n + i];
        out[i] = oracle_torch_sum_col(col, k, i, n) / (float)k;
    }
    free(col);
}

void oracle_torch_sum_rows(const float* rows, int32_t k, int64_t n, float* out) {
    float* col = (float*)malloc(sizeof(float) * (size_t)k);
    for (int64_t i = 0; i < n; ++i) {
        for (int32_t r = 0; r < k; ++r) col[r] = rows[(int64_t)r * n + i];
        out[i] = oracle_torch_sum_col(col, k, i, n);
    }
    free(col);
}

static float row_value(const void* row, int32_t packed, float scale, int64_t i) {
    int v;
    if (packed) {
        uint8_t b = ((const uint8_t*)row)[i / 2];
        v = (i & 1) ? ((b & 0xF) - 8) : (((b >> 4) & 0xF) - 8);
    } else {
        v = ((const int8_t*)row)[i];
    }
    return scale * (float)v;
}

/* The receiving peer's mean with its own update exact (Src/ADFL/Client/async_peer.py:170-174,
 * Examples/ray_ad.py:183-188: own fp32 parameters appended after the received updates, then
 * stack(...).mean(0)): the row sequence is the rows other than self_row in r order, then self_x; summed in
 * torch's order for an n-element tensor, then / K. self_row < 0: all K rows (simple_aggregate of K decodes).
 * int4 rows when packed != 0 (compression.py:51-66). */
void oracle_slq_dequantize_mean_self(const void* const* rows, const float* scales, int32_t k, int64_t n,
                                     int32_t self_row, const float* self_x, int32_t packed, float* out) {
    float* col = (float*)malloc(sizeof(float) * (size_t)k);
    for (int64_t i = 0; i < n; ++i) {
        int32_t s = 0;
        for (int32_t r = 0; r < k; ++r) {
            if (r == self_row) continue;
            col[s++] = row_value(rows[r], packed, scales[r], i);
        }
        if (self_row >= 0) col[s++] = self_x[i];
        out[i] = oracle_torch_sum_col(col, k, i, n) / (float)k;
    }
    free(col);
}

/* Peer mean / aggregate of K decoded int8 payloads of one n-element tensor. */
void oracle_slq_dequantize_mean(const int8_t* const* qs, const float* scales, int32_t k, int64_t n, float* out) {
    oracle_slq_dequantize_mean_self((const void* const*)qs, scales, k, n, -1, NULL, 0, out);
}

/* Same mean over K int4-packed payloads (unpack_4bit then dequantize, compression.py:51-66). */
void oracle_slq_dequantize_mean_int4(const uint8_t* const* ps, const float* scales, int32_t k, int64_t n, float* out) {
    oracle_slq_dequantize_mean_self((const void* const*)ps, scales, k, n, -1, NULL, 1, out);
}

/* Thread-free helper the tests use for SHA inputs of recipe cases. */
uint32_t oracle_f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* torch.linalg.vector_norm(x, ord=2) on an fp32 CPU tensor as torch 2.10 computes it (the reference's
 * QSGD / CNAT scale, Src/ADFL/Channel/quant.py:226,512), restated from its observed behaviour and pinned
 * against torch itself (tests/test_torch_norm_dtypes.py) and every L2 norm in tests/golden/stoch.npz:
 *   the vectorised kernel: 8 fp32 lane accumulators, acc[j] = fma(x[8i+j], x[8i+j], acc[j]) over the
 *   n - n % 8 leading elements in order; b = acc[0] + acc[1] + ... + acc[7] left to right; then the n % 8
 *   tail as the compiler emitted the scalar loop `b += x * x`: a first group of 4 (when the tail holds 4
 *   or more) with the squares rounded and added in order (an in-order vectorised reduction), the rest
 *   with fma. Below 8 elements the same rules with no lane accumulators (b starts at 0).
 *   result: the correctly rounded fp32 sqrt of b. A one-element tensor's norm is |x| (every dtype).
 * fmaf() is C99's single-rounding fused multiply-add. */
float oracle_torch_l2_norm(const float* x, int64_t n) {
    if (n == 1) return fabsf(x[0]);  /* a one-element tensor's norm is |x| (no square: no underflow) */
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t nv = n - n % 8;
    for (int64_t i = 0; i < nv; i += 8)
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(x[i + j], x[i + j], acc[j]);
    float b = acc[0];
    for (int j = 1; j < 8; ++j) b = b + acc[j];
    int64_t d = nv;
    if (n - d >= 4) {
        for (int k = 0; k < 4; ++k) {
            const float sq = x[d + k] * x[d + k];
            b = b + sq;
        }
        d += 4;
    }
    for (int64_t i = d; i < n; ++i) b = fmaf(x[i], x[i], b);
    return sqrtf(b);
}

/* The same norm for the reference's other float dtypes (QSGD / CNAT on an fp16 / bf16 / fp64 tensor,
 * quant.py:226,512), torch 2.10's CPU kernels restated from their observed behaviour and pinned against
 * torch itself (tests/test_torch_norm_dtypes.py, tests/golden/torch_norm_dt.npz). The fp32 sqrt is returned;
 * the caller rounds it to the dtype (torch's round-to-nearest-even conversion). x*x of an fp16 / bf16 value
 * is exact in fp32, so fused and separate multiply-add give the same steps.
 *   bf16: the vectorised kernel over 16-element vectors: 8 fp32 lane accumulators, element e into lane e % 8
 *         for e < n - n % 16, in order; lane sum left to right; the n % 16 tail added in order.
 *   fp16: the generic reduction (binary_kernel_reduce): below 32768 elements or with one thread, one fp32
 *         accumulator over every element in order; otherwise at::parallel_for's split — nt = min(threads,
 *         ceil(n / 32768)) chunks of ceil(n / nt) elements, each summed in order from 0 — then the chunk
 *         sums added in chunk order to 0. `threads` is torch.get_num_threads() of the calling process.
 *   fp64: 4 fp64 FMA lane accumulators (element e into lane e % 4 for e < n - n % 4), lane sum left to
 *         right, the n % 4 tail with fma (also below 4 elements); correctly rounded fp64 sqrt. */
static float bf16_f(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }
static float f16_f(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1F, m = h & 0x3FF;
    float f;
    if (e == 0) {
        f = ldexpf((float)m, -24);
        if (s) f = -f;
        return f;
    }
    uint32_t u = s | (e == 31 ? (0xFFu << 23) | (m << 13) : ((e + 112) << 23) | (m << 13));
    memcpy(&f, &u, 4);
    return f;
}

float oracle_torch_l2_norm_bf16(const uint16_t* x, int64_t n) {
    if (n == 1) return fabsf(bf16_f(x[0]));
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t nv = n - n % 16;
    for (int64_t i = 0; i < nv; ++i) {
        const float v = bf16_f(x[i]);
        acc[i % 8] = fmaf(v, v, acc[i % 8]);
    }
    float b = acc[0];
    for (int j = 1; j < 8; ++j) b = b + acc[j];
    for (int64_t i = nv; i < n; ++i) {
        const float v = bf16_f(x[i]);
        b = fmaf(v, v, b);
    }
    return sqrtf(b);
}

float oracle_torch_l2_norm_f16(const uint16_t* x, int64_t n, int32_t threads) {
    if (n == 1) return fabsf(f16_f(x[0]));
    int64_t nt = 1;
    if (n >= 32768 && threads > 1) {
        nt = (n + 32767) / 32768;
        if (nt > threads) nt = threads;
    }
    const int64_t cs = (n + nt - 1) / nt;
    float tot = 0.0f;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t b0 = t * cs, e0 = b0 + cs < n ? b0 + cs : n;
        float a = 0.0f;
        for (int64_t i = b0; i < e0; ++i) {
            const float v = f16_f(x[i]);
            a = fmaf(v, v, a);
        }
        tot = tot + a;
    }
    return sqrtf(tot);
}

double oracle_torch_l2_norm_f64(const double* x, int64_t n) {
    if (n == 1) return fabs(x[0]);
    double acc[4] = {0, 0, 0, 0};
    const int64_t nv = n - n % 4;
    for (int64_t i = 0; i < nv; i += 4)
        for (int j = 0; j < 4; ++j) acc[j] = fma(x[i + j], x[i + j], acc[j]);
    double b = acc[0];
    for (int j = 1; j < 4; ++j) b = b + acc[j];
    for (int64_t i = nv; i < n; ++i) b = fma(x[i], x[i], b);
    return sqrt(b);
}

/* torch.sum(t) of a contiguous fp32 CPU tensor to a scalar, as torch 2.10 computes it (cascade_sum over a
 * TensorIterator reduced to one output; aten/src/ATen/native/cpu/SumKernel.cpp with 8-float AVX2 vectors,
 * TensorIteratorReduce.cpp parallel_reduce), restated and pinned against torch itself
 * (tests/test_qerror_order.py). The reference's q-error metrics take it per tensor,
 * torch.sum((a - b) ** 2) (Src/ADFL/model.py:266-284), and over the product vector of
 * cosine_similarity (model.py:302-323).
 *   level(count)  multi_row_sum's cascade over one column of `count` values: level_power lp =
 *                 max(4, CeilLog2(count) / 4) (CeilLog2(x) = 1 for x <= 2, else floor(log2(x - 1)) + 1);
 *                 acc0 adds values in order; after every 2^lp values acc1 += acc0, acc0 = 0, and at every
 *                 2^(2 lp) acc2 += acc1, acc1 = 0, at every 2^(3 lp) acc3 += acc2, acc2 = 0; at the end
 *                 ((acc0 + acc1) + acc2) + acc3.
 *   row(L)        row_sum: four partials (values 4g + p, g < L / 4, each a level() cascade over L / 4), the
 *                 L % 4 leftovers added to partial 0 in order, then ((p0 + p1) + p2) + p3.
 *   inner(L)      L >= 8 (vectorized_inner_sum): lane l (0..7) is row() over the L / 8 vectors' element l;
 *                 0 + the L % 8 trailing values in order, then + lane 0, .., lane 7. L < 8: row(L).
 *   sum(n, T)     n < 32768 (at::internal::GRAIN_SIZE) or T == 1: 0 + inner(n). Otherwise the two-pass
 *                 reduction: at::parallel_for's split (nt = min(T, ceil(n / 32768)) ranges of ceil(n / nt)),
 *                 buffer[t] = 0 + inner(range t) for each range, zeros in the other T - nt slots, and the
 *                 result 0 + inner over the T buffer values. T is torch.get_num_threads() of the caller. */
static int level_power(int64_t count) {
    int c = 1;
    if (count > 2) {
        uint64_t v = (uint64_t)count - 1;
        c = 0;
        while (v) { ++c; v >>= 1; }
    }
    return c / 4 > 4 ? c / 4 : 4;
}

static float level_sum(const float* d, int64_t count, int64_t stride) {
    const int lp = level_power(count);
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int64_t i = 0;
    while (i + step <= count) {
        for (int64_t j = 0; j < step; ++j, ++i) acc[0] = acc[0] + d[i * stride];
        for (int j = 1; j < 4; ++j) {
            acc[j] = acc[j] + acc[j - 1];
            acc[j - 1] = 0.0f;
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < count; ++i) acc[0] = acc[0] + d[i * stride];
    for (int j = 1; j < 4; ++j) acc[0] = acc[0] + acc[j];
    return acc[0];
}

static float row_sum_f(const float* d, int64_t n, int64_t stride) {
    const int64_t g = n / 4;
    float p[4];
    for (int k = 0; k < 4; ++k) p[k] = level_sum(d + k * stride, g, 4 * stride);
    for (int64_t i = 4 * g; i < n; ++i) p[0] = p[0] + d[i * stride];
    for (int k = 1; k < 4; ++k) p[0] = p[0] + p[k];
    return p[0];
}

static float inner_sum_f(const float* d, int64_t n) {
    if (n < 8) return row_sum_f(d, n, 1);
    const int64_t v = n / 8;
    float acc = 0.0f;
    for (int64_t i = 8 * v; i < n; ++i) acc = acc + d[i];
    for (int l = 0; l < 8; ++l) acc = acc + row_sum_f(d + l, v, 8);
    return acc;
}

float oracle_torch_sum_f32(const float* x, int64_t n, int32_t threads) {
    if (n < 32768 || threads <= 1) return 0.0f + inner_sum_f(x, n);
    int64_t nt = (n + 32767) / 32768;
    if (nt > threads) nt = threads;
    const int64_t cs = (n + nt - 1) / nt;
    float* buf = (float*)calloc((size_t)threads, sizeof(float));
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t b = t * cs;
        if (b < n) buf[t] = 0.0f + inner_sum_f(x + b, (cs < n - b ? cs : n - b));
    }
    const float r = 0.0f + inner_sum_f(buf, threads);
    free(buf);
    return r;
}

/* The reference's q-error metrics of an update x against its decode d (Src/ADFL/Client/worker.py:186-189:
 * parameter_relative_mse and parameter_cosine_similarity with exclude_bias=True, Src/ADFL/model.py:256-323),
 * for the ndim > 1 tensors given back to back in x / d (sizes[t] elements each, dict order):
 *   e[t] = torch.sum((x_t - d_t) ** 2), s[t] = torch.sum((x_t - 0) ** 2)   (fp32, the order above)
 *   *cos = torch.sum((x / max(|x|, 1e-8)) * (d / max(|d|, 1e-8)))           (F.cosine_similarity, dim=0)
 * with |.| the reference-order fp32 norm (oracle_torch_l2_norm) and max the NaN-propagating clamp_min.
 * The caller forms the Python doubles: mse = sum(float(e[t])) / N etc. */
void oracle_qerror_ref(const float* x, const float* d, const int64_t* sizes, int32_t ntensors, int32_t threads,
                       float* e, float* s, float* cos_out) {
    int64_t total = 0, mx = 0;
    for (int32_t t = 0; t < ntensors; ++t) {
        total += sizes[t];
        if (sizes[t] > mx) mx = sizes[t];
    }
    float* tmp = (float*)malloc(sizeof(float) * (size_t)(total > 0 ? total : 1));
    int64_t off = 0;
    for (int32_t t = 0; t < ntensors; ++t) {
        const int64_t n = sizes[t];
        for (int64_t i = 0; i < n; ++i) {
            const float df = x[off + i] - d[off + i];
            tmp[i] = df * df;
        }
        e[t] = oracle_torch_sum_f32(tmp, n, threads);
        for (int64_t i = 0; i < n; ++i) {
            const float a = x[off + i] - 0.0f;
            tmp[i] = a * a;
        }
        s[t] = oracle_torch_sum_f32(tmp, n, threads);
        off += n;
    }
    float n1 = oracle_torch_l2_norm(x, total), n2 = oracle_torch_l2_norm(d, total);
    const float eps = 1e-8f;
    if (!(n1 != n1) && n1 < eps) n1 = eps;
    if (!(n2 != n2) && n2 < eps) n2 = eps;
    for (int64_t i = 0; i < total; ++i) {
        const float a = x[i] / n1, b = d[i] / n2;
        tmp[i] = a * b;
    }
    *cos_out = oracle_torch_sum_f32(tmp, total, threads);
    free(tmp);
    (void)mx;
}
