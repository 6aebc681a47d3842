// slq_codec.hip — MI355X (gfx950, CDNA4) kernels for ADFL's SLQ gradient codec + the C ABI of
// include/adfl_slq.h.
//
// Reference behaviour restated here (bit-exact, pinned by tests/golden):
//   encode  Src/ADFL/Channel/quant.py:97-104   scale = max|x| / q_max ; torch.quantize_per_tensor
//   decode  Src/ADFL/Channel/quant.py:107-112  q.dequantize()
//   loop    Src/ADFL/Channel/quant.py:74-94    per-tensor scales over a whole state dict (bucketed)
//   int4    Src/ADFL/compression.py:35-66      pack_4bit / unpack_4bit nibble layout
//   mean    Examples/ray_ad.py:188             stack(updates).mean(0) after the peer exchange
//
// Design (DESIGN.md has the byte accounting): the codec is a pure HBM stream, ~6 VALU ops per
// element, so every kernel is built for bandwidth — 16-byte loads and stores per lane (1 KiB per
// wave-instruction), grid-stride loops sized to fill 256 CUs x 8 resident 256-thread blocks, no
// atomics and no inter-workgroup hand-off inside a launch. The one grid-wide dependency (the scale
// needs max|x| over the whole tensor) is a kernel boundary: pass 1 writes one absmax partial per
// block, pass 2 re-reduces those partials (<= 8 KiB, L2-resident) in every block's prologue.
// Pass 2 walks the tensor in the opposite direction to pass 1, so its first ~200 MB are the bytes
// pass 1 read last and are still resident in the 256 MiB Infinity Cache; decode walks opposite to
// pass 2 for the same reason on the payload. Outputs do not depend on traversal order.
//
// Numerics: no fast-math, fp32 denormals preserved (gfx950 default), -ffp-contract=off. Scale and
// reciprocal are computed as fp64 quotients rounded once to fp32, which equals the correctly
// rounded fp32 quotient (53 >= 2*24+2), independent of the compiler's fp32 division lowering.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "adfl_slq.h"

namespace {

constexpr int kBlock = 256;                 // 4 waves of 64
constexpr int kMaxFlatBlocks = 2048;        // 256 CUs x 8 resident blocks
constexpr int kCountSlot = kMaxFlatBlocks;  // workspace word holding pass 1's partial count
constexpr int64_t kWorkspaceBytes = 16384;  // >= (kMaxFlatBlocks + 1) * 4, padded

// ------------------------------------------------------------------------------------------------
// element helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t abs_bits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

// max|x| as an unsigned compare of the magnitude bits: identical to the float order on non-NaN
// values, and every NaN (> 0x7f800000) wins, so NaN propagates exactly like torch.max.
__device__ __forceinline__ uint32_t abs_bits4(float4 v) {
  return max(max(abs_bits(v.x), abs_bits(v.y)), max(abs_bits(v.z), abs_bits(v.w)));
}

// torch.quantize_per_tensor(x, scale, 0, qint8) on one element, given inv = fp32(1/scale).
__device__ __forceinline__ int quant1(float x, float inv) {
  float y = x * inv;
  y = __builtin_isnan(y) ? 127.0f : __builtin_fminf(__builtin_fmaxf(y, -128.0f), 127.0f);
  return (int)__builtin_rintf(y);  // v_rndne_f32: round half to even
}

__device__ __forceinline__ uint32_t quant4(float4 v, float inv) {
  return (uint32_t(quant1(v.x, inv)) & 0xffu) | ((uint32_t(quant1(v.y, inv)) & 0xffu) << 8) |
         ((uint32_t(quant1(v.z, inv)) & 0xffu) << 16) | (uint32_t(quant1(v.w, inv)) << 24);
}

__device__ __forceinline__ float4 dequant4(uint32_t w, float s) {
  float4 r;
  r.x = s * (float)(int8_t)(w & 0xffu);
  r.y = s * (float)(int8_t)((w >> 8) & 0xffu);
  r.z = s * (float)(int8_t)((w >> 16) & 0xffu);
  r.w = s * (float)(int8_t)(w >> 24);
  return r;
}

// pack_4bit on one pair: ((hi+8) << 4 | (lo+8)) in int8 wraparound; lo is deliberately NOT masked
// to a nibble (compression.py:45-48 ORs the full shifted int8), so out-of-range values alias.
__device__ __forceinline__ uint32_t pack_pair(int hi, int lo) {
  return ((uint32_t(hi + 8) << 4) | uint32_t(lo + 8)) & 0xffu;
}

// 8 quantized elements (two float4) -> 4 packed bytes.
__device__ __forceinline__ uint32_t quant8_int4(float4 a, float4 b, float inv) {
  return pack_pair(quant1(a.x, inv), quant1(a.y, inv)) | (pack_pair(quant1(a.z, inv), quant1(a.w, inv)) << 8) |
         (pack_pair(quant1(b.x, inv), quant1(b.y, inv)) << 16) | (pack_pair(quant1(b.z, inv), quant1(b.w, inv)) << 24);
}

// unpack_4bit (compression.py:60-61) on one packed byte: high nibble = even element.
__device__ __forceinline__ void dequant_byte_int4(uint32_t b, float s, float& e0, float& e1) {
  e0 = s * (float)((int)((b >> 4) & 0xfu) - 8);
  e1 = s * (float)((int)(b & 0xfu) - 8);
}

__device__ __forceinline__ void dequant8_int4(uint32_t w, float s, float4& a, float4& b) {
  dequant_byte_int4(w & 0xffu, s, a.x, a.y);
  dequant_byte_int4((w >> 8) & 0xffu, s, a.z, a.w);
  dequant_byte_int4((w >> 16) & 0xffu, s, b.x, b.y);
  dequant_byte_int4(w >> 24, s, b.z, b.w);
}

// scale = fp32(absmax / q_max) (quant.py:99-100: fp32 tensor / Python int, i.e. / float(q_max));
// inv = fp32(1 / scale) as fbgemm's quantizer forms it.
struct ScaleInv {
  float scale, inv;
};
__device__ __forceinline__ ScaleInv make_scale(uint32_t absmax_bits, float qmax) {
  const float amax = __uint_as_float(absmax_bits);
  ScaleInv r;
  r.scale = (float)((double)amax / (double)qmax);
  r.inv = (float)(1.0 / (double)r.scale);
  return r;
}

// ------------------------------------------------------------------------------------------------
// reductions
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Block-wide max, result broadcast to every thread.
__device__ __forceinline__ uint32_t block_max(uint32_t v) {
  __shared__ uint32_t red[kBlock / 64];
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = max(max(red[0], red[1]), max(red[2], red[3]));
  return v;
}

// Every block of a pass-2 kernel re-reduces the pass-1 partials (a kernel boundary separates them,
// so plain loads see pass 1's stores).
__device__ __forceinline__ uint32_t reduce_partials(const uint32_t* __restrict__ p, int count) {
  uint32_t m = 0;
  for (int k = threadIdx.x; k < count; k += kBlock) m = max(m, p[k]);
  return block_max(m);
}

// ------------------------------------------------------------------------------------------------
// flat kernels (one tensor)
// ------------------------------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(kBlock) void k_absmax_flat(const float* __restrict__ x, int64_t n,
                                                        uint32_t* __restrict__ partials) {
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t m = 0;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x4[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) m = max(m, abs_bits4(v[u]));
  }
  for (; i < n4; i += stride) m = max(m, abs_bits4(x4[i]));
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) m = max(m, abs_bits(x[(n4 << 2) + threadIdx.x]));
  m = block_max(m);
  if (threadIdx.x == 0) partials[blockIdx.x] = m;
  if (blockIdx.x == 0 && threadIdx.x == 0) partials[kCountSlot] = gridDim.x;  // self-describing workspace
}

// One lane = one 16-element group: four 16-byte loads, one 16-byte store.
template <bool REVERSE>
__global__ __launch_bounds__(kBlock) void k_quantize_flat(const float* __restrict__ x, int64_t n, float qmax,
                                                          const uint32_t* __restrict__ partials,
                                                          int8_t* __restrict__ q, float* __restrict__ scale_out) {
  const ScaleInv si = make_scale(reduce_partials(partials, (int)partials[kCountSlot]), qmax);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = si.scale;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint4* q16 = reinterpret_cast<uint4*>(q);
  const int64_t ng = n >> 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t g0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; g0 < ng; g0 += stride) {
    const int64_t g = REVERSE ? ng - 1 - g0 : g0;
    const float4 a = x4[4 * g], b = x4[4 * g + 1], c = x4[4 * g + 2], d = x4[4 * g + 3];
    q16[g] = make_uint4(quant4(a, si.inv), quant4(b, si.inv), quant4(c, si.inv), quant4(d, si.inv));
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = (ng << 4) + threadIdx.x; i < n; i += kBlock) q[i] = (int8_t)quant1(x[i], si.inv);
}

// One lane = one 16-element group: one 16-byte load, four 16-byte stores.
template <bool REVERSE>
__global__ __launch_bounds__(kBlock) void k_dequantize_flat(const int8_t* __restrict__ q, int64_t n,
                                                            const float* __restrict__ scale_p,
                                                            float* __restrict__ out) {
  const float s = *scale_p;
  const uint4* q16 = reinterpret_cast<const uint4*>(q);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ng = n >> 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t g0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; g0 < ng; g0 += stride) {
    const int64_t g = REVERSE ? ng - 1 - g0 : g0;
    const uint4 p = q16[g];
    o4[4 * g] = dequant4(p.x, s);
    o4[4 * g + 1] = dequant4(p.y, s);
    o4[4 * g + 2] = dequant4(p.z, s);
    o4[4 * g + 3] = dequant4(p.w, s);
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = (ng << 4) + threadIdx.x; i < n; i += kBlock) out[i] = s * (float)q[i];
}

// int4: one lane = one 32-element group: eight 16-byte loads, one 16-byte store of packed nibbles.
template <bool REVERSE>
__global__ __launch_bounds__(kBlock) void k_quantize_int4_flat(const float* __restrict__ x, int64_t n, float qmax,
                                                               const uint32_t* __restrict__ partials,
                                                               uint8_t* __restrict__ packed,
                                                               float* __restrict__ scale_out) {
  const ScaleInv si = make_scale(reduce_partials(partials, (int)partials[kCountSlot]), qmax);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = si.scale;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint4* p16 = reinterpret_cast<uint4*>(packed);
  const int64_t ng = n >> 5;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t g0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; g0 < ng; g0 += stride) {
    const int64_t g = REVERSE ? ng - 1 - g0 : g0;
    const float4* s = x4 + 8 * g;
    const float4 v0 = s[0], v1 = s[1], v2 = s[2], v3 = s[3], v4 = s[4], v5 = s[5], v6 = s[6], v7 = s[7];
    p16[g] = make_uint4(quant8_int4(v0, v1, si.inv), quant8_int4(v2, v3, si.inv), quant8_int4(v4, v5, si.inv),
                        quant8_int4(v6, v7, si.inv));
  }
  if (blockIdx.x == gridDim.x - 1) {
    const int64_t np = (n + 1) >> 1;
    for (int64_t j = (ng << 4) + threadIdx.x; j < np; j += kBlock) {
      const int hi = quant1(x[2 * j], si.inv);
      const int lo = (2 * j + 1 < n) ? quant1(x[2 * j + 1], si.inv) : 0;  // pad with one zero (compression.py:42-43)
      packed[j] = (uint8_t)pack_pair(hi, lo);
    }
  }
}

// int4 decode: one lane = one 32-element group: one 16-byte load, eight 16-byte stores.
template <bool REVERSE>
__global__ __launch_bounds__(kBlock) void k_dequantize_int4_flat(const uint8_t* __restrict__ packed, int64_t n,
                                                                 const float* __restrict__ scale_p,
                                                                 float* __restrict__ out) {
  const float s = *scale_p;
  const uint4* p16 = reinterpret_cast<const uint4*>(packed);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ng = n >> 5;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t g0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; g0 < ng; g0 += stride) {
    const int64_t g = REVERSE ? ng - 1 - g0 : g0;
    const uint4 p = p16[g];
    float4 a, b;
    float4* d = o4 + 8 * g;
    dequant8_int4(p.x, s, a, b);
    d[0] = a;
    d[1] = b;
    dequant8_int4(p.y, s, a, b);
    d[2] = a;
    d[3] = b;
    dequant8_int4(p.z, s, a, b);
    d[4] = a;
    d[5] = b;
    dequant8_int4(p.w, s, a, b);
    d[6] = a;
    d[7] = b;
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = (ng << 5) + threadIdx.x; i < n; i += kBlock) {
      const uint32_t b = packed[i >> 1];
      float e0, e1;
      dequant_byte_int4(b, s, e0, e1);
      out[i] = (i & 1) ? e1 : e0;
    }
}

// Standalone pack_4bit / unpack_4bit over int8 payloads (compression.py:35-66).
__global__ __launch_bounds__(kBlock) void k_pack_int4(const int8_t* __restrict__ q, int64_t n,
                                                      uint8_t* __restrict__ packed) {
  const int64_t np = (n + 1) >> 1;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < np; j += stride) {
    const int hi = q[2 * j];
    const int lo = (2 * j + 1 < n) ? (int)q[2 * j + 1] : 0;
    packed[j] = (uint8_t)pack_pair(hi, lo);
  }
}

__global__ __launch_bounds__(kBlock) void k_unpack_int4(const uint8_t* __restrict__ packed, int64_t n,
                                                        int8_t* __restrict__ q) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint32_t b = packed[i >> 1];
    q[i] = (int8_t)((i & 1) ? (int)(b & 0xfu) - 8 : (int)((b >> 4) & 0xfu) - 8);
  }
}

// Peer-exchange epilogue: mean of K dequantized rows, fp32, rows summed in order then / K.
__global__ __launch_bounds__(kBlock) void k_dequantize_mean(const int8_t* __restrict__ q, int64_t row_stride, int k,
                                                            int64_t n, const float* __restrict__ scales,
                                                            int64_t scale_stride, float* __restrict__ out) {
  const int64_t ng = n >> 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const double dk = (double)k;
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < ng; g += stride) {
    float acc[16];
    {
      const uint4 p = *reinterpret_cast<const uint4*>(q + 16 * g);
      const float s = scales[0];
      const uint32_t w[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = dequant4(w[j], s);
        acc[4 * j] = v.x;
        acc[4 * j + 1] = v.y;
        acc[4 * j + 2] = v.z;
        acc[4 * j + 3] = v.w;
      }
    }
    for (int r = 1; r < k; ++r) {
      const uint4 p = *reinterpret_cast<const uint4*>(q + r * row_stride + 16 * g);
      const float s = scales[r * scale_stride];
      const uint32_t w[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = dequant4(w[j], s);
        acc[4 * j] += v.x;
        acc[4 * j + 1] += v.y;
        acc[4 * j + 2] += v.z;
        acc[4 * j + 3] += v.w;
      }
    }
    float4* o4 = reinterpret_cast<float4*>(out + 16 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o4[j] = make_float4((float)((double)acc[4 * j] / dk), (float)((double)acc[4 * j + 1] / dk),
                          (float)((double)acc[4 * j + 2] / dk), (float)((double)acc[4 * j + 3] / dk));
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = (ng << 4) + threadIdx.x; i < n; i += kBlock) {
      float acc = scales[0] * (float)q[i];
      for (int r = 1; r < k; ++r) acc += scales[r * scale_stride] * (float)q[r * row_stride + i];
      out[i] = (float)((double)acc / dk);
    }
}

// int4 variant of the exchange epilogue: K packed rows (ceil(n/2) bytes each), one lane = 32 elements.
__global__ __launch_bounds__(kBlock) void k_dequantize_mean_int4(const uint8_t* __restrict__ p, int64_t row_stride,
                                                                 int k, int64_t n, const float* __restrict__ scales,
                                                                 int64_t scale_stride, float* __restrict__ out) {
  const int64_t ng = n >> 5;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const double dk = (double)k;
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < ng; g += stride) {
    float acc[32];
    for (int r = 0; r < k; ++r) {
      const uint4 w = *reinterpret_cast<const uint4*>(p + r * row_stride + 16 * g);
      const float s = scales[r * scale_stride];
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float4 a, b;
        dequant8_int4(ws[j], s, a, b);
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[8 * j + e] = (r == 0) ? v[e] : acc[8 * j + e] + v[e];
      }
    }
    float4* o4 = reinterpret_cast<float4*>(out + 32 * g);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o4[j] = make_float4((float)((double)acc[4 * j] / dk), (float)((double)acc[4 * j + 1] / dk),
                          (float)((double)acc[4 * j + 2] / dk), (float)((double)acc[4 * j + 3] / dk));
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = (ng << 5) + threadIdx.x; i < n; i += kBlock) {
      float acc = 0.0f;
      for (int r = 0; r < k; ++r) {
        float e0, e1;
        dequant_byte_int4(p[r * row_stride + (i >> 1)], scales[r * scale_stride], e0, e1);
        acc = (r == 0) ? ((i & 1) ? e1 : e0) : acc + ((i & 1) ? e1 : e0);
      }
      out[i] = (float)((double)acc / dk);
    }
}

// ------------------------------------------------------------------------------------------------
// bucketed kernels (many tensors, one block per chunk of <= 8192 elements)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_absmax_batched(const float* __restrict__ x,
                                                           const adfl_slq_chunk* __restrict__ chunks,
                                                           uint32_t* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  const float4* x4 = reinterpret_cast<const float4*>(xc);
  const int ng = c.len >> 4;
  uint32_t m = 0;
  for (int g = threadIdx.x; g < ng; g += kBlock) {
    const float4 a = x4[4 * g], b = x4[4 * g + 1], d = x4[4 * g + 2], e = x4[4 * g + 3];
    m = max(m, max(max(abs_bits4(a), abs_bits4(b)), max(abs_bits4(d), abs_bits4(e))));
  }
  for (int i = (ng << 4) + threadIdx.x; i < c.len; i += kBlock) m = max(m, abs_bits(xc[i]));
  m = block_max(m);
  if (threadIdx.x == 0) partials[blockIdx.x] = m;
}

__global__ __launch_bounds__(kBlock) void k_quantize_batched(const float* __restrict__ x,
                                                             const adfl_slq_chunk* __restrict__ chunks,
                                                             int64_t nchunks, float qmax,
                                                             const uint32_t* __restrict__ partials,
                                                             int8_t* __restrict__ q, float* __restrict__ scales) {
  const int64_t ci = nchunks - 1 - (int64_t)blockIdx.x;  // reverse of pass 1 (Infinity Cache reuse)
  const adfl_slq_chunk c = chunks[ci];
  const ScaleInv si = make_scale(reduce_partials(partials + c.first_chunk, c.nchunks), qmax);
  if (ci == c.first_chunk && threadIdx.x == 0) scales[c.tensor] = si.scale;
  const float* xc = x + c.start;
  int8_t* qc = q + c.start;
  const float4* x4 = reinterpret_cast<const float4*>(xc);
  uint4* q16 = reinterpret_cast<uint4*>(qc);
  const int ng = c.len >> 4;
  for (int g = threadIdx.x; g < ng; g += kBlock) {
    const float4 a = x4[4 * g], b = x4[4 * g + 1], d = x4[4 * g + 2], e = x4[4 * g + 3];
    q16[g] = make_uint4(quant4(a, si.inv), quant4(b, si.inv), quant4(d, si.inv), quant4(e, si.inv));
  }
  for (int i = (ng << 4) + threadIdx.x; i < c.len; i += kBlock) qc[i] = (int8_t)quant1(xc[i], si.inv);
}

__global__ __launch_bounds__(kBlock) void k_dequantize_batched(const int8_t* __restrict__ q,
                                                               const adfl_slq_chunk* __restrict__ chunks,
                                                               const float* __restrict__ scales,
                                                               float* __restrict__ out) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float s = scales[c.tensor];
  const int8_t* qc = q + c.start;
  float* oc = out + c.start;
  const uint4* q16 = reinterpret_cast<const uint4*>(qc);
  float4* o4 = reinterpret_cast<float4*>(oc);
  const int ng = c.len >> 4;
  for (int g = threadIdx.x; g < ng; g += kBlock) {
    const uint4 p = q16[g];
    o4[4 * g] = dequant4(p.x, s);
    o4[4 * g + 1] = dequant4(p.y, s);
    o4[4 * g + 2] = dequant4(p.z, s);
    o4[4 * g + 3] = dequant4(p.w, s);
  }
  for (int i = (ng << 4) + threadIdx.x; i < c.len; i += kBlock) oc[i] = s * (float)qc[i];
}

// ------------------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------------------
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int grid_for(int64_t work_items) {
  int64_t g = (work_items + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > kMaxFlatBlocks ? kMaxFlatBlocks : g);
}

inline int check_bits(int bits) { return (bits >= 1 && bits <= 16) ? ADFL_OK : ADFL_E_BITS; }

// q_max as the fp32 value torch divides by (quant.py:99-100).
inline float qmax_f(int bits) { return (float)((1LL << (bits - 1)) - 1); }

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ADFL_OK : (int)e;
}

// Pass-1 grid for a flat tensor: the partial count pass 2 must reduce.
inline int absmax_grid(int64_t n) { return grid_for(((n >> 2) + 3) / 4); }

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int adfl_slq_abi_version(void) { return ADFL_SLQ_ABI_VERSION; }

const char* adfl_slq_strerror(int status) {
  switch (status) {
    case ADFL_OK: return "ok";
    case ADFL_E_ARG: return "adfl_slq: invalid argument (null pointer, count or tensor table)";
    case ADFL_E_BITS: return "adfl_slq: bits must be in [1, 16]";
    case ADFL_E_ALIGN: return "adfl_slq: device data pointers must be 16-byte aligned";
    case ADFL_E_WORKSPACE: return "adfl_slq: workspace smaller than adfl_slq_workspace_bytes()";
    default: return status > 0 ? hipGetErrorString((hipError_t)status) : "adfl_slq: unknown error";
  }
}

int64_t adfl_slq_workspace_bytes(void) { return kWorkspaceBytes; }

int adfl_slq_absmax(const float* d_x, int64_t n, void* d_workspace, int64_t workspace_bytes, void* stream) {
  if (!d_x || !d_workspace || n < 1) return ADFL_E_ARG;
  if (!aligned16(d_x) || !aligned16(d_workspace)) return ADFL_E_ALIGN;
  if (workspace_bytes < kWorkspaceBytes) return ADFL_E_WORKSPACE;
  hipLaunchKernelGGL(k_absmax_flat<4>, dim3(absmax_grid(n)), dim3(kBlock), 0, (hipStream_t)stream, d_x, n,
                     (uint32_t*)d_workspace);
  return launch_status();
}

int adfl_slq_quantize(const float* d_x, int64_t n, int bits, const void* d_workspace, int8_t* d_q, float* d_scale,
                      void* stream) {
  if (!d_x || !d_workspace || !d_q || !d_scale || n < 1) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_q)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_quantize_flat<true>, dim3(grid_for(n >> 4)), dim3(kBlock), 0, (hipStream_t)stream, d_x, n,
                     qmax_f(bits), (const uint32_t*)d_workspace, d_q, d_scale);
  return launch_status();
}

int adfl_slq_encode(const float* d_x, int64_t n, int bits, int8_t* d_q, float* d_scale, void* d_workspace,
                    int64_t workspace_bytes, void* stream) {
  if (int s = check_bits(bits)) return s;
  if (int s = adfl_slq_absmax(d_x, n, d_workspace, workspace_bytes, stream)) return s;
  return adfl_slq_quantize(d_x, n, bits, d_workspace, d_q, d_scale, stream);
}

int adfl_slq_dequantize(const int8_t* d_q, int64_t n, const float* d_scale, float* d_out, void* stream) {
  if (!d_q || !d_scale || !d_out || n < 1) return ADFL_E_ARG;
  if (!aligned16(d_q) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_flat<false>, dim3(grid_for(n >> 4)), dim3(kBlock), 0, (hipStream_t)stream, d_q, n,
                     d_scale, d_out);
  return launch_status();
}

int64_t adfl_slq_build_chunks(const int64_t* offsets, const int64_t* sizes, int32_t ntensors, adfl_slq_chunk* chunks,
                              int64_t capacity) {
  if (!offsets || !sizes || ntensors < 1) return ADFL_E_ARG;
  int64_t count = 0;
  for (int32_t t = 0; t < ntensors; ++t) {
    if (sizes[t] < 1 || offsets[t] < 0 || offsets[t] % ADFL_SLQ_ALIGN_ELEMS != 0) return ADFL_E_ARG;
    const int64_t nc = (sizes[t] + ADFL_SLQ_CHUNK_ELEMS - 1) / ADFL_SLQ_CHUNK_ELEMS;
    if (nc > INT32_MAX || count + nc > INT32_MAX) return ADFL_E_ARG;
    if (chunks) {
      if (count + nc > capacity) return ADFL_E_ARG;
      for (int64_t k = 0; k < nc; ++k) {
        adfl_slq_chunk& c = chunks[count + k];
        c.start = offsets[t] + k * ADFL_SLQ_CHUNK_ELEMS;
        const int64_t rem = sizes[t] - k * ADFL_SLQ_CHUNK_ELEMS;
        c.len = (int32_t)(rem < ADFL_SLQ_CHUNK_ELEMS ? rem : ADFL_SLQ_CHUNK_ELEMS);
        c.tensor = t;
        c.first_chunk = (int32_t)count;
        c.nchunks = (int32_t)nc;
      }
    }
    count += nc;
  }
  return count;
}

int adfl_slq_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits, int8_t* d_q,
                            float* d_scales, uint32_t* d_partials, void* stream) {
  if (!d_x || !d_chunks || !d_q || !d_scales || !d_partials || nchunks < 1 || nchunks > INT32_MAX) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_q)) return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_absmax_batched, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, d_partials);
  if (int s = launch_status()) return s;
  hipLaunchKernelGGL(k_quantize_batched, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, nchunks,
                     qmax_f(bits), (const uint32_t*)d_partials, d_q, d_scales);
  return launch_status();
}

int adfl_slq_dequantize_batched(const int8_t* d_q, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                const float* d_scales, float* d_out, void* stream) {
  if (!d_q || !d_chunks || !d_scales || !d_out || nchunks < 1 || nchunks > INT32_MAX) return ADFL_E_ARG;
  if (!aligned16(d_q) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_batched, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_q,
                     d_chunks, d_scales, d_out);
  return launch_status();
}

int adfl_slq_quantize_int4(const float* d_x, int64_t n, int bits, const void* d_workspace, uint8_t* d_packed,
                           float* d_scale, void* stream) {
  if (!d_x || !d_workspace || !d_packed || !d_scale || n < 1) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_packed)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_quantize_int4_flat<true>, dim3(grid_for(n >> 5)), dim3(kBlock), 0, (hipStream_t)stream, d_x,
                     n, qmax_f(bits), (const uint32_t*)d_workspace, d_packed, d_scale);
  return launch_status();
}

int adfl_slq_encode_int4(const float* d_x, int64_t n, int bits, uint8_t* d_packed, float* d_scale, void* d_workspace,
                         int64_t workspace_bytes, void* stream) {
  if (int s = check_bits(bits)) return s;
  if (int s = adfl_slq_absmax(d_x, n, d_workspace, workspace_bytes, stream)) return s;
  return adfl_slq_quantize_int4(d_x, n, bits, d_workspace, d_packed, d_scale, stream);
}

int adfl_slq_dequantize_int4(const uint8_t* d_packed, int64_t n, const float* d_scale, float* d_out, void* stream) {
  if (!d_packed || !d_scale || !d_out || n < 1) return ADFL_E_ARG;
  if (!aligned16(d_packed) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_int4_flat<false>, dim3(grid_for(n >> 5)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_packed, n, d_scale, d_out);
  return launch_status();
}

int adfl_pack_int4(const int8_t* d_q, int64_t n, uint8_t* d_packed, void* stream) {
  if (!d_q || !d_packed || n < 1) return ADFL_E_ARG;
  hipLaunchKernelGGL(k_pack_int4, dim3(grid_for((n + 1) >> 1)), dim3(kBlock), 0, (hipStream_t)stream, d_q, n,
                     d_packed);
  return launch_status();
}

int adfl_unpack_int4(const uint8_t* d_packed, int64_t n, int8_t* d_q, void* stream) {
  if (!d_packed || !d_q || n < 1) return ADFL_E_ARG;
  hipLaunchKernelGGL(k_unpack_int4, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, d_packed, n, d_q);
  return launch_status();
}

int adfl_slq_dequantize_mean(const int8_t* d_q, int64_t row_stride_bytes, int32_t k, int64_t n,
                             const float* d_scales, int64_t scale_stride, float* d_out, void* stream) {
  if (!d_q || !d_scales || !d_out || n < 1 || k < 1 || row_stride_bytes < n || scale_stride < 1) return ADFL_E_ARG;
  if (!aligned16(d_q) || !aligned16(d_out) || (row_stride_bytes & 15) != 0) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_mean, dim3(grid_for(n >> 4)), dim3(kBlock), 0, (hipStream_t)stream, d_q,
                     row_stride_bytes, (int)k, n, d_scales, scale_stride, d_out);
  return launch_status();
}

int adfl_slq_dequantize_mean_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k, int64_t n,
                                  const float* d_scales, int64_t scale_stride, float* d_out, void* stream) {
  if (!d_packed || !d_scales || !d_out || n < 1 || k < 1 || row_stride_bytes < (n + 1) / 2 || scale_stride < 1)
    return ADFL_E_ARG;
  if (!aligned16(d_packed) || !aligned16(d_out) || (row_stride_bytes & 15) != 0) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_mean_int4, dim3(grid_for(n >> 5)), dim3(kBlock), 0, (hipStream_t)stream, d_packed,
                     row_stride_bytes, (int)k, n, d_scales, scale_stride, d_out);
  return launch_status();
}

}  // extern "C"
