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
// Design (DESIGN.md has the byte accounting and the measurements behind every choice): the codec is a
// pure HBM stream with ~6 VALU ops per element, so every kernel is built for bandwidth.
//  * Wave tiles. A wave owns a tile of 1024 elements (int4: 2048). Every global access is a 16-byte
//    per-lane access that is contiguous across the wave (1 KiB per wave-instruction). Where the natural
//    per-lane shape differs between input and output (4 floats in, 4 bytes out), the wave transposes
//    through 1 KiB of LDS, so both the loads and the stores stay fully coalesced.
//  * The one grid-wide dependency (scale needs max|x| over the whole tensor) is a kernel boundary:
//    pass 1 writes one absmax partial per block, pass 2 re-reduces them (<= 8 KiB, L2) in every block's
//    prologue. No atomics, no in-launch hand-off, deterministic.
//  * Cache policy per stream (MI355X 256 MiB Infinity Cache): pass 1 reads x block-contiguously with
//    non-temporal loads (kCacheKeepBytes = 0: keeping x's tail on-die for pass 2 measured slower).
//    Pass 2 reads x non-temporally (x is dead afterwards) and writes the payload backwards with
//    allocating stores; decode reads the payload forwards, starting on the bytes pass 2 wrote last,
//    which are still in the Infinity Cache. Decode writes its fp32 output with non-temporal stores
//    (nothing re-reads it soon; it must not evict the next pass's lines). No output bit depends on it.
//
// Numerics: no fast-math, fp32 denormals preserved (gfx950 default), -ffp-contract=off. Scale and
// reciprocal are fp64 quotients rounded once to fp32 = the correctly rounded fp32 quotient (53 >= 2*24+2),
// independent of the compiler's fp32 division lowering.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "adfl_slq.h"
#include "torch_sum_order.h"

namespace {

constexpr int kBlock = 256;                        // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kTile = 1024;                        // int8 path: elements per wave tile
constexpr int kTile4 = 2048;                       // int4 path: elements per wave tile
constexpr int kMaxFlatBlocks = 2048;               // 256 CUs x 8 resident 256-thread blocks
constexpr int kAbsmaxBlocks = 1024;                // pass-1 grid (block-contiguous ranges)
constexpr int kCountSlot = kMaxFlatBlocks;         // workspace word holding pass 1's partial count
constexpr int64_t kWorkspaceBytes = 16384;         // >= (kMaxFlatBlocks + 1) * 4, padded
constexpr int64_t kCacheKeepBytes = 0;             // tail of x pass 1 leaves in the Infinity Cache

typedef float f4v __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// memory helpers
// ------------------------------------------------------------------------------------------------
template <bool NT>
__device__ __forceinline__ float4 load4(const float4* p) {
  if (NT) {
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *p;
}

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 load16(const uint4* p) {
  if (NT) {
    const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}

template <bool NT>
__device__ __forceinline__ void store16(uint4* p, uint4 d) {
  if (NT) {
    const u4v v = {d.x, d.y, d.z, d.w};
    __builtin_nontemporal_store(v, reinterpret_cast<u4v*>(p));
  } else {
    *p = d;
  }
}

__device__ __forceinline__ void store4_nt(float4* p, float4 d) {
  const f4v v = {d.x, d.y, d.z, d.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
}

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

// 4 elements -> 2 packed bytes (high nibble = even element).
__device__ __forceinline__ uint32_t quant4_int4(float4 v, float inv) {
  return pack_pair(quant1(v.x, inv), quant1(v.y, inv)) | (pack_pair(quant1(v.z, inv), quant1(v.w, inv)) << 8);
}

// unpack_4bit (compression.py:60-61) on one packed byte: high nibble = even element.
__device__ __forceinline__ void dequant_byte_int4(uint32_t b, float s, float& e0, float& e1) {
  e0 = s * (float)((int)((b >> 4) & 0xfu) - 8);
  e1 = s * (float)((int)(b & 0xfu) - 8);
}

// 2 packed bytes -> 4 elements.
__device__ __forceinline__ float4 dequant2_int4(uint32_t h, float s) {
  float4 r;
  dequant_byte_int4(h & 0xffu, s, r.x, r.y);
  dequant_byte_int4((h >> 8) & 0xffu, s, r.z, r.w);
  return r;
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// fp32 mean = correctly rounded acc / K (torch: sum then true division).
__device__ __forceinline__ float4 div4(float4 a, double k) {
  return make_float4((float)((double)a.x / k), (float)((double)a.y / k), (float)((double)a.z / k),
                     (float)((double)a.w / k));
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
  __shared__ uint32_t red[kWaves];
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
// wave-tile bodies (shared by the flat and the bucketed kernels)
//   lane l, instruction j in 0..3 of an int8 tile: elements 4*(j*64 + l) .. +3 (float4 j*64+l), whose
//   payload is dword j*64+l of the tile's 1 KiB; the LDS transpose hands lane l dwords 4l..4l+3.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void load_tile(const float4* __restrict__ x4, float4 (&v)[4], int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = load4<true>(x4 + j * 64 + lane);
}

template <bool ST_NT = false>
__device__ __forceinline__ void quantize_tile_regs(const float4 (&v)[4], uint4* __restrict__ q16, float inv,
                                                   uint32_t* __restrict__ lds, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) lds[j * 64 + lane] = quant4(v[j], inv);
  __builtin_amdgcn_wave_barrier();
  const uint4 o = reinterpret_cast<const uint4*>(lds)[lane];
  __builtin_amdgcn_wave_barrier();
  store16<ST_NT>(q16 + lane, o);
}

template <bool ST_NT = false>
__device__ __forceinline__ void quantize_tile(const float4* __restrict__ x4, uint4* __restrict__ q16, float inv,
                                              uint32_t* __restrict__ lds, int lane) {
  float4 v[4];
  load_tile(x4, v, lane);
  quantize_tile_regs<ST_NT>(v, q16, inv, lds, lane);
}

template <bool LD_NT = false>
__device__ __forceinline__ void dequantize_tile(const uint4* __restrict__ q16, float4* __restrict__ o4, float s,
                                                uint32_t* __restrict__ lds, int lane) {
  reinterpret_cast<uint4*>(lds)[lane] = load16<LD_NT>(q16 + lane);
  __builtin_amdgcn_wave_barrier();
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = lds[j * 64 + lane];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 4; ++j) store4_nt(o4 + j * 64 + lane, dequant4(w[j], s));
}

// ------------------------------------------------------------------------------------------------
// flat kernels (one tensor)
// ------------------------------------------------------------------------------------------------
template <int U, bool NT>
__device__ __forceinline__ uint32_t absmax_range(const float4* __restrict__ x4, int64_t b0, int64_t b1) {
  uint32_t m = 0;
  int64_t i = b0 + threadIdx.x;
  for (; i + (U - 1) * kBlock < b1; i += U * kBlock) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = load4<NT>(x4 + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) m = max(m, abs_bits4(v[u]));
  }
  for (; i < b1; i += kBlock) m = max(m, abs_bits4(load4<NT>(x4 + i)));
  return m;
}

// Pass 1: block b owns float4s [b*per, (b+1)*per). Blocks wholly before the last keep4 float4s read
// non-temporally; the rest with allocating loads (they stay in the Infinity Cache for pass 2). The
// product uses keep4 = 0 (kCacheKeepBytes): measured, the non-temporal read's speed-up outweighs what
// pass 2 gains from finding x's tail on-die (profiles/r01/microbench_keep_sweep.txt).
template <int U>
__global__ __launch_bounds__(kBlock) void k_absmax_flat(const float* __restrict__ x, int64_t n, int64_t keep4,
                                                        uint32_t* __restrict__ partials) {
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int64_t n4 = n >> 2;
  const int64_t per = ((n4 + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
  const int64_t b0 = (int64_t)blockIdx.x * per;
  const int64_t b1 = min(n4, b0 + per);
  uint32_t m = (b1 <= n4 - keep4) ? absmax_range<U, true>(x4, b0, b1) : absmax_range<U, false>(x4, b0, b1);
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) m = max(m, abs_bits(x[(n4 << 2) + threadIdx.x]));
  m = block_max(m);
  if (threadIdx.x == 0) partials[blockIdx.x] = m;
  if (blockIdx.x == 0 && threadIdx.x == 0) partials[kCountSlot] = gridDim.x;  // self-describing workspace
}

// Pass 2: tiles walked from the END of x, so decode (which walks forwards) starts on the payload bytes
// written last. Template knobs exist for tools/microbench.hip; the ABI uses <true, false>.
template <bool REVERSE, bool ST_NT>
__global__ __launch_bounds__(kBlock) void k_quantize_flat(const float* __restrict__ x, int64_t n, float qmax,
                                                          const uint32_t* __restrict__ partials,
                                                          int8_t* __restrict__ q, float* __restrict__ scale_out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][kTile / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint4* q16 = reinterpret_cast<uint4*>(q);
  const int64_t ntiles = n / kTile;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  int64_t t0 = (int64_t)blockIdx.x * kWaves + wave;
  // The first tile's loads do not need the scale: issue them before the partial reduction, whose
  // latency they then hide.
  float4 v[4];
  if (t0 < ntiles) load_tile(x4 + (REVERSE ? ntiles - 1 - t0 : t0) * (kTile / 4), v, lane);
  const ScaleInv si = make_scale(reduce_partials(partials, (int)partials[kCountSlot]), qmax);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = si.scale;
  for (; t0 < ntiles; t0 += wstride) {
    const int64_t t = REVERSE ? ntiles - 1 - t0 : t0;
    if (t0 != (int64_t)blockIdx.x * kWaves + wave) load_tile(x4 + t * (kTile / 4), v, lane);
    quantize_tile_regs<ST_NT>(v, q16 + t * (kTile / 16), si.inv, lds[wave], lane);
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile + threadIdx.x; i < n; i += kBlock) q[i] = (int8_t)quant1(x[i], si.inv);
}

// max|x| as a value (torch.max(torch.abs(t)), quant.py:100): pass 1's partials reduced by one block. The
// abs bit patterns order like the magnitudes, and a NaN's pattern exceeds +inf's, so NaN propagates.
__global__ __launch_bounds__(kBlock) void k_absmax_value(const uint32_t* __restrict__ partials,
                                                         float* __restrict__ out) {
  const uint32_t m = reduce_partials(partials, (int)partials[kCountSlot]);
  if (threadIdx.x == 0) *out = __uint_as_float(m);
}

// Decode: tiles walked forwards (pass 2 wrote the head of the payload last). ABI: <false, false>.
template <bool REVERSE, bool LD_NT>
__global__ __launch_bounds__(kBlock) void k_dequantize_flat(const int8_t* __restrict__ q, int64_t n,
                                                            const float* __restrict__ scale_p,
                                                            float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][kTile / 4];
  const float s = *scale_p;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* q16 = reinterpret_cast<const uint4*>(q);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ntiles = n / kTile;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  for (int64_t t0 = (int64_t)blockIdx.x * kWaves + wave; t0 < ntiles; t0 += wstride) {
    const int64_t t = REVERSE ? ntiles - 1 - t0 : t0;
    dequantize_tile<LD_NT>(q16 + t * (kTile / 16), o4 + t * (kTile / 4), s, lds[wave], lane);
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile + threadIdx.x; i < n; i += kBlock) out[i] = s * (float)q[i];
}

// int4 wave tile: 2048 elements = 8 coalesced 16-byte loads per lane -> 16 packed bytes per lane,
// transposed through 1 KiB of LDS (lane l, load j packs float4 j*64+l into halfword j*64+l).
__device__ __forceinline__ void load_tile_int4(const float4* __restrict__ xs, float4 (&v)[8], int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = load4<true>(xs + j * 64 + lane);
}

__device__ __forceinline__ void quantize_tile_int4_regs(const float4 (&v)[8], uint4* __restrict__ p16, float inv,
                                                        uint16_t* __restrict__ lds, int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) lds[j * 64 + lane] = (uint16_t)quant4_int4(v[j], inv);
  __builtin_amdgcn_wave_barrier();
  const uint4 o = reinterpret_cast<const uint4*>(lds)[lane];
  __builtin_amdgcn_wave_barrier();
  p16[lane] = o;
}

// int4 decode tile: one coalesced 16-byte load per lane, LDS transpose, 8 coalesced float4 NT stores.
__device__ __forceinline__ void dequantize_tile_int4(const uint4* __restrict__ p16, float4* __restrict__ o4, float s,
                                                     uint16_t* __restrict__ lds, int lane) {
  reinterpret_cast<uint4*>(lds)[lane] = p16[lane];
  __builtin_amdgcn_wave_barrier();
  uint32_t h[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = lds[j * 64 + lane];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 8; ++j) store4_nt(o4 + j * 64 + lane, dequant2_int4(h[j], s));
}

// int4 pass 2 (flat).
__global__ __launch_bounds__(kBlock) void k_quantize_int4_flat(const float* __restrict__ x, int64_t n, float qmax,
                                                               const uint32_t* __restrict__ partials,
                                                               uint8_t* __restrict__ packed,
                                                               float* __restrict__ scale_out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint4* p16 = reinterpret_cast<uint4*>(packed);
  const int64_t ntiles = n / kTile4;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  const int64_t first = (int64_t)blockIdx.x * kWaves + wave;
  // the first tile's loads do not need the scale: issued before the partial reduction they hide
  float4 v[8];
  if (first < ntiles) load_tile_int4(x4 + (ntiles - 1 - first) * (kTile4 / 4), v, lane);
  const ScaleInv si = make_scale(reduce_partials(partials, (int)partials[kCountSlot]), qmax);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = si.scale;
  for (int64_t t0 = first; t0 < ntiles; t0 += wstride) {
    const int64_t t = ntiles - 1 - t0;
    if (t0 != first) load_tile_int4(x4 + t * (kTile4 / 4), v, lane);
    quantize_tile_int4_regs(v, p16 + t * 64, si.inv, lds[wave], lane);
  }
  if (blockIdx.x == gridDim.x - 1) {
    const int64_t np = (n + 1) >> 1;
    for (int64_t j = ntiles * (kTile4 / 2) + threadIdx.x; j < np; j += kBlock) {
      const int hi = quant1(x[2 * j], si.inv);
      const int lo = (2 * j + 1 < n) ? quant1(x[2 * j + 1], si.inv) : 0;  // pad one zero (compression.py:42-43)
      packed[j] = (uint8_t)pack_pair(hi, lo);
    }
  }
}

// int4 decode (flat).
__global__ __launch_bounds__(kBlock) void k_dequantize_int4_flat(const uint8_t* __restrict__ packed, int64_t n,
                                                                 const float* __restrict__ scale_p,
                                                                 float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const float s = *scale_p;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* p16 = reinterpret_cast<const uint4*>(packed);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ntiles = n / kTile4;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < ntiles; t += wstride)
    dequantize_tile_int4(p16 + t * 64, o4 + t * (kTile4 / 4), s, lds[wave], lane);
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile4 + threadIdx.x; i < n; i += kBlock) {
      float e0, e1;
      dequant_byte_int4(packed[i >> 1], s, e0, e1);
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

// Peer-exchange epilogue / synchronous aggregate: mean of K dequantized rows in torch's summation order
// (torch_sum_order.h: the CPU sum(stack(rows), dim=0) that stack(...).mean(0) at ray_ad.py:188 and
// simple_aggregate at model.py:229-231 compute), then a correctly rounded division by K. The row sequence is
// rows r != self_row in r order, then (self_row >= 0) the rank's own fp32 update self_x, exactly, LAST
// (async_peer.py:170-174 / ray_ad.py:183-188 append the local parameters after the received updates).
// Vector tiles are SEQ-order columns of the one tensor (a tile ends below n & ~31); the < 1024 tail elements
// take each element's own order. Per row: one coalesced 16-byte load per lane + LDS transpose; output:
// coalesced NT float4 stores. DEEP: K >= 256 (the cascade's levels 2-3).
__device__ __forceinline__ int seq_row(int s, int self_row) { return (self_row >= 0 && s >= self_row) ? s + 1 : s; }

// Element e of the rows, summed in torch's order for tensor-relative index j of an n-element tensor.
template <class Dequant>
__device__ __forceinline__ float mean_elem_torch(const Dequant& dq, int k, int self_row,
                                                 const float* __restrict__ self_x, int64_t e, int64_t j, int64_t n,
                                                 double dk) {
  auto get = [&](int s) -> float {
    if (self_row >= 0 && s == k - 1) return self_x[e];
    return dq(seq_row(s, self_row), e);
  };
  return (float)((double)adfl_sum::sum_elem(get, k, adfl_sum::mode_of(j, n, k)) / dk);
}

template <bool DEEP>
__global__ __launch_bounds__(kBlock) void k_dequantize_mean(const int8_t* __restrict__ q, int64_t row_stride, int k,
                                                            int64_t n, const float* __restrict__ scales,
                                                            int64_t scale_stride, int self_row,
                                                            const float* __restrict__ self_x,
                                                            float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][kTile / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ntiles = n / kTile;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  const double dk = (double)k;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < ntiles; t += wstride) {
    adfl_sum::SeqTile<4, DEEP> acc;
    acc.init();
    for (int r = 0; r < k; ++r) {
      if (r == self_row) continue;
      const uint4* q16 = reinterpret_cast<const uint4*>(q + r * row_stride) + t * (kTile / 16);
      const float s = scales[r * scale_stride];
      reinterpret_cast<uint4*>(lds[wave])[lane] = q16[lane];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.add(j, dequant4(lds[wave][j * 64 + lane], s));
      __builtin_amdgcn_wave_barrier();
      acc.step();
    }
    if (self_row >= 0) {
      const float4* xs = reinterpret_cast<const float4*>(self_x) + t * (kTile / 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.add(j, xs[j * 64 + lane]);
      acc.step();
    }
    float4* o4 = reinterpret_cast<float4*>(out) + t * (kTile / 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) store4_nt(o4 + j * 64 + lane, div4(acc.result(j), dk));
  }
  if (blockIdx.x == gridDim.x - 1) {
    auto dq = [&](int r, int64_t e) -> float { return scales[r * scale_stride] * (float)q[r * row_stride + e]; };
    for (int64_t i = ntiles * kTile + threadIdx.x; i < n; i += kBlock)
      out[i] = mean_elem_torch(dq, k, self_row, self_x, i, i, n, dk);
  }
}

// Same over K int4-packed rows (2048-element wave tiles, 1 KiB of packed bytes per row per tile).
template <bool DEEP>
__global__ __launch_bounds__(kBlock) void k_dequantize_mean_int4(const uint8_t* __restrict__ p, int64_t row_stride,
                                                                 int k, int64_t n, const float* __restrict__ scales,
                                                                 int64_t scale_stride, int self_row,
                                                                 const float* __restrict__ self_x,
                                                                 float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ntiles = n / kTile4;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  const double dk = (double)k;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < ntiles; t += wstride) {
    adfl_sum::SeqTile<8, DEEP> acc;
    acc.init();
    for (int r = 0; r < k; ++r) {
      if (r == self_row) continue;
      const uint4* p16 = reinterpret_cast<const uint4*>(p + r * row_stride) + t * 64;
      const float s = scales[r * scale_stride];
      reinterpret_cast<uint4*>(lds[wave])[lane] = p16[lane];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.add(j, dequant2_int4(lds[wave][j * 64 + lane], s));
      __builtin_amdgcn_wave_barrier();
      acc.step();
    }
    if (self_row >= 0) {
      const float4* xs = reinterpret_cast<const float4*>(self_x) + t * (kTile4 / 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.add(j, xs[j * 64 + lane]);
      acc.step();
    }
    float4* o4 = reinterpret_cast<float4*>(out) + t * (kTile4 / 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) store4_nt(o4 + j * 64 + lane, div4(acc.result(j), dk));
  }
  if (blockIdx.x == gridDim.x - 1) {
    auto dq = [&](int r, int64_t e) -> float {
      float e0, e1;
      dequant_byte_int4(p[r * row_stride + (e >> 1)], scales[r * scale_stride], e0, e1);
      return (e & 1) ? e1 : e0;
    };
    for (int64_t i = ntiles * kTile4 + threadIdx.x; i < n; i += kBlock)
      out[i] = mean_elem_torch(dq, k, self_row, self_x, i, i, n, dk);
  }
}

// ------------------------------------------------------------------------------------------------
// bucketed kernels (many tensors, one block per chunk of <= 8192 elements = 8 wave tiles)
// ------------------------------------------------------------------------------------------------
// Chunks may start anywhere (a compact bucket packs tensors back to back): the first `head` elements
// up to the next `align`-element boundary are done element-wise, the rest in vector units.
__device__ __forceinline__ int chunk_head(int64_t start, int len, int align) {
  const int h = (int)((align - (start % align)) % align);
  return h < len ? h : len;
}

// A chunk (<= 8192 elements) is at most 2 wave tiles per wave + < 1024 tail elements + < 16 head
// elements: small enough to hold in VGPRs, so each pass issues ALL of a chunk's loads before the first
// use (8 x 16 B per lane in flight; a one-tile-at-a-time loop leaves a 32 KiB chunk latency-bound).
constexpr int kChunkTilesPerWave = ADFL_SLQ_CHUNK_ELEMS / kTile / kWaves;  // 2
constexpr int kChunkTailPerThread = kTile / kBlock;                        // < 1024 tail elements -> 4
static_assert(ADFL_SLQ_CHUNK_ELEMS % (kTile * kWaves) == 0, "chunk = whole tiles per wave");

struct ChunkRegs {
  float4 v[kChunkTilesPerWave][4];
  float tail[kChunkTailPerThread];
  float head;
};

// Load chunk c (x non-temporal: dead after this pass) into registers in the quantize tile layout.
__device__ __forceinline__ void chunk_load(const float* __restrict__ x, const adfl_slq_chunk& c, ChunkRegs& r,
                                           int lane, int wave) {
  const float* xc = x + c.start;
  const int head = chunk_head(c.start, c.len, 16);  // 16 elements: 64-B x and 16-B payload alignment
  const int ntiles = (c.len - head) / kTile;
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
#pragma unroll
  for (int k = 0; k < kChunkTilesPerWave; ++k) {
    const int t = wave + k * kWaves;
    if (t < ntiles) load_tile(x4 + t * (kTile / 4), r.v[k], lane);
  }
  r.head = (int)threadIdx.x < head ? xc[threadIdx.x] : 0.0f;
  const int t0 = head + ntiles * kTile;
#pragma unroll
  for (int k = 0; k < kChunkTailPerThread; ++k) {
    const int i = t0 + k * kBlock + (int)threadIdx.x;
    r.tail[k] = i < c.len ? __builtin_nontemporal_load(xc + i) : 0.0f;
  }
}

// Quantize the registers of chunk c into the payload (tiles through the wave's LDS transpose).
__device__ __forceinline__ void chunk_store(const adfl_slq_chunk& c, const ChunkRegs& r, float inv,
                                            int8_t* __restrict__ q, uint32_t* __restrict__ lds, int lane, int wave) {
  int8_t* qc = q + c.start;
  const int head = chunk_head(c.start, c.len, 16);
  const int ntiles = (c.len - head) / kTile;
  uint4* q16 = reinterpret_cast<uint4*>(qc + head);
#pragma unroll
  for (int k = 0; k < kChunkTilesPerWave; ++k) {
    const int t = wave + k * kWaves;
    if (t < ntiles) quantize_tile_regs(r.v[k], q16 + t * (kTile / 16), inv, lds, lane);
  }
  if ((int)threadIdx.x < head) qc[threadIdx.x] = (int8_t)quant1(r.head, inv);
  const int t0 = head + ntiles * kTile;
#pragma unroll
  for (int k = 0; k < kChunkTailPerThread; ++k) {
    const int i = t0 + k * kBlock + (int)threadIdx.x;
    if (i < c.len) qc[i] = (int8_t)quant1(r.tail[k], inv);
  }
}

// Pass 1: one partial per chunk, all of the chunk's loads in flight. Non-temporal: in the C3 config
// bench, allocating loads (x left in the Infinity Cache for pass 2) measured the same (A/B in
// profiles/r01/c3_absmax_policy.txt), and NT leaves the cache to the payload.
// chunk_base: the first chunk of the launch (adfl_slq_absmax_batched_range; 0 for the whole table).
__global__ __launch_bounds__(kBlock) void k_absmax_batched(const float* __restrict__ x,
                                                           const adfl_slq_chunk* __restrict__ chunks,
                                                           uint32_t* __restrict__ partials,
                                                           int64_t chunk_base = 0) {
  const int64_t ci = chunk_base + blockIdx.x;
  const adfl_slq_chunk c = chunks[ci];
  const float* xc = x + c.start;
  const int head = chunk_head(c.start, c.len, 4);
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
  const int n4 = (c.len - head) >> 2;
  constexpr int U = ADFL_SLQ_CHUNK_ELEMS / 4 / kBlock;  // 8 float4 per thread
  float4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int i = (int)threadIdx.x + k * kBlock;
    v[k] = i < n4 ? load4<true>(x4 + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  uint32_t m = 0;
  if (threadIdx.x < head) m = abs_bits(xc[threadIdx.x]);
  const int tail = head + (n4 << 2);
  if (threadIdx.x < c.len - tail) m = max(m, abs_bits(xc[tail + threadIdx.x]));
#pragma unroll
  for (int k = 0; k < U; ++k) m = max(m, abs_bits4(v[k]));
  m = block_max(m);
  if (threadIdx.x == 0) partials[ci] = m;
}

// Pass 2: the chunk's loads are issued before the partial reduction, whose latency they hide.
// chunk_base: the first chunk of the launch (adfl_slq_quantize_batched_range; 0 for the whole table).
__global__ __launch_bounds__(kBlock) void k_quantize_batched(const float* __restrict__ x,
                                                             const adfl_slq_chunk* __restrict__ chunks,
                                                             float qmax, const uint32_t* __restrict__ partials,
                                                             int8_t* __restrict__ q, float* __restrict__ scales,
                                                             int64_t chunk_base = 0) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][kTile / 4];
  const int64_t ci = chunk_base + blockIdx.x;
  const adfl_slq_chunk c = chunks[ci];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  ChunkRegs r;
  chunk_load(x, c, r, lane, wave);
  const ScaleInv si = make_scale(reduce_partials(partials + c.first_chunk, c.nchunks), qmax);
  if (ci == c.first_chunk && threadIdx.x == 0) scales[c.tensor] = si.scale;
  chunk_store(c, r, si.inv, q, lds[wave], lane, wave);
}

// A one-launch encode for tensors of any size (chunk blocks meeting per tensor in a cooperative launch) was
// measured in round 2 and removed in round 3: the cooperative launch cost ~20 us more than an ordinary
// one on C3 (log-uniform 43 vs 24.7 us two-pass; equal 38 vs 17 us resident; profiles/r02/coop/).


// ---- one-launch encode of a bucket of small tensors (a whole tensor per block, x read once) -------
// A tensor of up to kSegChunks chunks (<= 65536 elements) fits the VGPRs of one 1024-thread block
// (16 waves x 4 wave tiles x 4 float4 per lane = 64 VGPRs). When EVERY tensor of the bucket does, the
// encode is one launch: each block loads its whole tensor, reduces max|x| in-block, forms the scale and
// quantizes from registers — no cross-block dependency, no second pass, x read once (5 B/element
// instead of 9). C3's 256 x 45,662 layout: encode 22.8 -> 16.4 us, round trip 0.63 -> 0.78 of 8 TB/s
// with the Infinity Cache flushed (profiles/r02/microbench_c3.txt).
// Blocks walk a host-built work list (adfl_slq_build_encode_work: the first chunk of every tensor), so no
// block is launched only to exit: a 1024-thread block takes a whole CU's wave slots, and idle ones queued
// behind the working blocks (27.6 us with the chunk table as the grid).
// With any larger tensor the two-pass encode runs instead: big blocks pay off only while there are about
// as many of them as CUs, and segmenting the large tensors (one absmax per 65,536-element segment, then
// a segment quantize launch) measured slower than the two passes (log-uniform layout: 28.4 vs 23.9 us).
constexpr int kSegBlock = 1024;
constexpr int kSegWaves = kSegBlock / 64;
constexpr int kSegTilesPerWave = 4;
constexpr int64_t kSegMaxElems = (int64_t)kSegWaves * kSegTilesPerWave * kTile;  // 65536
constexpr int kSegChunks = (int)(kSegMaxElems / ADFL_SLQ_CHUNK_ELEMS);            // 8
static_assert(kSegChunks == ADFL_SLQ_RESIDENT_CHUNKS, "header constant");
static_assert(kSegMaxElems % ADFL_SLQ_CHUNK_ELEMS == 0, "segment = whole chunks");
static_assert(kSegBlock == kTile, "tail: one element per thread");

__device__ __forceinline__ uint32_t block_max_seg(uint32_t v) {
  __shared__ uint32_t red[kSegWaves];
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t m = red[0];
#pragma unroll
  for (int w = 1; w < kSegWaves; ++w) m = max(m, red[w]);
  return m;
}

// work[b] = the first chunk of tensor b (every tensor <= kSegChunks chunks).
// ST_NT: non-temporal payload stores. The block's stores are the tail of a launch in which every CU loads,
// reduces and stores in lockstep (tools/microbench_resident_timeline.hip: entry spread 0.6 us, block max
// at 8.5 us, stores acknowledged at 11.5-12 us); streaming them past the L2 shortens the encode (15.7 vs
// 16.6 us, profiles/r03/c3_resident/timeline.txt) but the decode that follows then reads the payload from
// HBM: C3 round trip 30.3 vs 27.0 us (profiles/r03/c3_resident/c3_nt_stores.json). kResidentNtStores = false.
template <bool ST_NT>
__global__ __launch_bounds__(kSegBlock) void k_encode_resident(const float* __restrict__ x,
                                                               const adfl_slq_chunk* __restrict__ chunks,
                                                               const int32_t* __restrict__ work, float qmax,
                                                               int8_t* __restrict__ q, float* __restrict__ scales) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kSegWaves][kTile / 4];
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk c = chunks[ci];
  if (c.nchunks > kSegChunks) {  // not a resident work list (a direct C caller's): NaN scale, nothing written
    if (threadIdx.x == 0) scales[c.tensor] = __builtin_nanf("");
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int len = (c.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + c.nchunks - 1].len;
  const float* xt = x + c.start;
  // all of the tensor's loads in flight at once (x non-temporal: dead after this pass)
  const int head = chunk_head(c.start, len, 16);
  const int ntiles = (len - head) / kTile;
  const float4* x4 = reinterpret_cast<const float4*>(xt + head);
  float4 v[kSegTilesPerWave][4];
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles) {
      load_tile(x4 + t * (kTile / 4), v[k], lane);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[k][j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float hv = (int)threadIdx.x < head ? xt[threadIdx.x] : 0.0f;
  const int ti = head + ntiles * kTile + (int)threadIdx.x;  // < 1024 tail elements: one per thread
  const float tv = ti < len ? __builtin_nontemporal_load(xt + ti) : 0.0f;
  uint32_t m = max(abs_bits(hv), abs_bits(tv));
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) m = max(m, abs_bits4(v[k][j]));
  const ScaleInv si = make_scale(block_max_seg(m), qmax);
  if (threadIdx.x == 0) scales[c.tensor] = si.scale;
  int8_t* qt = q + c.start;
  uint4* q16 = reinterpret_cast<uint4*>(qt + head);
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles) quantize_tile_regs<ST_NT>(v[k], q16 + t * (kTile / 16), si.inv, lds[wave], lane);
  }
  if ((int)threadIdx.x < head) qt[threadIdx.x] = (int8_t)quant1(hv, si.inv);
  if (ti < len) qt[ti] = (int8_t)quant1(tv, si.inv);
}
constexpr bool kResidentNtStores = false;

// int4 variant (PackedSLQChannel's buckets: even tensor offsets, packed byte e/2 = flat elements e, e+1):
// 2048-element int4 wave tiles, 2 per wave (16 float4 per lane); the < 32-element head and the < 2048-
// element tail go pairwise, one pair per thread, an odd tensor's last element paired with pack_4bit's
// zero pad (compression.py:42-43).
constexpr int kSegTiles4PerWave = (int)(kSegMaxElems / kTile4 / kSegWaves);  // 2
static_assert(kSegTiles4PerWave * kTile4 * kSegWaves == kSegMaxElems, "int4 tiles cover a segment");
static_assert(2 * kSegBlock == kTile4, "int4 tail: one pair per thread");

__global__ __launch_bounds__(kSegBlock) void k_encode_resident_int4(const float* __restrict__ x,
                                                                    const adfl_slq_chunk* __restrict__ chunks,
                                                                    const int32_t* __restrict__ work, float qmax,
                                                                    uint8_t* __restrict__ packed,
                                                                    float* __restrict__ scales) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kSegWaves][kTile4 / 4];
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk c = chunks[ci];
  if (c.nchunks > kSegChunks) {  // not a resident work list (a direct C caller's): NaN scale, nothing written
    if (threadIdx.x == 0) scales[c.tensor] = __builtin_nanf("");
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int len = (c.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + c.nchunks - 1].len;
  const float* xt = x + c.start;
  const int head = chunk_head(c.start, len, 32);  // even: tensor offsets are even
  const int ntiles = (len - head) / kTile4;
  const float4* x4 = reinterpret_cast<const float4*>(xt + head);
  float4 v[kSegTiles4PerWave][8];
#pragma unroll
  for (int k = 0; k < kSegTiles4PerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles) {
      load_tile_int4(x4 + t * (kTile4 / 4), v[k], lane);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // head pair (element 2*tid of [0, head)) and tail pair (t0 + 2*tid of [t0, len))
  const int hi = 2 * (int)threadIdx.x;
  const bool has_h = hi < head;
  const float h0 = has_h ? xt[hi] : 0.0f, h1 = (has_h && hi + 1 < len) ? xt[hi + 1] : 0.0f;
  const int ti = head + ntiles * kTile4 + 2 * (int)threadIdx.x;
  const bool has_t = ti < len;
  const float t0v = has_t ? __builtin_nontemporal_load(xt + ti) : 0.0f;
  const float t1v = (has_t && ti + 1 < len) ? __builtin_nontemporal_load(xt + ti + 1) : 0.0f;
  uint32_t m = max(max(abs_bits(h0), abs_bits(h1)), max(abs_bits(t0v), abs_bits(t1v)));
#pragma unroll
  for (int k = 0; k < kSegTiles4PerWave; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) m = max(m, abs_bits4(v[k][j]));
  const ScaleInv si = make_scale(block_max_seg(m), qmax);
  if (threadIdx.x == 0) scales[c.tensor] = si.scale;
  uint8_t* pt = packed + (c.start >> 1);
#pragma unroll
  for (int k = 0; k < kSegTiles4PerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles)
      quantize_tile_int4_regs(v[k], reinterpret_cast<uint4*>(pt + (head >> 1)) + t * 64, si.inv, lds[wave], lane);
  }
  // the pad of an odd tensor's last pair is a zero CODE (compression.py:42-43), not quant1(0)
  if (has_h) pt[hi >> 1] = (uint8_t)pack_pair(quant1(h0, si.inv), hi + 1 < len ? quant1(h1, si.inv) : 0);
  if (has_t) pt[ti >> 1] = (uint8_t)pack_pair(quant1(t0v, si.inv), ti + 1 < len ? quant1(t1v, si.inv) : 0);
}

__global__ __launch_bounds__(kBlock) void k_dequantize_batched(const int8_t* __restrict__ q,
                                                               const adfl_slq_chunk* __restrict__ chunks,
                                                               const float* __restrict__ scales,
                                                               float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][kTile / 4];
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float s = scales[c.tensor];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int8_t* qc = q + c.start;
  float* oc = out + c.start;
  const int head = chunk_head(c.start, c.len, 16);
  if (threadIdx.x < head) oc[threadIdx.x] = s * (float)qc[threadIdx.x];
  const int ntiles = (c.len - head) / kTile;
  for (int t = wave; t < ntiles; t += kWaves)
    dequantize_tile(reinterpret_cast<const uint4*>(qc + head) + t * (kTile / 16),
                    reinterpret_cast<float4*>(oc + head) + t * (kTile / 4), s, lds[wave], lane);
  for (int i = head + ntiles * kTile + threadIdx.x; i < c.len; i += kBlock) oc[i] = s * (float)qc[i];
}

// Peer mean of K bucketed payloads with per-tensor scales — the decentralized exchange of a whole state dict
// under SLQChannel's per-tensor codec (ray_ad.py:164-190 averaging every tensor; quant.py:74-94 giving each
// tensor its own scale), and SLQChannel.receive_mean (simple_aggregate over K decoded dicts, model.py:221-234):
// for tensor t and element i of the bucket, the torch-order sum (torch_sum_order.h, per tensor: the column
// index is i's offset in its tensor) of fp32(scale_r[t] * q_r[i]) over the row sequence (rows != self_row in
// r order, then self_x[i]), then / K correctly rounded — k_dequantize_mean's arithmetic per tensor. Row r's
// payload is q + r * row_stride (one bucket payload each, the same layout), its scales
// scales + r * scale_stride. One block per chunk: wave tiles over the chunk's SEQ columns (16-element aligned
// in the bucket), the < 16 head elements and everything past the tiles element-wise in each one's order.
struct TensorSpan {
  int64_t start, n;  // the chunk's tensor: bucket offset and element count
};
__device__ __forceinline__ TensorSpan tensor_span(const adfl_slq_chunk* __restrict__ chunks, const adfl_slq_chunk& c) {
  TensorSpan t;
  t.start = chunks[c.first_chunk].start;
  t.n = (int64_t)(c.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[c.first_chunk + c.nchunks - 1].len;
  return t;
}

// wave tiles of `tile` elements the chunk can take: from `head` up to the tensor's last SEQ column
__device__ __forceinline__ int seq_tiles(const adfl_slq_chunk& c, const TensorSpan& ts, int head, int tile) {
  int64_t lim = ts.start + adfl_sum::seq_end(ts.n) - c.start;  // chunk-relative end of the SEQ columns
  lim = lim < c.len ? lim : c.len;
  return lim > head ? (int)((lim - head) / tile) : 0;
}

template <bool DEEP>
__global__ __launch_bounds__(kBlock) void k_dequantize_mean_batched(const int8_t* __restrict__ q, int64_t row_stride,
                                                                    int k, const adfl_slq_chunk* __restrict__ chunks,
                                                                    const float* __restrict__ scales,
                                                                    int64_t scale_stride, int self_row,
                                                                    const float* __restrict__ self_x,
                                                                    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][kTile / 4];
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const TensorSpan ts = tensor_span(chunks, c);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double dk = (double)k;
  const int head = chunk_head(c.start, c.len, 16);
  const int ntiles = seq_tiles(c, ts, head, kTile);
  auto dq = [&](int r, int64_t e) -> float {
    return scales[r * scale_stride + c.tensor] * (float)q[r * row_stride + e];
  };
  if ((int)threadIdx.x < head) {
    const int64_t e = c.start + threadIdx.x;
    out[e] = mean_elem_torch(dq, k, self_row, self_x, e, e - ts.start, ts.n, dk);
  }
  for (int t = wave; t < ntiles; t += kWaves) {
    const int64_t base = c.start + head + (int64_t)t * kTile;  // 16-element aligned
    adfl_sum::SeqTile<4, DEEP> acc;
    acc.init();
    for (int r = 0; r < k; ++r) {
      if (r == self_row) continue;
      const uint4* q16 = reinterpret_cast<const uint4*>(q + r * row_stride + base);
      const float s = scales[r * scale_stride + c.tensor];
      reinterpret_cast<uint4*>(lds[wave])[lane] = q16[lane];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.add(j, dequant4(lds[wave][j * 64 + lane], s));
      __builtin_amdgcn_wave_barrier();
      acc.step();
    }
    if (self_row >= 0) {
      const float4* xs = reinterpret_cast<const float4*>(self_x + base);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.add(j, xs[j * 64 + lane]);
      acc.step();
    }
    float4* o4 = reinterpret_cast<float4*>(out + base);
#pragma unroll
    for (int j = 0; j < 4; ++j) store4_nt(o4 + j * 64 + lane, div4(acc.result(j), dk));
  }
  for (int i = head + ntiles * kTile + threadIdx.x; i < c.len; i += kBlock) {
    const int64_t e = c.start + i;
    out[e] = mean_elem_torch(dq, k, self_row, self_x, e, e - ts.start, ts.n, dk);
  }
}

// The same mean over K int4-packed bucket payloads (PackedSLQChannel per tensor; encode_batched_int4's
// layout: even tensor offsets, flat element e in byte e/2, high nibble for even e). Heads run to a 32-element
// (16-byte) boundary, wave tiles are kTile4 = 2048 elements = 1 KiB of packed bytes per row.
template <bool DEEP>
__global__ __launch_bounds__(kBlock) void k_dequantize_mean_batched_int4(
    const uint8_t* __restrict__ p, int64_t row_stride, int k, const adfl_slq_chunk* __restrict__ chunks,
    const float* __restrict__ scales, int64_t scale_stride, int self_row, const float* __restrict__ self_x,
    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const TensorSpan ts = tensor_span(chunks, c);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double dk = (double)k;
  const int head = chunk_head(c.start, c.len, 32);
  const int ntiles = seq_tiles(c, ts, head, kTile4);
  auto dq = [&](int r, int64_t e) -> float {
    float e0, e1;
    dequant_byte_int4(p[r * row_stride + (e >> 1)], scales[r * scale_stride + c.tensor], e0, e1);
    return (e & 1) ? e1 : e0;
  };
  if ((int)threadIdx.x < head) {
    const int64_t e = c.start + threadIdx.x;
    out[e] = mean_elem_torch(dq, k, self_row, self_x, e, e - ts.start, ts.n, dk);
  }
  for (int t = wave; t < ntiles; t += kWaves) {
    const int64_t base = c.start + head + (int64_t)t * kTile4;  // 32-element aligned
    adfl_sum::SeqTile<8, DEEP> acc;
    acc.init();
    for (int r = 0; r < k; ++r) {
      if (r == self_row) continue;
      const uint4* p16 = reinterpret_cast<const uint4*>(p + r * row_stride + (base >> 1));
      const float s = scales[r * scale_stride + c.tensor];
      reinterpret_cast<uint4*>(lds[wave])[lane] = p16[lane];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.add(j, dequant2_int4(lds[wave][j * 64 + lane], s));
      __builtin_amdgcn_wave_barrier();
      acc.step();
    }
    if (self_row >= 0) {
      const float4* xs = reinterpret_cast<const float4*>(self_x + base);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc.add(j, xs[j * 64 + lane]);
      acc.step();
    }
    float4* o4 = reinterpret_cast<float4*>(out + base);
#pragma unroll
    for (int j = 0; j < 8; ++j) store4_nt(o4 + j * 64 + lane, div4(acc.result(j), dk));
  }
  for (int i = head + ntiles * kTile4 + threadIdx.x; i < c.len; i += kBlock) {
    const int64_t e = c.start + i;
    out[e] = mean_elem_torch(dq, k, self_row, self_x, e, e - ts.start, ts.n, dk);
  }
}

// Decode + accumulate into K models (pool.py:62-75, qafel.py:176-179 via model.py:337-347): the chunk's
// payload is decoded once into registers (8 float4 per thread), then every model's slice is read, added
// (fp32(a + d), what mul_(1).add_(d, alpha=1) computes) and written back with 16-byte accesses when the
// tensor's offset in the bucket is a multiple of 4 (the payload dwords and the targets' float4s line up).
// Any other offset (a compact bucket) takes an element-wise path with the same sums: every chunk of a
// tensor shares its offset's residue mod 4, so the branch is block-uniform.
__global__ __launch_bounds__(kBlock) void k_dequantize_add_batched(const int8_t* __restrict__ q,
                                                                   const adfl_slq_chunk* __restrict__ chunks,
                                                                   const float* __restrict__ scales,
                                                                   float* const* __restrict__ targets,
                                                                   int ntensors, int ntargets) {
  constexpr int kPer = ADFL_SLQ_CHUNK_ELEMS / 4 / kBlock;
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float s = scales[c.tensor];
  const int64_t in_tensor = (int64_t)(blockIdx.x - c.first_chunk) * ADFL_SLQ_CHUNK_ELEMS;
  const int8_t* qc = q + c.start;
  if (c.start & 3) {
    for (int m = 0; m < ntargets; ++m) {
      float* tg = targets[(int64_t)m * ntensors + c.tensor] + in_tensor;
      for (int i = threadIdx.x; i < c.len; i += kBlock) tg[i] = tg[i] + s * (float)qc[i];
    }
    return;
  }
  const uint32_t* q4 = reinterpret_cast<const uint32_t*>(qc);
  const int n4 = c.len >> 2;
  float4 dv[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = threadIdx.x + j * kBlock;
    dv[j] = k < n4 ? dequant4(q4[k], s) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int tail = n4 << 2;
  const bool has_tail = (int)threadIdx.x < c.len - tail;
  const float dt = has_tail ? s * (float)qc[tail + threadIdx.x] : 0.0f;
  for (int m = 0; m < ntargets; ++m) {
    float* tg = targets[(int64_t)m * ntensors + c.tensor] + in_tensor;
    float4* t4 = reinterpret_cast<float4*>(tg);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int k = threadIdx.x + j * kBlock;
      if (k < n4) t4[k] = add4(t4[k], dv[j]);
    }
    if (has_tail) tg[tail + threadIdx.x] = tg[tail + threadIdx.x] + dt;
  }
}

// Quantization-error statistics of a bucket against its own payload (worker.py:186-189 computes
// parameter_relative_mse and parameter_cosine_similarity from a full decode; here they are four sums
// per chunk, fp64): S0 = sum (x - s*q)^2, S1 = sum x^2, S2 = sum x*(s*q), S3 = sum (s*q)^2.
// PACKED: q is an int4 bucket (pack_4bit layout, even tensor offsets): element e's code is the high
// (even e) or low (odd e) nibble of byte e/2, minus 8 — what unpack_4bit hands the dequantize.
template <bool PACKED>
__global__ __launch_bounds__(kBlock) void k_qerror_batched(const float* __restrict__ x, const int8_t* __restrict__ q,
                                                           const adfl_slq_chunk* __restrict__ chunks,
                                                           const float* __restrict__ scales,
                                                           double* __restrict__ partials) {
  __shared__ double red[4][kWaves];
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float s = scales[c.tensor];
  const float* xc = x + c.start;
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  for (int i = threadIdx.x; i < c.len; i += kBlock) {
    const double xv = xc[i];
    int code;
    if (PACKED) {
      const int64_t e = c.start + i;
      const uint32_t b = reinterpret_cast<const uint8_t*>(q)[e >> 1];
      code = (e & 1) ? (int)(b & 0xfu) - 8 : (int)((b >> 4) & 0xfu) - 8;
    } else {
      code = q[c.start + i];
    }
    const double dv = (double)(s * (float)code);  // the dequantized fp32 value the reference compares
    const double e = (double)(xc[i] - (float)dv);  // fp32 difference, as (a - b) in parameter_mse
    a0 += e * e;
    a1 += xv * xv;
    a2 += xv * dv;
    a3 += dv * dv;
  }
  double v[4] = {a0, a1, a2, a3};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double t = 0;
    for (int w = 0; w < kWaves; ++w) t += red[threadIdx.x][w];
    partials[4 * (int64_t)blockIdx.x + threadIdx.x] = t;
  }
}

// int4 buckets: every tensor offset is even, so flat element e's nibble lives in packed byte e/2 (high
// nibble = even element) and an odd-sized tensor's last byte pairs its last element with a zero pad
// (compression.py:42-43). Vector tiles need 32-element alignment (16-B packed, 64-B x).
__device__ __forceinline__ void quantize_pairs_int4(const float* __restrict__ xc, uint8_t* __restrict__ pc, int a,
                                                    int b, int len, float inv) {
  for (int i = a + 2 * (int)threadIdx.x; i < b; i += 2 * kBlock) {
    const int hi = quant1(xc[i], inv);
    const int lo = (i + 1 < len) ? quant1(xc[i + 1], inv) : 0;
    pc[i >> 1] = (uint8_t)pack_pair(hi, lo);
  }
}

__device__ __forceinline__ void dequantize_elems_int4(const uint8_t* __restrict__ pc, float* __restrict__ oc, int a,
                                                      int b, float s) {
  for (int i = a + (int)threadIdx.x; i < b; i += kBlock) {
    float e0, e1;
    dequant_byte_int4(pc[i >> 1], s, e0, e1);
    oc[i] = (i & 1) ? e1 : e0;
  }
}

__global__ __launch_bounds__(kBlock) void k_quantize_batched_int4(const float* __restrict__ x,
                                                                  const adfl_slq_chunk* __restrict__ chunks,
                                                                  int64_t nchunks, float qmax,
                                                                  const uint32_t* __restrict__ partials,
                                                                  uint8_t* __restrict__ packed,
                                                                  float* __restrict__ scales) {
  static_assert(ADFL_SLQ_CHUNK_ELEMS == kTile4 * kWaves, "one int4 tile per wave per chunk");
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const int64_t ci = nchunks - 1 - (int64_t)blockIdx.x;
  const adfl_slq_chunk c = chunks[ci];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* xc = x + c.start;
  uint8_t* pc = packed + (c.start >> 1);
  const int head = chunk_head(c.start, c.len, 32);
  const int ntiles = (c.len - head) / kTile4;
  // the wave's tile is loaded before the partial reduction, whose latency it hides
  float4 v[8];
  if (wave < ntiles) load_tile_int4(reinterpret_cast<const float4*>(xc + head) + wave * (kTile4 / 4), v, lane);
  const ScaleInv si = make_scale(reduce_partials(partials + c.first_chunk, c.nchunks), qmax);
  if (ci == c.first_chunk && threadIdx.x == 0) scales[c.tensor] = si.scale;
  quantize_pairs_int4(xc, pc, 0, head, c.len, si.inv);
  if (wave < ntiles)
    quantize_tile_int4_regs(v, reinterpret_cast<uint4*>(pc + (head >> 1)) + wave * 64, si.inv, lds[wave], lane);
  quantize_pairs_int4(xc, pc, head + ntiles * kTile4, c.len, c.len, si.inv);
}

__global__ __launch_bounds__(kBlock) void k_dequantize_batched_int4(const uint8_t* __restrict__ packed,
                                                                    const adfl_slq_chunk* __restrict__ chunks,
                                                                    const float* __restrict__ scales,
                                                                    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float s = scales[c.tensor];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint8_t* pc = packed + (c.start >> 1);
  float* oc = out + c.start;
  const int head = chunk_head(c.start, c.len, 32);
  dequantize_elems_int4(pc, oc, 0, head, s);
  const int ntiles = (c.len - head) / kTile4;
  for (int t = wave; t < ntiles; t += kWaves)
    dequantize_tile_int4(reinterpret_cast<const uint4*>(pc + (head >> 1)) + t * 64,
                         reinterpret_cast<float4*>(oc + head) + t * (kTile4 / 4), s, lds[wave], lane);
  dequantize_elems_int4(pc, oc, head + ntiles * kTile4, c.len, s);
}

// ------------------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------------------
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int clamp_grid(int64_t g, int cap) { return (int)(g < 1 ? 1 : (g > cap ? cap : g)); }

// grid for a wave-tile kernel over `tiles` tiles (4 tiles per block per sweep)
inline int tile_grid(int64_t tiles) { return clamp_grid((tiles + kWaves - 1) / kWaves, kMaxFlatBlocks); }

inline int absmax_grid(int64_t n) { return clamp_grid((n >> 2) / (8 * kBlock), kAbsmaxBlocks); }

inline int check_bits(int bits) { return (bits >= 1 && bits <= 16) ? ADFL_OK : ADFL_E_BITS; }

// mean kernels: K rows from which the cascade needs its levels 2-3 (torch_sum_order.h), and the most rows
constexpr int kDeepRows = 256;
inline bool bad_rows(int k) { return k < 1 || k > adfl_sum::kMaxRows; }

// q_max as the fp32 value torch divides by (quant.py:99-100).
inline float qmax_f(int bits) { return (float)((1LL << (bits - 1)) - 1); }

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ADFL_OK : (int)e;
}

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
  hipLaunchKernelGGL(k_absmax_flat<8>, dim3(absmax_grid(n)), dim3(kBlock), 0, (hipStream_t)stream, d_x, n,
                     (int64_t)(kCacheKeepBytes / 16), (uint32_t*)d_workspace);
  return launch_status();
}

int adfl_slq_absmax_value(const void* d_workspace, float* d_absmax, void* stream) {
  if (!d_workspace || !d_absmax) return ADFL_E_ARG;
  if (!aligned16(d_workspace)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_absmax_value, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, (const uint32_t*)d_workspace,
                     d_absmax);
  return launch_status();
}

int adfl_slq_quantize(const float* d_x, int64_t n, int bits, const void* d_workspace, int8_t* d_q, float* d_scale,
                      void* stream) {
  if (!d_x || !d_workspace || !d_q || !d_scale || n < 1) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_q)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL((k_quantize_flat<true, false>), dim3(tile_grid(n / kTile)), dim3(kBlock), 0, (hipStream_t)stream, d_x, n,
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
  hipLaunchKernelGGL((k_dequantize_flat<false, false>), dim3(tile_grid(n / kTile)), dim3(kBlock), 0, (hipStream_t)stream, d_q, n,
                     d_scale, d_out);
  return launch_status();
}

int64_t adfl_slq_build_chunks(const int64_t* offsets, const int64_t* sizes, int32_t ntensors, adfl_slq_chunk* chunks,
                              int64_t capacity) {
  if (!offsets || !sizes || ntensors < 1) return ADFL_E_ARG;
  int64_t count = 0;
  for (int32_t t = 0; t < ntensors; ++t) {
    if (sizes[t] < 1 || offsets[t] < 0) return ADFL_E_ARG;
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
  hipLaunchKernelGGL(k_quantize_batched, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, qmax_f(bits),
                     (const uint32_t*)d_partials, d_q, d_scales, (int64_t)0);
  return launch_status();
}

int adfl_slq_quantize_batched_range(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t chunk_begin,
                                    int64_t count, int bits, const uint32_t* d_partials, int8_t* d_q,
                                    float* d_scales, void* stream) {
  if (!d_x || !d_chunks || !d_q || !d_scales || !d_partials || chunk_begin < 0 || count < 1 || count > INT32_MAX)
    return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_q)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_quantize_batched, dim3((unsigned)count), dim3(kBlock), 0, (hipStream_t)stream, d_x, d_chunks,
                     qmax_f(bits), d_partials, d_q, d_scales, chunk_begin);
  return launch_status();
}

int adfl_slq_absmax_batched_range(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t chunk_begin, int64_t count,
                                  uint32_t* d_partials, void* stream) {
  if (!d_x || !d_chunks || !d_partials || chunk_begin < 0 || count < 1 || count > INT32_MAX) return ADFL_E_ARG;
  if (!aligned16(d_x)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_absmax_batched, dim3((unsigned)count), dim3(kBlock), 0, (hipStream_t)stream, d_x, d_chunks,
                     d_partials, chunk_begin);
  return launch_status();
}

int64_t adfl_slq_build_encode_work(const adfl_slq_chunk* chunks, int64_t nchunks, int32_t* work, int64_t capacity) {
  if (!chunks || nchunks < 1 || nchunks > INT32_MAX) return ADFL_E_ARG;
  int64_t n = 0;
  for (int64_t i = 0; i < nchunks; ++i) {
    const adfl_slq_chunk& c = chunks[i];
    if (c.first_chunk < 0 || c.nchunks < 1 || i < c.first_chunk || i >= (int64_t)c.first_chunk + c.nchunks)
      return ADFL_E_ARG;
    if (c.nchunks > kSegChunks) return 0;  // a tensor too large for one block: the two-pass encode
    if (i != c.first_chunk) continue;
    if (work) {
      if (n >= capacity) return ADFL_E_ARG;
      work[n] = (int32_t)i;
    }
    ++n;
  }
  return n;
}

int adfl_slq_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                 const int32_t* d_work, int64_t nwork, int bits, int8_t* d_q, float* d_scales,
                                 uint32_t* d_partials, void* stream) {
  if (nwork == 0) return adfl_slq_encode_batched(d_x, d_chunks, nchunks, bits, d_q, d_scales, d_partials, stream);
  if (!d_x || !d_chunks || !d_work || !d_q || !d_scales || nchunks < 1 || nchunks > INT32_MAX || nwork < 0 ||
      nwork > nchunks)
    return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_q)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_encode_resident<kResidentNtStores>, dim3((unsigned)nwork), dim3(kSegBlock), 0, (hipStream_t)stream, d_x,
                     d_chunks, d_work, qmax_f(bits), d_q, d_scales);
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

int adfl_slq_qerror_batched(const float* d_x, const int8_t* d_q, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                            const float* d_scales, double* d_partials, void* stream) {
  if (!d_x || !d_q || !d_chunks || !d_scales || !d_partials || nchunks < 1 || nchunks > INT32_MAX) return ADFL_E_ARG;
  hipLaunchKernelGGL(k_qerror_batched<false>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_x,
                     d_q, d_chunks, d_scales, d_partials);
  return launch_status();
}

int adfl_slq_qerror_batched_int4(const float* d_x, const uint8_t* d_packed, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, const float* d_scales, double* d_partials, void* stream) {
  if (!d_x || !d_packed || !d_chunks || !d_scales || !d_partials || nchunks < 1 || nchunks > INT32_MAX)
    return ADFL_E_ARG;
  hipLaunchKernelGGL(k_qerror_batched<true>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_x,
                     (const int8_t*)d_packed, d_chunks, d_scales, d_partials);
  return launch_status();
}

int adfl_slq_encode_batched_int4(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                                 uint8_t* d_packed, float* d_scales, uint32_t* d_partials, void* stream) {
  if (!d_x || !d_chunks || !d_packed || !d_scales || !d_partials || nchunks < 1 || nchunks > INT32_MAX)
    return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_packed)) return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_absmax_batched, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, d_partials);
  if (int s = launch_status()) return s;
  hipLaunchKernelGGL(k_quantize_batched_int4, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, nchunks,
                     qmax_f(bits), (const uint32_t*)d_partials, d_packed, d_scales);
  return launch_status();
}

int adfl_slq_encode_batched_int4_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                      const int32_t* d_work, int64_t nwork, int bits, uint8_t* d_packed,
                                      float* d_scales, uint32_t* d_partials, void* stream) {
  if (nwork == 0)
    return adfl_slq_encode_batched_int4(d_x, d_chunks, nchunks, bits, d_packed, d_scales, d_partials, stream);
  if (!d_x || !d_chunks || !d_work || !d_packed || !d_scales || nchunks < 1 || nchunks > INT32_MAX || nwork < 0 ||
      nwork > nchunks)
    return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_packed)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_encode_resident_int4, dim3((unsigned)nwork), dim3(kSegBlock), 0, (hipStream_t)stream, d_x,
                     d_chunks, d_work, qmax_f(bits), d_packed, d_scales);
  return launch_status();
}

int adfl_slq_dequantize_batched_int4(const uint8_t* d_packed, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                     const float* d_scales, float* d_out, void* stream) {
  if (!d_packed || !d_chunks || !d_scales || !d_out || nchunks < 1 || nchunks > INT32_MAX) return ADFL_E_ARG;
  if (!aligned16(d_packed) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_batched_int4, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream,
                     d_packed, d_chunks, d_scales, d_out);
  return launch_status();
}

int adfl_slq_quantize_int4(const float* d_x, int64_t n, int bits, const void* d_workspace, uint8_t* d_packed,
                           float* d_scale, void* stream) {
  if (!d_x || !d_workspace || !d_packed || !d_scale || n < 1) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_packed)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_quantize_int4_flat, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, (hipStream_t)stream, d_x, n,
                     qmax_f(bits), (const uint32_t*)d_workspace, d_packed, d_scale);
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
  hipLaunchKernelGGL(k_dequantize_int4_flat, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_packed, n, d_scale, d_out);
  return launch_status();
}

int adfl_pack_int4(const int8_t* d_q, int64_t n, uint8_t* d_packed, void* stream) {
  if (!d_q || !d_packed || n < 1) return ADFL_E_ARG;
  hipLaunchKernelGGL(k_pack_int4, dim3(clamp_grid((((n + 1) >> 1) + kBlock - 1) / kBlock, kMaxFlatBlocks)),
                     dim3(kBlock), 0, (hipStream_t)stream, d_q, n, d_packed);
  return launch_status();
}

int adfl_unpack_int4(const uint8_t* d_packed, int64_t n, int8_t* d_q, void* stream) {
  if (!d_packed || !d_q || n < 1) return ADFL_E_ARG;
  hipLaunchKernelGGL(k_unpack_int4, dim3(clamp_grid((n + kBlock - 1) / kBlock, kMaxFlatBlocks)), dim3(kBlock), 0,
                     (hipStream_t)stream, d_packed, n, d_q);
  return launch_status();
}

int adfl_slq_dequantize_mean(const int8_t* d_q, int64_t row_stride_bytes, int32_t k, int64_t n,
                             const float* d_scales, int64_t scale_stride, float* d_out, void* stream) {
  return adfl_slq_dequantize_mean_self(d_q, row_stride_bytes, k, n, d_scales, scale_stride, -1, nullptr, d_out,
                                       stream);
}

int adfl_slq_dequantize_mean_self(const int8_t* d_q, int64_t row_stride_bytes, int32_t k, int64_t n,
                                  const float* d_scales, int64_t scale_stride, int32_t self_row,
                                  const float* d_self_x, float* d_out, void* stream) {
  if (!d_q || !d_scales || !d_out || n < 1 || bad_rows(k) || row_stride_bytes < n || scale_stride < 1) return ADFL_E_ARG;
  if (self_row >= k || self_row < -1 || (self_row >= 0 && !d_self_x)) return ADFL_E_ARG;
  if (!aligned16(d_q) || !aligned16(d_out) || (row_stride_bytes & 15) != 0) return ADFL_E_ALIGN;
  if (self_row >= 0 && !aligned16(d_self_x)) return ADFL_E_ALIGN;
  auto kern = k >= kDeepRows ? k_dequantize_mean<true> : k_dequantize_mean<false>;
  hipLaunchKernelGGL(kern, dim3(tile_grid(n / kTile)), dim3(kBlock), 0, (hipStream_t)stream, d_q, row_stride_bytes,
                     (int)k, n, d_scales, scale_stride, (int)self_row, d_self_x, d_out);
  return launch_status();
}

int adfl_slq_dequantize_mean_batched(const int8_t* d_q, int64_t row_stride_bytes, int32_t k,
                                     const adfl_slq_chunk* d_chunks, int64_t nchunks, const float* d_scales,
                                     int64_t scale_stride, int32_t self_row, const float* d_self_x, float* d_out,
                                     void* stream) {
  if (!d_q || !d_chunks || !d_scales || !d_out || bad_rows(k) || nchunks < 1 || nchunks > INT32_MAX || scale_stride < 1 ||
      row_stride_bytes < 1)
    return ADFL_E_ARG;
  if (self_row >= k || self_row < -1 || (self_row >= 0 && !d_self_x)) return ADFL_E_ARG;
  if (!aligned16(d_q) || !aligned16(d_out) || (row_stride_bytes & 15) != 0) return ADFL_E_ALIGN;
  if (self_row >= 0 && !aligned16(d_self_x)) return ADFL_E_ALIGN;
  auto kern = k >= kDeepRows ? k_dequantize_mean_batched<true> : k_dequantize_mean_batched<false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_q, row_stride_bytes,
                     (int)k, d_chunks, d_scales, scale_stride, (int)self_row, d_self_x, d_out);
  return launch_status();
}

int adfl_slq_dequantize_mean_batched_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k,
                                          const adfl_slq_chunk* d_chunks, int64_t nchunks, const float* d_scales,
                                          int64_t scale_stride, int32_t self_row, const float* d_self_x,
                                          float* d_out, void* stream) {
  if (!d_packed || !d_chunks || !d_scales || !d_out || bad_rows(k) || nchunks < 1 || nchunks > INT32_MAX ||
      scale_stride < 1 || row_stride_bytes < 1)
    return ADFL_E_ARG;
  if (self_row >= k || self_row < -1 || (self_row >= 0 && !d_self_x)) return ADFL_E_ARG;
  if (!aligned16(d_packed) || !aligned16(d_out) || (row_stride_bytes & 15) != 0) return ADFL_E_ALIGN;
  if (self_row >= 0 && !aligned16(d_self_x)) return ADFL_E_ALIGN;
  auto kern = k >= kDeepRows ? k_dequantize_mean_batched_int4<true> : k_dequantize_mean_batched_int4<false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_packed, row_stride_bytes,
                     (int)k, d_chunks, d_scales, scale_stride, (int)self_row, d_self_x, d_out);
  return launch_status();
}

int adfl_slq_dequantize_add_batched(const int8_t* d_q, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                    const float* d_scales, float* const* d_targets, int32_t ntensors,
                                    int32_t ntargets, void* stream) {
  if (!d_q || !d_chunks || !d_scales || !d_targets || nchunks < 1 || nchunks > INT32_MAX || ntensors < 1 ||
      ntargets < 1)
    return ADFL_E_ARG;
  if (!aligned16(d_q)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_dequantize_add_batched, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_q,
                     d_chunks, d_scales, d_targets, (int)ntensors, (int)ntargets);
  return launch_status();
}

int adfl_slq_dequantize_mean_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k, int64_t n,
                                  const float* d_scales, int64_t scale_stride, float* d_out, void* stream) {
  return adfl_slq_dequantize_mean_self_int4(d_packed, row_stride_bytes, k, n, d_scales, scale_stride, -1, nullptr,
                                            d_out, stream);
}

int adfl_slq_dequantize_mean_self_int4(const uint8_t* d_packed, int64_t row_stride_bytes, int32_t k, int64_t n,
                                       const float* d_scales, int64_t scale_stride, int32_t self_row,
                                       const float* d_self_x, float* d_out, void* stream) {
  if (!d_packed || !d_scales || !d_out || n < 1 || bad_rows(k) || row_stride_bytes < (n + 1) / 2 || scale_stride < 1)
    return ADFL_E_ARG;
  if (self_row >= k || self_row < -1 || (self_row >= 0 && !d_self_x)) return ADFL_E_ARG;
  if (!aligned16(d_packed) || !aligned16(d_out) || (row_stride_bytes & 15) != 0) return ADFL_E_ALIGN;
  if (self_row >= 0 && !aligned16(d_self_x)) return ADFL_E_ALIGN;
  auto kern = k >= kDeepRows ? k_dequantize_mean_int4<true> : k_dequantize_mean_int4<false>;
  hipLaunchKernelGGL(kern, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, (hipStream_t)stream, d_packed,
                     row_stride_bytes, (int)k, n, d_scales, scale_stride, (int)self_row, d_self_x, d_out);
  return launch_status();
}

}  // extern "C"
