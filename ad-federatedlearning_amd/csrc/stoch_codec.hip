// stoch_codec.hip — MI355X (gfx950, CDNA4) kernels for ADFL's stochastic gradient codecs + the C ABI of
// include/adfl_stoch.h.
//
// Reference behaviour restated here (bit-exact given the same norm and uniforms; tests/golden/stoch.npz):
//   QSGD   Src/ADFL/Channel/quant.py:223-252   L2 norm, stochastic level rounding, norm*l/levels*sign
//   RQSGD  Src/ADFL/Channel/quant.py:364-398   max|x| norm, min|x| factor for zero levels
//   CNAT   Src/ADFL/Channel/quant.py:509-545   stochastic power-of-two exponents, norm*sign*2^e
//
// Design. Like the SLQ codec these are HBM streams (read 4 B/elem of x, write 2 B/elem of levels+signs;
// decode reads 2 B and writes 4 B), so every kernel walks a chunk (<= 8192 elements, one block) in
// 16-byte float4 groups: x / out accesses are 16 B per lane, the byte planes 4 B per lane, all contiguous
// across the wave. Grid-wide dependencies (a tensor's norm) are kernel boundaries: chunk partials ->
// per-tensor finalize -> quantize. CNAT's rounding does not depend on the norm, so its encode reads x
// once (exponents + norm partials in the same pass) and a per-chunk fix-up rewrites the (rare) all-zero
// tensors the way the reference's norm == 0 branch returns them.
//
// Uniforms come from an in-register Philox4x32-10 stream (4 uniforms per 128-bit block, one block per
// float4 group: no uniform ever touches HBM) or from an injected plane (parity tests).
//
// Numerics: no fast-math, -ffp-contract=off, IEEE fp32 denormals; divisions are correctly rounded
// (__fdiv_rn) because the reference divides element by element in fp32; CNAT's floor/ceil(log2) is the
// exact integer band rule of cnat_log2_table.h (no transcendental, no rounding risk).

#include <hip/hip_runtime.h>

#include <cstdint>

#include "adfl_stoch.h"
#include "cnat_log2_table.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kFinalizeGrid = 1024;
constexpr int64_t kPartialBytes = 16;  // per chunk: fp64 sum of squares, or {max, min} |x| bits

// ------------------------------------------------------------------------------------------------
// uniforms
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint64_t ctr, uint64_t seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // full 32x32 -> 64 products: one v_mad_u64_u32 each instead of a v_mul_hi_u32 + v_mul_lo_u32 pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    c1 = (uint32_t)p1;
    c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ float u24(uint32_t w) { return (float)(w >> 8) * 0x1p-24f; }

struct Uniforms {
  const float* inj;  // injected plane (indexed like x) or null
  uint64_t seed, counter;

  // u for elements g .. g+3, g % 4 == 0
  __device__ __forceinline__ float4 group(int64_t g) const {
    if (inj) return *reinterpret_cast<const float4*>(inj + g);
    const uint4 w = philox4x32_10(counter + (uint64_t)(g >> 2), seed);
    return make_float4(u24(w.x), u24(w.y), u24(w.z), u24(w.w));
  }
  __device__ __forceinline__ float one(int64_t g) const {
    if (inj) return inj[g];
    const uint4 w = philox4x32_10(counter + (uint64_t)(g >> 2), seed);
    const int k = (int)(g & 3);
    return u24(k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : w.w);
  }
};

// ------------------------------------------------------------------------------------------------
// element rules
// ------------------------------------------------------------------------------------------------
// torch's fp32 -> uint8 / int8 conversion on x86: truncate to int32 (NaN and out-of-range give INT32_MIN,
// whose low byte is 0), keep the low byte.
__device__ __forceinline__ uint32_t low_byte(float v) {
  if (!(v > -2147483648.0f && v < 2147483648.0f)) return 0u;
  return (uint32_t)(int)v & 0xffu;
}

__device__ __forceinline__ uint32_t sign_byte(float x) { return (uint32_t)((x > 0.0f) - (x < 0.0f)) & 0xffu; }

__device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return a | (b << 8) | (c << 16) | (d << 24);
}

// QSGD / RQSGD level (quant.py:230-236): s * |x| / norm in fp32, floor, stochastic round up.
__device__ __forceinline__ uint32_t qsgd_level(float x, float s, float norm, float u) {
  const float scaled = __fdiv_rn(s * __builtin_fabsf(x), norm);
  const float l = __builtin_floorf(scaled);
  const float prob = scaled - l;
  return low_byte(l + (u < prob ? 1.0f : 0.0f));
}

__device__ __forceinline__ float pow2i(int k) {  // 2^k for k in [-126, 128] (128 -> inf), exact
  return __uint_as_float((uint32_t)(k + 127) << 23);
}

// CNAT exponent (quant.py:516-532). v = fl(|x| + eps) >= 2^-23 is normal, so its binary exponent e and the
// band table give floor / ceil of fl32(log2 v) exactly.
__device__ __forceinline__ uint32_t cnat_exp(float x, float u, float min_e, float max_e) {
  if (x == 0.0f) return low_byte(min_e);  // final_exponents[x == 0] = min_exp
  const float xa = __builtin_fabsf(x);
  const float v = xa + 0x1p-23f;
  if (__builtin_isnan(v)) return 0u;                 // log2 NaN -> ceil NaN -> clamp keeps NaN -> int8 0
  if (__builtin_isinf(v)) return low_byte(max_e);    // prob = NaN -> ceil = inf -> clamped to max_exp
  const uint32_t bits = __float_as_uint(v);
  const int e = (int)(bits >> 23) - 127;
  const uint32_t m = bits & 0x7fffffu;
  int f = e, c = e + 1;
  if (m <= kCnatBand[e - kCnatKMin].above) {
    c = e;
  } else if (0x800000u - m <= kCnatBand[e + 1 - kCnatKMin].below) {
    f = e + 1;
  }
  const float prob = __fdiv_rn(pow2i(c) - xa, pow2i(f));
  float ef = (u < prob) ? (float)f : (float)c;
  ef = __builtin_fminf(__builtin_fmaxf(ef, min_e), max_e);
  return low_byte(ef);
}

// decoders
__device__ __forceinline__ float qsgd_value(uint32_t l, uint32_t sgn, float norm, float s) {
  return __fdiv_rn(norm * (float)l, s) * (float)(int8_t)sgn;
}

__device__ __forceinline__ float rqsgd_value(uint32_t l, uint32_t sgn, float norm, float mn, float s) {
  const float sf = (float)(int8_t)sgn;
  return l == 0u ? mn * sf : __fdiv_rn((norm * sf) * (float)l, s);
}

__device__ __forceinline__ float cnat_value(uint32_t e, uint32_t sgn, float norm) {
  const int k = (int)(int8_t)e;  // in [-128, 127]
  // 2^k exactly: normal for k >= -126, the denormals 2^-127 / 2^-128 below
  const float p = k >= -126 ? pow2i(k) : __uint_as_float(0x00400000u >> (-127 - k));
  return (norm * (float)(int8_t)sgn) * p;
}

// ------------------------------------------------------------------------------------------------
// reductions
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double red[kWaves];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return v;
}

__device__ __forceinline__ uint2 block_maxmin(uint32_t mx, uint32_t mn) {
  __shared__ uint32_t red[2][kWaves];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = mx;
    red[1][threadIdx.x >> 6] = mn;
  }
  __syncthreads();
  const uint2 r = make_uint2(max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3])),
                             min(min(red[1][0], red[1][1]), min(red[1][2], red[1][3])));
  __syncthreads();
  return r;
}

__device__ __forceinline__ uint32_t abs_bits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

__device__ __forceinline__ double sq(float v) { return (double)(v * v); }  // fp32 square, as torch

// elements [0, head) of a chunk are done one by one, up to the first 4-element boundary of the bucket
__device__ __forceinline__ int chunk_head4(int64_t start, int len) {
  const int h = (int)((4 - (start & 3)) & 3);
  return h < len ? h : len;
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
// Norm partials, one block per chunk: fp64 sum of fp32 squares (L2) or {max, min} of |x| bits (LINF).
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_norm_partials(const float* __restrict__ x,
                                                          const adfl_slq_chunk* __restrict__ chunks,
                                                          void* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  const int head = chunk_head4(c.start, c.len);
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
  const int n4 = (c.len - head) >> 2;
  const int tail = head + (n4 << 2);
  if (MODE == ADFL_NORM_L2) {
    double s = 0.0;
    if ((int)threadIdx.x < head) s = sq(xc[threadIdx.x]);
    for (int i = threadIdx.x; i < n4; i += kBlock) {
      const float4 v = x4[i];
      s += (sq(v.x) + sq(v.y)) + (sq(v.z) + sq(v.w));
    }
    if ((int)threadIdx.x < c.len - tail) s += sq(xc[tail + threadIdx.x]);
    s = block_sum(s);
    if (threadIdx.x == 0) reinterpret_cast<double*>(partials)[blockIdx.x] = s;
  } else {
    uint32_t mx = 0u, mn = 0xffffffffu;
    if ((int)threadIdx.x < head) mx = mn = abs_bits(xc[threadIdx.x]);
    for (int i = threadIdx.x; i < n4; i += kBlock) {
      const float4 v = x4[i];
      const uint32_t a = abs_bits(v.x), b = abs_bits(v.y), d = abs_bits(v.z), e = abs_bits(v.w);
      mx = max(mx, max(max(a, b), max(d, e)));
      mn = min(mn, min(min(a, b), min(d, e)));
    }
    if ((int)threadIdx.x < c.len - tail) {
      const uint32_t a = abs_bits(xc[tail + threadIdx.x]);
      mx = max(mx, a);
      mn = min(mn, a);
    }
    const uint2 r = block_maxmin(mx, mn);
    if (threadIdx.x == 0) reinterpret_cast<uint2*>(partials)[blockIdx.x] = r;
  }
}

// Per-tensor finalize: the block that meets a tensor's first chunk reduces its partials in a fixed
// order and writes the norm (and min).
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_norm_finalize(const adfl_slq_chunk* __restrict__ chunks, int64_t nchunks,
                                                          const void* __restrict__ partials,
                                                          float* __restrict__ norms, float* __restrict__ mins) {
  for (int64_t ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const adfl_slq_chunk c = chunks[ci];
    if (c.first_chunk != ci) continue;  // uniform per block
    if (MODE == ADFL_NORM_L2) {
      const double* p = reinterpret_cast<const double*>(partials) + ci;
      double s = 0.0;
      for (int k = threadIdx.x; k < c.nchunks; k += kBlock) s += p[k];
      s = block_sum(s);
      // round the sum once to fp32 (as torch's fp32 sum ends), then the correctly rounded fp32 sqrt
      if (threadIdx.x == 0) norms[c.tensor] = (float)__builtin_sqrt((double)(float)s);
    } else {
      const uint2* p = reinterpret_cast<const uint2*>(partials) + ci;
      uint32_t mx = 0u, mn = 0xffffffffu;
      for (int k = threadIdx.x; k < c.nchunks; k += kBlock) {
        const uint2 v = p[k];
        mx = max(mx, v.x);
        mn = min(mn, v.y);
      }
      const uint2 r = block_maxmin(mx, mn);
      if (threadIdx.x == 0) {
        const bool nan = r.x > 0x7f800000u;  // NaN anywhere: torch's max and min both propagate it
        norms[c.tensor] = nan ? __builtin_nanf("") : __uint_as_float(r.x);
        if (mins) mins[c.tensor] = nan ? __builtin_nanf("") : __uint_as_float(r.y);
      }
    }
  }
}

__device__ __forceinline__ void fill_zero_norm(uint8_t* __restrict__ lv, int8_t* __restrict__ sg, int len) {
  for (int i = threadIdx.x; i < len; i += kBlock) {
    lv[i] = 0;
    sg[i] = 1;
  }
}

__global__ __launch_bounds__(kBlock) void k_qsgd_quantize(const float* __restrict__ x,
                                                          const adfl_slq_chunk* __restrict__ chunks, float s,
                                                          const float* __restrict__ norms, Uniforms U,
                                                          uint8_t* __restrict__ levels, int8_t* __restrict__ signs) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float norm = norms[c.tensor];
  uint8_t* lv = levels + c.start;
  int8_t* sg = signs + c.start;
  if (norm == 0.0f) {  // quant.py:227-228
    fill_zero_norm(lv, sg, c.len);
    return;
  }
  const float* xc = x + c.start;
  const int head = chunk_head4(c.start, c.len);
  if ((int)threadIdx.x < head) {
    const int i = threadIdx.x;
    lv[i] = (uint8_t)qsgd_level(xc[i], s, norm, U.one(c.start + i));
    sg[i] = (int8_t)sign_byte(xc[i]);
  }
  const int n4 = (c.len - head) >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
  uint32_t* l4 = reinterpret_cast<uint32_t*>(lv + head);
  uint32_t* s4 = reinterpret_cast<uint32_t*>(sg + head);
  for (int k = threadIdx.x; k < n4; k += kBlock) {
    const float4 v = x4[k];
    const float4 u = U.group(c.start + head + 4 * (int64_t)k);
    l4[k] = pack4(qsgd_level(v.x, s, norm, u.x), qsgd_level(v.y, s, norm, u.y), qsgd_level(v.z, s, norm, u.z),
                  qsgd_level(v.w, s, norm, u.w));
    s4[k] = pack4(sign_byte(v.x), sign_byte(v.y), sign_byte(v.z), sign_byte(v.w));
  }
  const int tail = head + (n4 << 2);
  if ((int)threadIdx.x < c.len - tail) {
    const int i = tail + threadIdx.x;
    lv[i] = (uint8_t)qsgd_level(xc[i], s, norm, U.one(c.start + i));
    sg[i] = (int8_t)sign_byte(xc[i]);
  }
}

// CNAT: exponents + signs + L2 partials in one read of x.
__global__ __launch_bounds__(kBlock) void k_cnat_quantize(const float* __restrict__ x,
                                                          const adfl_slq_chunk* __restrict__ chunks, float min_e,
                                                          float max_e, Uniforms U, int8_t* __restrict__ exps,
                                                          int8_t* __restrict__ signs, double* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  int8_t* ex = exps + c.start;
  int8_t* sg = signs + c.start;
  const int head = chunk_head4(c.start, c.len);
  double ss = 0.0;
  if ((int)threadIdx.x < head) {
    const int i = threadIdx.x;
    const float v = xc[i];
    ex[i] = (int8_t)cnat_exp(v, U.one(c.start + i), min_e, max_e);
    sg[i] = (int8_t)sign_byte(v);
    ss = sq(v);
  }
  const int n4 = (c.len - head) >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
  uint32_t* e4 = reinterpret_cast<uint32_t*>(ex + head);
  uint32_t* s4 = reinterpret_cast<uint32_t*>(sg + head);
  for (int k = threadIdx.x; k < n4; k += kBlock) {
    const float4 v = x4[k];
    const float4 u = U.group(c.start + head + 4 * (int64_t)k);
    e4[k] = pack4(cnat_exp(v.x, u.x, min_e, max_e), cnat_exp(v.y, u.y, min_e, max_e),
                  cnat_exp(v.z, u.z, min_e, max_e), cnat_exp(v.w, u.w, min_e, max_e));
    s4[k] = pack4(sign_byte(v.x), sign_byte(v.y), sign_byte(v.z), sign_byte(v.w));
    ss += (sq(v.x) + sq(v.y)) + (sq(v.z) + sq(v.w));
  }
  const int tail = head + (n4 << 2);
  if ((int)threadIdx.x < c.len - tail) {
    const int i = tail + threadIdx.x;
    const float v = xc[i];
    ex[i] = (int8_t)cnat_exp(v, U.one(c.start + i), min_e, max_e);
    sg[i] = (int8_t)sign_byte(v);
    ss += sq(v);
  }
  ss = block_sum(ss);
  if (threadIdx.x == 0) partials[blockIdx.x] = ss;
}

// CNAT norm == 0 (an all-zero tensor): the reference returns u8 zeros and int8 ones (quant.py:513-514).
__global__ __launch_bounds__(kBlock) void k_cnat_zero_fixup(const adfl_slq_chunk* __restrict__ chunks,
                                                            const float* __restrict__ norms,
                                                            int8_t* __restrict__ exps, int8_t* __restrict__ signs) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  if (norms[c.tensor] != 0.0f) return;
  fill_zero_norm(reinterpret_cast<uint8_t*>(exps) + c.start, signs + c.start, c.len);
}

__device__ __forceinline__ void store4_nt(float4* p, float4 d) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v v = {d.x, d.y, d.z, d.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
}

// Decoders. KIND 0 = QSGD, 1 = RQSGD, 2 = CNAT.
template <int KIND>
__device__ __forceinline__ float decode1(uint32_t l, uint32_t sgn, float norm, float mn, float s) {
  if (KIND == 0) return qsgd_value(l, sgn, norm, s);
  if (KIND == 1) return rqsgd_value(l, sgn, norm, mn, s);
  return cnat_value(l, sgn, norm);
}

template <int KIND>
__global__ __launch_bounds__(kBlock) void k_stoch_dequantize(const uint8_t* __restrict__ levels,
                                                             const int8_t* __restrict__ signs,
                                                             const adfl_slq_chunk* __restrict__ chunks,
                                                             const float* __restrict__ norms,
                                                             const float* __restrict__ mins, float s,
                                                             float* __restrict__ out) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float norm = norms[c.tensor];
  const float mn = KIND == 1 ? mins[c.tensor] : 0.0f;
  float* oc = out + c.start;
  if (norm == 0.0f) {  // quant.py:248-249 / :390-391 / :542-543
    for (int i = threadIdx.x; i < c.len; i += kBlock) oc[i] = 0.0f;
    return;
  }
  const uint8_t* lv = levels + c.start;
  const uint8_t* sg = reinterpret_cast<const uint8_t*>(signs) + c.start;
  const int head = chunk_head4(c.start, c.len);
  if ((int)threadIdx.x < head) oc[threadIdx.x] = decode1<KIND>(lv[threadIdx.x], sg[threadIdx.x], norm, mn, s);
  const int n4 = (c.len - head) >> 2;
  const uint32_t* l4 = reinterpret_cast<const uint32_t*>(lv + head);
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(sg + head);
  float4* o4 = reinterpret_cast<float4*>(oc + head);
  for (int k = threadIdx.x; k < n4; k += kBlock) {
    const uint32_t l = l4[k], g = s4[k];
    float4 r;
    r.x = decode1<KIND>(l & 0xffu, g & 0xffu, norm, mn, s);
    r.y = decode1<KIND>((l >> 8) & 0xffu, (g >> 8) & 0xffu, norm, mn, s);
    r.z = decode1<KIND>((l >> 16) & 0xffu, (g >> 16) & 0xffu, norm, mn, s);
    r.w = decode1<KIND>(l >> 24, g >> 24, norm, mn, s);
    store4_nt(o4 + k, r);
  }
  const int tail = head + (n4 << 2);
  if ((int)threadIdx.x < c.len - tail) {
    const int i = tail + threadIdx.x;
    oc[i] = decode1<KIND>(lv[i], sg[i], norm, mn, s);
  }
}

__global__ __launch_bounds__(kBlock) void k_philox_uniforms(float* __restrict__ out, int64_t n, int64_t start,
                                                            Uniforms U) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    out[i] = U.one(start + i);
}

// ------------------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------------------
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int check_bits(int bits) { return (bits >= 1 && bits <= 16) ? ADFL_OK : ADFL_E_BITS; }

inline float levels_f(int bits) { return (float)((1LL << bits) - 1); }  // self.levels = 2**bits - 1

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ADFL_OK : (int)e;
}

inline bool bad_table(const adfl_slq_chunk* d_chunks, int64_t nchunks) {
  return !d_chunks || nchunks < 1 || nchunks > INT32_MAX;
}

inline int check_ws(const void* d_ws, int64_t bytes, int64_t nchunks) {
  if (!d_ws) return ADFL_E_ARG;
  if (!aligned16(d_ws)) return ADFL_E_ALIGN;
  return bytes < nchunks * kPartialBytes ? ADFL_E_WORKSPACE : ADFL_OK;
}

inline int finalize_grid(int64_t nchunks) { return (int)(nchunks < kFinalizeGrid ? nchunks : kFinalizeGrid); }

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int64_t adfl_stoch_workspace_bytes(int64_t nchunks) { return nchunks < 1 ? kPartialBytes : nchunks * kPartialBytes; }

int adfl_stoch_norms_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int mode,
                             void* d_workspace, int64_t workspace_bytes, float* d_norms, float* d_mins,
                             void* stream) {
  if (!d_x || !d_norms || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (mode != ADFL_NORM_L2 && mode != ADFL_NORM_LINF) return ADFL_E_ARG;
  if (int s = check_ws(d_workspace, workspace_bytes, nchunks)) return s;
  if (!aligned16(d_x)) return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  if (mode == ADFL_NORM_L2) {
    hipLaunchKernelGGL(k_norm_partials<ADFL_NORM_L2>, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks,
                       d_workspace);
    if (int s = launch_status()) return s;
    hipLaunchKernelGGL(k_norm_finalize<ADFL_NORM_L2>, dim3(finalize_grid(nchunks)), dim3(kBlock), 0, st, d_chunks,
                       nchunks, (const void*)d_workspace, d_norms, d_mins);
  } else {
    hipLaunchKernelGGL(k_norm_partials<ADFL_NORM_LINF>, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x,
                       d_chunks, d_workspace);
    if (int s = launch_status()) return s;
    hipLaunchKernelGGL(k_norm_finalize<ADFL_NORM_LINF>, dim3(finalize_grid(nchunks)), dim3(kBlock), 0, st,
                       d_chunks, nchunks, (const void*)d_workspace, d_norms, d_mins);
  }
  return launch_status();
}

int adfl_qsgd_quantize_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                               const float* d_norms, const float* d_uniforms, uint64_t seed, uint64_t counter,
                               uint8_t* d_levels, int8_t* d_signs, void* stream) {
  if (!d_x || !d_norms || !d_levels || !d_signs || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_levels) || !aligned16(d_signs) || (d_uniforms && !aligned16(d_uniforms)))
    return ADFL_E_ALIGN;
  const Uniforms U{d_uniforms, seed, counter};
  hipLaunchKernelGGL(k_qsgd_quantize, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_x, d_chunks,
                     levels_f(bits), d_norms, U, d_levels, d_signs);
  return launch_status();
}

int adfl_qsgd_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                             const float* d_uniforms, uint64_t seed, uint64_t counter, void* d_workspace,
                             int64_t workspace_bytes, uint8_t* d_levels, int8_t* d_signs, float* d_norms,
                             void* stream) {
  if (int s = check_bits(bits)) return s;
  if (int s = adfl_stoch_norms_batched(d_x, d_chunks, nchunks, ADFL_NORM_L2, d_workspace, workspace_bytes, d_norms,
                                       nullptr, stream))
    return s;
  return adfl_qsgd_quantize_batched(d_x, d_chunks, nchunks, bits, d_norms, d_uniforms, seed, counter, d_levels,
                                    d_signs, stream);
}

int adfl_rqsgd_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                              const float* d_uniforms, uint64_t seed, uint64_t counter, void* d_workspace,
                              int64_t workspace_bytes, uint8_t* d_levels, int8_t* d_signs, float* d_norms,
                              float* d_mins, void* stream) {
  if (!d_mins) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (int s = adfl_stoch_norms_batched(d_x, d_chunks, nchunks, ADFL_NORM_LINF, d_workspace, workspace_bytes,
                                       d_norms, d_mins, stream))
    return s;
  return adfl_qsgd_quantize_batched(d_x, d_chunks, nchunks, bits, d_norms, d_uniforms, seed, counter, d_levels,
                                    d_signs, stream);
}

int adfl_qsgd_dequantize_batched(const uint8_t* d_levels, const int8_t* d_signs, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, int bits, const float* d_norms, float* d_out, void* stream) {
  if (!d_levels || !d_signs || !d_norms || !d_out || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_levels) || !aligned16(d_signs) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_stoch_dequantize<0>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_levels,
                     d_signs, d_chunks, d_norms, (const float*)nullptr, levels_f(bits), d_out);
  return launch_status();
}

int adfl_rqsgd_dequantize_batched(const uint8_t* d_levels, const int8_t* d_signs, const adfl_slq_chunk* d_chunks,
                                  int64_t nchunks, int bits, const float* d_norms, const float* d_mins,
                                  float* d_out, void* stream) {
  if (!d_levels || !d_signs || !d_norms || !d_mins || !d_out || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_levels) || !aligned16(d_signs) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_stoch_dequantize<1>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_levels,
                     d_signs, d_chunks, d_norms, d_mins, levels_f(bits), d_out);
  return launch_status();
}

int adfl_cnat_encode_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                             const float* d_uniforms, uint64_t seed, uint64_t counter, void* d_workspace,
                             int64_t workspace_bytes, int8_t* d_exps, int8_t* d_signs, float* d_norms,
                             void* stream) {
  if (!d_x || !d_exps || !d_signs || !d_norms || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (int s = check_ws(d_workspace, workspace_bytes, nchunks)) return s;
  if (!aligned16(d_x) || !aligned16(d_exps) || !aligned16(d_signs) || (d_uniforms && !aligned16(d_uniforms)))
    return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  const Uniforms U{d_uniforms, seed, counter};
  const float min_e = -(float)(1LL << (bits - 1)), max_e = (float)((1LL << (bits - 1)) - 1);  // quant.py:519-520
  hipLaunchKernelGGL(k_cnat_quantize, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, min_e, max_e, U,
                     d_exps, d_signs, (double*)d_workspace);
  if (int s = launch_status()) return s;
  hipLaunchKernelGGL(k_norm_finalize<ADFL_NORM_L2>, dim3(finalize_grid(nchunks)), dim3(kBlock), 0, st, d_chunks,
                     nchunks, (const void*)d_workspace, d_norms, (float*)nullptr);
  if (int s = launch_status()) return s;
  hipLaunchKernelGGL(k_cnat_zero_fixup, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_chunks,
                     (const float*)d_norms, d_exps, d_signs);
  return launch_status();
}

int adfl_cnat_dequantize_batched(const int8_t* d_exps, const int8_t* d_signs, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, const float* d_norms, float* d_out, void* stream) {
  if (!d_exps || !d_signs || !d_norms || !d_out || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (!aligned16(d_exps) || !aligned16(d_signs) || !aligned16(d_out)) return ADFL_E_ALIGN;
  hipLaunchKernelGGL(k_stoch_dequantize<2>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint8_t*>(d_exps), d_signs, d_chunks, d_norms, (const float*)nullptr,
                     1.0f, d_out);
  return launch_status();
}

int adfl_philox_uniforms(float* d_out, int64_t n, int64_t start, uint64_t seed, uint64_t counter, void* stream) {
  if (!d_out || n < 1 || start < 0) return ADFL_E_ARG;
  const Uniforms U{nullptr, seed, counter};
  const int64_t g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_philox_uniforms, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_out, n, start, U);
  return launch_status();
}

}  // extern "C"
