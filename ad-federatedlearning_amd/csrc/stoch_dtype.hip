// stoch_dtype.hip — the stochastic codecs (QSGD / RQSGD / CNAT) on fp16, bf16 and fp64 tensors, in the
// tensor's own dtype as the reference computes them (Src/ADFL/Channel/quant.py:223-240, :364-382,
// :509-534), and the C ABI of include/adfl_stoch.h's *_dt entries.
//
// The reference's ops on an fp16 / bf16 tensor each compute in fp32 and round the result to the dtype
// once (torch's CPU kernels); on fp64 they are fp64 ops. Every step below does the same: arithmetic in
// C = fp32 (fp64 for fp64), R() = round to the dtype after each op, in the reference's operation order:
//   QSGD / RQSGD  scaled = R(R(s*|x|) / norm); l = floor(scaled); prob = R(scaled - l);
//                 q = u8(l + (u < prob)); signs = i8(sign(x))
//   CNAT          v = R(|x| + eps); f, c = floor / ceil of fl(log2 v) (the exact band rule of
//                 cnat_log2_dt_table.h, from torch's own log2 in each dtype); prob = R(R(R(2^c) - |x|) / R(2^f));
//                 e = (u < prob) ? f : c, clamped, min_exp where x == 0; i8(e)
// Uniforms are on torch.rand's grid for the dtype (2^-11 fp16, 2^-8 bf16, 2^-53 fp64): injected (a plane of
// the dtype, indexed like x) or drawn from the Philox4x32-7 stream (oracle/stoch_dt_oracle.py restates it).
// Norms: fp16 / bf16 squares in fp32 accumulated in fp64, rounded once to fp32, correctly rounded sqrt,
// rounded to the dtype; fp64 squares accumulated in fp64. Returned as fp64 (exactly the dtype's value).
// Decode is the fp32 codecs' (the reference decodes to fp32 with scale = fp32(norm)).
//
// These tensors are rare in ADFL (models train in fp32), so the kernels keep one simple shape: one 256-thread
// block per chunk, each thread one 16-byte vector of x per step (8 fp16 / bf16 or 2 fp64 elements; two
// Philox blocks or one), kBatch steps' loads in flight, scalar head / tail elements around the vectors.
// QSGD / RQSGD: norm partials, per-tensor finalize, quantize (x read twice). CNAT: quantize + partials in one
// read of x, finalize, zero-norm fix-up; its band tables in LDS and its exponent carried as an integer.

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "adfl_stoch.h"
#include "cnat_log2_dt_table.h"
#include "philox.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// ------------------------------------------------------------------------------------------------
// dtypes: storage S, compute C, rounding R, uniform from Philox words, CNAT's band rule
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float rn_bf16(float v) {
  const uint32_t b = __float_as_uint(v);
  if ((b & 0x7fffffffu) > 0x7f800000u) return __uint_as_float((b | 0x00400000u) & 0xffff0000u);  // NaN
  return __uint_as_float((b + 0x7fffu + ((b >> 16) & 1u)) & 0xffff0000u);
}

struct DtF16 {
  using S = uint16_t;
  using C = float;
  static constexpr int kMBits = 10, kBias = 15, kKMin = kCnatF16KMin;
  static constexpr float kEps = 0x1p-10f;
  __device__ static float load(S s) { return __half2float(__ushort_as_half(s)); }
  __device__ static float rn(float v) { return __half2float(__float2half_rn(v)); }
  __device__ static uint32_t bits(float v_on_grid) { return __half_as_ushort(__float2half_rn(v_on_grid)); }
  __device__ static float uniform(uint32_t w) { return (float)(w >> 21) * 0x1p-11f; }
  static constexpr int kBands = kCnatF16KMax - kCnatF16KMin + 1;
  __device__ static const uint16_t* below_tab() { return kCnatF16Below; }
  __device__ static const uint16_t* above_tab() { return kCnatF16Above; }
};

struct DtBF16 {
  using S = uint16_t;
  using C = float;
  static constexpr int kMBits = 7, kBias = 127, kKMin = kCnatBF16KMin;
  static constexpr float kEps = 0x1p-7f;
  __device__ static float load(S s) { return __uint_as_float((uint32_t)s << 16); }
  __device__ static float rn(float v) { return rn_bf16(v); }
  __device__ static uint32_t bits(float v_on_grid) { return __float_as_uint(v_on_grid) >> 16; }
  __device__ static float uniform(uint32_t w) { return (float)(w >> 24) * 0x1p-8f; }
  static constexpr int kBands = kCnatBF16KMax - kCnatBF16KMin + 1;
  __device__ static const uint16_t* below_tab() { return kCnatBF16Below; }
  __device__ static const uint16_t* above_tab() { return kCnatBF16Above; }
};

struct DtF64 {
  using S = double;
  using C = double;
  static constexpr int kMBits = 52, kBias = 1023, kKMin = kCnatF64KMin;
  static constexpr double kEps = 0x1p-52;
  __device__ static double load(S s) { return s; }
  __device__ static double rn(double v) { return v; }
  __device__ static uint64_t bits(double v) { return (uint64_t)__double_as_longlong(v); }
  static constexpr int kBands = kCnatF64KMax - kCnatF64KMin + 1;
  __device__ static const uint16_t* below_tab() { return kCnatF64Below; }
  __device__ static const uint16_t* above_tab() { return kCnatF64Above; }
};

// torch's fp -> uint8 / int8 conversion on x86: truncate to int32 (NaN / out of range -> INT32_MIN, low
// byte 0), keep the low byte.
template <typename C>
__device__ __forceinline__ uint32_t low_byte(C v) {
  if (!(v > (C)-2147483648.0 && v < (C)2147483648.0)) return 0u;
  return (uint32_t)(int)v & 0xffu;
}

template <typename C>
__device__ __forceinline__ uint32_t sign_byte(C x) {
  return (uint32_t)((x > (C)0) - (x < (C)0)) & 0xffu;
}

// The four uniforms of elements g0 .. g0+3 (g0 % 4 == 0) of the stream.
template <typename T>
__device__ __forceinline__ void stream4(uint64_t seed, uint64_t counter, int64_t g0, typename T::C (&u)[4]) {
  if constexpr (sizeof(typename T::S) == 8) {   // fp64: two Philox blocks, 64 bits per element
    const uint4 a = adfl::philox4x32(counter + (uint64_t)(g0 >> 1), seed);
    const uint4 b = adfl::philox4x32(counter + (uint64_t)(g0 >> 1) + 1, seed);
    const uint64_t w[4] = {((uint64_t)a.x << 32) | a.y, ((uint64_t)a.z << 32) | a.w, ((uint64_t)b.x << 32) | b.y,
                           ((uint64_t)b.z << 32) | b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) u[j] = (double)(w[j] >> 11) * 0x1p-53;
  } else {
    const uint4 a = adfl::philox4x32(counter + (uint64_t)(g0 >> 2), seed);
    u[0] = T::uniform(a.x);
    u[1] = T::uniform(a.y);
    u[2] = T::uniform(a.z);
    u[3] = T::uniform(a.w);
  }
}

// The band tables of T, copied into LDS by the CNAT kernel (a lookup per element from the __constant__ arrays
// was a global load in every element's dependency chain).
struct Bands {
  const uint16_t* below;
  const uint16_t* above;
};

// CNAT's floor / ceil of fl(log2 v) for a finite v = R(|x| + eps) (>= eps: normal), by the band rule.
template <typename T>
__device__ __forceinline__ void cnat_bounds(typename T::C v, int& lo, int& hi, const Bands& tb) {
  const auto b = T::bits(v);
  using B = decltype(b);
  const B one = (B)1 << T::kMBits;  // 2^mantissa bits: ulps per binade
  const int e = (int)(b >> T::kMBits) - T::kBias;
  const B m = b & (one - 1);
  const B ab = tb.above[e - T::kKMin], bb = tb.below[e + 1 - T::kKMin];  // both read: no branch on the lookups
  lo = e;
  hi = e + 1;
  if (m <= ab) {
    hi = e;
  } else if (one - m <= bb) {
    lo = e + 1;
  }
}

// 2^k in C, exact, for the band range of every dtype (fp32: k in [-126, 128], 128 -> inf; fp64: k in
// [-1022, 1024], 1024 -> inf), built from the exponent field.
template <typename C>
__device__ __forceinline__ C pow2i(int k) {
  if constexpr (sizeof(C) == 4) {
    return __uint_as_float((uint32_t)(k + 127) << 23);
  } else {
    return __longlong_as_double((long long)(k + 1023) << 52);
  }
}

// One element -> (level / exponent byte, sign byte). KIND: 0 QSGD / 1 RQSGD (levels), 2 CNAT (exponents).
template <typename T, int KIND>
__device__ __forceinline__ uint32_t encode_elem(typename T::C x, typename T::C u, typename T::C norm, int bits,
                                                uint32_t& sg, const Bands& tb) {
  using C = typename T::C;
  const C xa = __builtin_fabs(x);
  sg = sign_byte(x);
  if constexpr (KIND != 2) {
    const C s = (C)((1 << bits) - 1);
    const C a = T::rn(s * xa);
    const C scaled = T::rn(a / norm);
    const C l = sizeof(C) == 4 ? (C)floorf((float)scaled) : (C)floor((double)scaled);
    const C prob = T::rn(scaled - l);
    const C lev = l + (u < prob ? (C)1 : (C)0);
    return low_byte(lev);
  } else {
    // The exponent is integral from here on. NaN x: ceil NaN, clamp_ keeps it, int8(NaN) = 0; inf x (the
    // only way v is inf): log2 inf = inf, prob = NaN, so ceil = inf, clamped to max_exp.
    const int min_e = -(1 << (bits - 1)), max_e = (1 << (bits - 1)) - 1;
    if (x == (C)0) return (uint32_t)min_e & 0xffu;
    const C v = T::rn(xa + (C)T::kEps);
    if (!(v == v)) return 0u;
    if (__builtin_isinf(v)) return (uint32_t)max_e & 0xffu;
    int lo, hi;
    cnat_bounds<T>(v, lo, hi, tb);
    // the reference's (2^c - |x|) / 2^f, each op rounded to the dtype (2^16 is inf in fp16: prob NaN, ceil).
    // f >= log2(eps) (v >= eps), so 2^f is a normal value of the dtype and the quotient of the rounded
    // numerator (0, or at least ulp(2^c) >= 2^(f - mantissa bits)) by it is exact in C: an exponent shift
    // (v_ldexp) gives the quotient the division would, without the ~10-instruction correctly rounded divide.
    const C num = T::rn(T::rn(pow2i<C>(hi)) - xa);
    C prob;
    if constexpr (sizeof(C) == 4) prob = T::rn(__builtin_ldexpf(num, -lo));
    else prob = __builtin_ldexp(num, -lo);
    const int r = u < prob ? lo : hi;
    return (uint32_t)min(max(r, min_e), max_e) & 0xffu;
  }
}

// 16-byte vectors: V elements (8 for fp16 / bf16, 2 for fp64). A chunk is split into a scalar head up to
// the first V-element boundary, whole vectors, and a scalar tail.
template <typename T>
constexpr int kVec = 16 / (int)sizeof(typename T::S);

struct Span {
  int64_t b0, nv, b1, end;  // vectors cover [b0, b1), b1 = b0 + nv * V
};

template <typename T>
__device__ __forceinline__ Span split_chunk(const adfl_slq_chunk& c) {
  constexpr int V = kVec<T>;
  Span sp;
  sp.end = c.start + c.len;
  const int64_t a0 = (c.start + V - 1) / V * V;
  sp.b0 = a0 < sp.end ? a0 : sp.end;
  sp.nv = (sp.end - sp.b0) / V;
  sp.b1 = sp.b0 + sp.nv * V;
  return sp;
}

// The uniform of element g alone (head / tail elements).
template <typename T>
__device__ __forceinline__ typename T::C stream1(uint64_t seed, uint64_t counter, int64_t g) {
  typename T::C u[4];
  stream4<T>(seed, counter, g & ~(int64_t)3, u);
  return u[g & 3];
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
// The chunk's whole 16-byte vectors, thread t taking vectors t, t + 256, ... in order: kBatch loads issued
// (index clamped to the last vector) before the first is used. One load per step left every step waiting
// on its own load's latency.
constexpr int kBatch = 4;

template <class F>
__device__ __forceinline__ void for_vectors(const uint4* __restrict__ xv, int64_t nv, F&& f) {
  for (int64_t i0 = threadIdx.x; i0 < nv; i0 += kBatch * kBlock) {
    uint4 w[kBatch];
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int64_t i = i0 + b * kBlock;
      w[b] = xv[i < nv ? i : nv - 1];
    }
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int64_t i = i0 + b * kBlock;
      if (i < nv) f(i, w[b]);
    }
  }
}

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

__device__ __forceinline__ double block_max(double v) {
  __shared__ double red[kWaves];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  return v;
}

__device__ __forceinline__ double block_min(double v) {
  __shared__ double red[kWaves];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  __syncthreads();
  return v;
}

// Chunk partials: L2 = fp64 sum of squares (fp16 / bf16: the fp32 square, exact); LINF = {max|x|, min|x|}
// with NaN carried as a count.
template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void k_dt_norm_partials(const typename T::S* __restrict__ x,
                                                             const adfl_slq_chunk* __restrict__ chunks,
                                                             double* __restrict__ partials) {
  using S = typename T::S;
  constexpr int V = kVec<T>;
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const Span sp = split_chunk<T>(c);
  double acc = 0.0, mx = 0.0, mn = __builtin_inf(), nan = 0.0;
  auto visit = [&](S raw) {
    const typename T::C v = T::load(raw);
    if (MODE == ADFL_NORM_L2) {
      acc += (double)(v * v);
    } else {
      const double a = fabs((double)v);
      if (a != a) nan = 1.0;
      mx = fmax(mx, a);
      mn = fmin(mn, a);
    }
  };
  for (int64_t g = c.start + threadIdx.x; g < sp.b0; g += kBlock) visit(x[g]);
  for_vectors(reinterpret_cast<const uint4*>(x + sp.b0), sp.nv, [&](int64_t, const uint4& w) {
    S vals[V];
    __builtin_memcpy(vals, &w, 16);
#pragma unroll
    for (int j = 0; j < V; ++j) visit(vals[j]);
  });
  for (int64_t g = sp.b1 + threadIdx.x; g < sp.end; g += kBlock) visit(x[g]);
  if (MODE == ADFL_NORM_L2) {
    acc = block_sum(acc);
    if (threadIdx.x == 0) partials[2 * blockIdx.x] = acc;
  } else {
    mx = block_max(mx);
    mn = block_min(mn);
    nan = block_max(nan);
    if (threadIdx.x == 0) {
      partials[2 * blockIdx.x] = nan != 0.0 ? (double)NAN : mx;
      partials[2 * blockIdx.x + 1] = nan != 0.0 ? (double)NAN : mn;
    }
  }
}

// Per tensor: one block per chunk, and the block of a tensor's first chunk reduces that tensor's partials
// (its 256 threads strided over the chunks, then a fixed tree: deterministic). A 1 GiB fp16 tensor has
// 65,536 chunks: one thread summing them in order would be a chain of dependent loads.
template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void k_dt_norm_finalize(const adfl_slq_chunk* __restrict__ chunks,
                                                             const double* __restrict__ partials,
                                                             double* __restrict__ norms, double* __restrict__ mins) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  if (c.first_chunk != (int32_t)blockIdx.x) return;  // block-uniform
  // Each thread's slots k = t, t + 256, ... in order, kU loads in flight (index clamped to the last slot,
  // absent slots masked): a plain `k < nchunks` loop waits on every load.
  constexpr int kU = 8;
  const int last = c.nchunks - 1;
  const double* p0 = partials + 2 * (int64_t)c.first_chunk;
  if (MODE == ADFL_NORM_L2) {
    double s = 0.0;
    for (int k0 = threadIdx.x; k0 <= last; k0 += kU * kBlock) {
      double p[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) p[u] = p0[2 * min(k0 + u * kBlock, last)];
#pragma unroll
      for (int u = 0; u < kU; ++u) s += k0 + u * kBlock <= last ? p[u] : 0.0;  // sums >= +0: adding +0 is exact
    }
    s = block_sum(s);
    if (threadIdx.x == 0) {
      if constexpr (sizeof(typename T::C) == 4) {
        const float n32 = __fsqrt_rn((float)s);  // fp32 sum, correctly rounded fp32 sqrt
        norms[c.tensor] = (double)T::rn(n32);
      } else {
        norms[c.tensor] = sqrt(s);
      }
    }
  } else {
    double mx = 0.0, mn = __builtin_inf(), nan = 0.0;
    for (int k0 = threadIdx.x; k0 <= last; k0 += kU * kBlock) {
      double a[kU], b[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int k = min(k0 + u * kBlock, last);  // repeats of the last slot are idempotent here
        a[u] = p0[2 * k];
        b[u] = p0[2 * k + 1];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (a[u] != a[u]) nan = 1.0;
        mx = fmax(mx, a[u]);
        mn = fmin(mn, b[u]);
      }
    }
    mx = block_max(mx);
    mn = block_min(mn);
    nan = block_max(nan);
    if (threadIdx.x == 0) {
      norms[c.tensor] = nan != 0.0 ? (double)NAN : mx;
      if (mins) mins[c.tensor] = nan != 0.0 ? (double)NAN : mn;
    }
  }
}

// Levels / exponents + signs from given per-tensor norms. Whole 16-byte vectors of x (V elements) per thread
// step, their V level bytes and V sign bytes stored together (8 B for fp16 / bf16, 2 B for fp64); the
// uniforms of a vector are one (fp64) or two (fp16 / bf16) Philox blocks. Head / tail elements one by one.
// CNAT's exponents do not depend on the norm: with `partials` set (CNAT only) the kernel takes no norms and
// writes the chunk's L2 partial instead, visiting the elements in k_dt_norm_partials' order (same sum), so the
// encode reads x once; k_dt_zero_fixup then applies the norm == 0 branch.
template <typename T, int KIND>
__global__ __launch_bounds__(kBlock) void k_dt_quantize(const typename T::S* __restrict__ x,
                                                        const adfl_slq_chunk* __restrict__ chunks, int bits,
                                                        const double* __restrict__ norms,
                                                        const typename T::S* __restrict__ inj, uint64_t seed,
                                                        uint64_t counter, uint8_t* __restrict__ levels,
                                                        int8_t* __restrict__ signs, double* __restrict__ partials) {
  using C = typename T::C;
  using S = typename T::S;
  constexpr int V = kVec<T>;
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const Span sp = split_chunk<T>(c);
  const bool fused = KIND == 2 && partials != nullptr;
  const C norm = fused ? (C)1 : (C)norms[c.tensor];
  if (norm == (C)0) {  // quant.py:227-228 / :368-369 / :513-514: u8 zeros, int8 ones
    for (int64_t g = c.start + threadIdx.x; g < sp.end; g += kBlock) {
      levels[g] = 0;
      signs[g] = 1;
    }
    return;
  }
  constexpr int kTab = KIND == 2 ? T::kBands : 1;
  __shared__ uint16_t s_below[kTab], s_above[kTab];
  if constexpr (KIND == 2) {
    for (int i = threadIdx.x; i < kTab; i += kBlock) {
      s_below[i] = T::below_tab()[i];
      s_above[i] = T::above_tab()[i];
    }
    __syncthreads();
  }
  const Bands tb{s_below, s_above};
  double acc = 0.0;
  auto one = [&](int64_t g) {
    const C u = inj ? T::load(inj[g]) : stream1<T>(seed, counter, g);
    const C v = T::load(x[g]);
    uint32_t sg;
    levels[g] = (uint8_t)encode_elem<T, KIND>(v, u, norm, bits, sg, tb);
    signs[g] = (int8_t)sg;
    if (fused) acc += (double)(v * v);
  };
  for (int64_t g = c.start + threadIdx.x; g < sp.b0; g += kBlock) one(g);
  for_vectors(reinterpret_cast<const uint4*>(x + sp.b0), sp.nv, [&](int64_t i, const uint4& w) {
    const int64_t g0 = sp.b0 + i * V;
    S vals[V];
    __builtin_memcpy(vals, &w, 16);
    C u[V];
    if (inj) {
#pragma unroll
      for (int j = 0; j < V; ++j) u[j] = T::load(inj[g0 + j]);
    } else if constexpr (V == 8) {
      C a[4], b2[4];
      stream4<T>(seed, counter, g0, a);
      stream4<T>(seed, counter, g0 + 4, b2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u[j] = a[j];
        u[4 + j] = b2[j];
      }
    } else {  // V == 2 (fp64): elements g0, g0 + 1 are words (x, y) and (z, w) of block counter + g0 / 2
      const uint4 q = adfl::philox4x32(counter + (uint64_t)(g0 >> 1), seed);
      u[0] = (double)((((uint64_t)q.x << 32) | q.y) >> 11) * 0x1p-53;
      u[1] = (double)((((uint64_t)q.z << 32) | q.w) >> 11) * 0x1p-53;
    }
    uint64_t lw = 0, sw = 0;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const C v = T::load(vals[j]);
      uint32_t sg;
      const uint32_t lb = encode_elem<T, KIND>(v, u[j], norm, bits, sg, tb);
      lw |= (uint64_t)lb << (8 * j);
      sw |= (uint64_t)sg << (8 * j);
      if (fused) acc += (double)(v * v);
    }
    if constexpr (V == 8) {
      *reinterpret_cast<uint64_t*>(levels + g0) = lw;
      *reinterpret_cast<uint64_t*>(signs + g0) = sw;
    } else {
      *reinterpret_cast<uint16_t*>(levels + g0) = (uint16_t)lw;
      *reinterpret_cast<uint16_t*>(signs + g0) = (uint16_t)sw;
    }
  });
  for (int64_t g = sp.b1 + threadIdx.x; g < sp.end; g += kBlock) one(g);
  if (fused) {  // block-uniform
    acc = block_sum(acc);
    if (threadIdx.x == 0) partials[2 * blockIdx.x] = acc;
  }
}

// CNAT norm == 0 after the fused encode (quant.py:513-514): one thread per chunk reads its tensor's norm; the
// wave then fills its zero-norm chunks one at a time, all 64 lanes on each (k_cnat_zero_fixup's shape).
__global__ __launch_bounds__(kBlock) void k_dt_zero_fixup(const adfl_slq_chunk* __restrict__ chunks, int64_t nchunks,
                                                          const double* __restrict__ norms,
                                                          uint8_t* __restrict__ levels, int8_t* __restrict__ signs) {
  const int64_t wave0 = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63);
  const int64_t ci = wave0 + (threadIdx.x & 63);
  uint64_t m = __ballot(ci < nchunks && norms[chunks[ci].tensor] == 0.0);
  while (m) {  // wave-uniform
    const int l = __builtin_ctzll(m);
    m &= m - 1;
    const adfl_slq_chunk c = chunks[wave0 + l];
    for (int64_t i = c.start + (threadIdx.x & 63); i < c.start + c.len; i += 64) {
      levels[i] = 0;
      signs[i] = 1;
    }
  }
}

// The stream's uniforms for elements start .. start+n-1, stored in the dtype (tests).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_dt_uniforms(typename T::S* __restrict__ out, int64_t n, int64_t start,
                                                        uint64_t seed, uint64_t counter) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int64_t g = start + i;
    typename T::C u[4];
    stream4<T>(seed, counter, g & ~(int64_t)3, u);
    const typename T::C v = u[g & 3];
    if constexpr (sizeof(typename T::S) == 8) {
      out[i] = v;
    } else {
      out[i] = (typename T::S)T::bits(v);
    }
  }
}

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <typename T>
int norms_t(const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int mode, void* d_ws, double* d_norms,
            double* d_mins, hipStream_t st) {
  const auto* x = static_cast<const typename T::S*>(d_x);
  double* part = static_cast<double*>(d_ws);
  const dim3 grid((unsigned)nchunks);
  if (mode == ADFL_NORM_L2) {
    hipLaunchKernelGGL((k_dt_norm_partials<T, ADFL_NORM_L2>), grid, dim3(kBlock), 0, st, x, d_chunks, part);
    hipLaunchKernelGGL((k_dt_norm_finalize<T, ADFL_NORM_L2>), grid, dim3(kBlock), 0, st, d_chunks, part, d_norms,
                       d_mins);
  } else {
    hipLaunchKernelGGL((k_dt_norm_partials<T, ADFL_NORM_LINF>), grid, dim3(kBlock), 0, st, x, d_chunks, part);
    hipLaunchKernelGGL((k_dt_norm_finalize<T, ADFL_NORM_LINF>), grid, dim3(kBlock), 0, st, d_chunks, part, d_norms,
                       d_mins);
  }
  return launch_status();
}

template <typename T>
int quantize_t(int codec, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
               const double* d_norms, const void* d_u, uint64_t seed, uint64_t counter, uint8_t* d_levels,
               int8_t* d_signs, hipStream_t st) {
  const auto* x = static_cast<const typename T::S*>(d_x);
  const auto* inj = static_cast<const typename T::S*>(d_u);
  if (codec == ADFL_CODEC_CNAT) {
    hipLaunchKernelGGL((k_dt_quantize<T, 2>), dim3((unsigned)nchunks), dim3(kBlock), 0, st, x, d_chunks, bits, d_norms,
                       inj, seed, counter, d_levels, d_signs, (double*)nullptr);
  } else {
    hipLaunchKernelGGL((k_dt_quantize<T, 0>), dim3((unsigned)nchunks), dim3(kBlock), 0, st, x, d_chunks, bits, d_norms,
                       inj, seed, counter, d_levels, d_signs, (double*)nullptr);
  }
  return launch_status();
}

// CNAT encode, x read once: exponents + signs + chunk partials, the per-tensor L2 finalize, the norm == 0 fix-up.
template <typename T>
int cnat_encode_t(const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits, const void* d_u,
                  uint64_t seed, uint64_t counter, void* d_ws, uint8_t* d_levels, int8_t* d_signs, double* d_norms,
                  hipStream_t st) {
  const auto* x = static_cast<const typename T::S*>(d_x);
  const auto* inj = static_cast<const typename T::S*>(d_u);
  double* part = static_cast<double*>(d_ws);
  const dim3 grid((unsigned)nchunks);
  hipLaunchKernelGGL((k_dt_quantize<T, 2>), grid, dim3(kBlock), 0, st, x, d_chunks, bits, (const double*)nullptr, inj,
                     seed, counter, d_levels, d_signs, part);
  hipLaunchKernelGGL((k_dt_norm_finalize<T, ADFL_NORM_L2>), grid, dim3(kBlock), 0, st, d_chunks, part, d_norms,
                     (double*)nullptr);
  hipLaunchKernelGGL(k_dt_zero_fixup, dim3((unsigned)((nchunks + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, d_chunks,
                     nchunks, d_norms, d_levels, d_signs);
  return launch_status();
}

int check_common(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks) {
  if (dtype != ADFL_DTYPE_F16 && dtype != ADFL_DTYPE_BF16 && dtype != ADFL_DTYPE_F64) return ADFL_E_ARG;
  if (!d_x || !d_chunks || nchunks < 1 || nchunks > INT32_MAX) return ADFL_E_ARG;
  if (!aligned16(d_x)) return ADFL_E_ALIGN;
  return 0;
}

}  // namespace

extern "C" {

int adfl_stoch_norms_batched_dt(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                int mode, void* d_workspace, int64_t workspace_bytes, double* d_norms, double* d_mins,
                                void* stream) {
  if (const int r = check_common(dtype, d_x, d_chunks, nchunks)) return r;
  if (!d_norms || !d_workspace) return ADFL_E_ARG;
  if (mode != ADFL_NORM_L2 && mode != ADFL_NORM_LINF) return ADFL_E_ARG;
  if (workspace_bytes < adfl_stoch_workspace_bytes(nchunks)) return ADFL_E_WORKSPACE;
  if (!aligned16(d_workspace)) return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADFL_DTYPE_F16) return norms_t<DtF16>(d_x, d_chunks, nchunks, mode, d_workspace, d_norms, d_mins, st);
  if (dtype == ADFL_DTYPE_BF16) return norms_t<DtBF16>(d_x, d_chunks, nchunks, mode, d_workspace, d_norms, d_mins, st);
  return norms_t<DtF64>(d_x, d_chunks, nchunks, mode, d_workspace, d_norms, d_mins, st);
}

int adfl_stoch_quantize_batched_dt(int32_t codec, int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks,
                                   int64_t nchunks, int bits, const double* d_norms, const void* d_uniforms,
                                   uint64_t seed, uint64_t counter, uint8_t* d_levels, int8_t* d_signs,
                                   void* stream) {
  if (const int r = check_common(dtype, d_x, d_chunks, nchunks)) return r;
  if (codec != ADFL_CODEC_QSGD && codec != ADFL_CODEC_RQSGD && codec != ADFL_CODEC_CNAT) return ADFL_E_ARG;
  if (bits < 1 || bits > 16) return ADFL_E_BITS;
  if (!d_norms || !d_levels || !d_signs) return ADFL_E_ARG;
  if ((d_uniforms && !aligned16(d_uniforms)) || !aligned16(d_levels) || !aligned16(d_signs)) return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADFL_DTYPE_F16)
    return quantize_t<DtF16>(codec, d_x, d_chunks, nchunks, bits, d_norms, d_uniforms, seed, counter, d_levels,
                             d_signs, st);
  if (dtype == ADFL_DTYPE_BF16)
    return quantize_t<DtBF16>(codec, d_x, d_chunks, nchunks, bits, d_norms, d_uniforms, seed, counter, d_levels,
                              d_signs, st);
  return quantize_t<DtF64>(codec, d_x, d_chunks, nchunks, bits, d_norms, d_uniforms, seed, counter, d_levels, d_signs,
                           st);
}

int adfl_stoch_encode_batched_dt(int32_t codec, int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks,
                                 int64_t nchunks, int bits, const void* d_uniforms, uint64_t seed, uint64_t counter,
                                 void* d_workspace, int64_t workspace_bytes, uint8_t* d_levels, int8_t* d_signs,
                                 double* d_norms, double* d_mins, void* stream) {
  if (codec == ADFL_CODEC_RQSGD && !d_mins) return ADFL_E_ARG;
  if (codec == ADFL_CODEC_CNAT) {  // the argument checks of the two calls below, then one read of x
    if (const int r = check_common(dtype, d_x, d_chunks, nchunks)) return r;
    if (bits < 1 || bits > 16) return ADFL_E_BITS;
    if (!d_norms || !d_workspace || !d_levels || !d_signs) return ADFL_E_ARG;
    if (workspace_bytes < adfl_stoch_workspace_bytes(nchunks)) return ADFL_E_WORKSPACE;
    if (!aligned16(d_workspace) || (d_uniforms && !aligned16(d_uniforms)) || !aligned16(d_levels) ||
        !aligned16(d_signs))
      return ADFL_E_ALIGN;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == ADFL_DTYPE_F16)
      return cnat_encode_t<DtF16>(d_x, d_chunks, nchunks, bits, d_uniforms, seed, counter, d_workspace, d_levels,
                                  d_signs, d_norms, st);
    if (dtype == ADFL_DTYPE_BF16)
      return cnat_encode_t<DtBF16>(d_x, d_chunks, nchunks, bits, d_uniforms, seed, counter, d_workspace, d_levels,
                                   d_signs, d_norms, st);
    return cnat_encode_t<DtF64>(d_x, d_chunks, nchunks, bits, d_uniforms, seed, counter, d_workspace, d_levels,
                                d_signs, d_norms, st);
  }
  const int mode = codec == ADFL_CODEC_RQSGD ? ADFL_NORM_LINF : ADFL_NORM_L2;
  if (const int r = adfl_stoch_norms_batched_dt(dtype, d_x, d_chunks, nchunks, mode, d_workspace, workspace_bytes,
                                                d_norms, d_mins, stream))
    return r;
  return adfl_stoch_quantize_batched_dt(codec, dtype, d_x, d_chunks, nchunks, bits, d_norms, d_uniforms, seed, counter,
                                        d_levels, d_signs, stream);
}

int adfl_philox_uniforms_dt(int32_t dtype, void* d_out, int64_t n, int64_t start, uint64_t seed, uint64_t counter,
                            void* stream) {
  if (dtype != ADFL_DTYPE_F16 && dtype != ADFL_DTYPE_BF16 && dtype != ADFL_DTYPE_F64) return ADFL_E_ARG;
  if (!d_out || n < 1 || start < 0) return ADFL_E_ARG;
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock < 4096 ? (n + kBlock - 1) / kBlock : 4096);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADFL_DTYPE_F16)
    hipLaunchKernelGGL(k_dt_uniforms<DtF16>, dim3(grid), dim3(kBlock), 0, st, static_cast<uint16_t*>(d_out), n, start,
                       seed, counter);
  else if (dtype == ADFL_DTYPE_BF16)
    hipLaunchKernelGGL(k_dt_uniforms<DtBF16>, dim3(grid), dim3(kBlock), 0, st, static_cast<uint16_t*>(d_out), n, start,
                       seed, counter);
  else
    hipLaunchKernelGGL(k_dt_uniforms<DtF64>, dim3(grid), dim3(kBlock), 0, st, static_cast<double*>(d_out), n, start,
                       seed, counter);
  return launch_status();
}

}  // extern "C"
