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
// Uniforms come from an in-register Philox4x32-7 stream (4 uniforms per 128-bit block, one block per
// float4 group: no uniform ever touches HBM) or from an injected plane (parity tests). Seven rounds is
// Random123's crush-resistant minimum for Philox4x32 (Salmon et al., SC'11: passes TestU01 BigCrush);
// the ten of curand's default buy margin, not quality these codecs can observe (their draws are compared
// with a threshold at 24-bit resolution), and each round is two quarter-rate 32x32->64 multiplies: 7 rounds
// cut the stream's VALU issue by 30%. Round function, constants and key schedule are
// Philox4x32's (pinned by the 10-round known-answer vectors in tests/test_stoch_golden.py).
//
// Numerics: no fast-math, -ffp-contract=off, IEEE fp32 denormals; divisions are correctly rounded
// (__fdiv_rn) because the reference divides element by element in fp32; CNAT's floor/ceil(log2) is the
// exact integer band rule of cnat_log2_table.h (no transcendental, no rounding risk).

#include <hip/hip_runtime.h>

#include <cstdint>

#include "adfl_stoch.h"
#include "cnat_log2_table.h"
#include "philox.h"
#include "torch_norm_walk.h"
#include "torch_sum_order.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int64_t kPartialBytes = 16;  // per chunk: fp64 sum of squares, or {max, min} |x| bits

// ------------------------------------------------------------------------------------------------
// uniforms
// ------------------------------------------------------------------------------------------------
using adfl::kPhiloxRounds;
using adfl::philox4x32;

__device__ __forceinline__ float u24(uint32_t w) { return (float)(w >> 8) * 0x1p-24f; }

// B independent Philox4x32 blocks with their rounds interleaved: a single block is a chain of dependent
// 64-bit multiply rounds, which with only 4-5 waves per SIMD leaves the VALU waiting on latency
// (tools/microbench_stoch_res.hip: 9.3 us of C3's resident QSGD encode); B chains in lockstep give the
// scheduler B independent instructions per step. Same words as philox4x32, bit for bit.
template <int B>
__device__ __forceinline__ void philox4x32_batch(const uint64_t (&ctr)[B], uint64_t seed, uint4 (&out)[B]) {
  uint32_t c0[B], c1[B], c2[B], c3[B];
#pragma unroll
  for (int i = 0; i < B; ++i) {
    c0[i] = (uint32_t)ctr[i];
    c1[i] = (uint32_t)(ctr[i] >> 32);
    c2[i] = 0;
    c3[i] = 0;
  }
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < kPhiloxRounds; ++r) {
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c0[i], p1 = (uint64_t)0xCD9E8D57u * c2[i];
      c0[i] = (uint32_t)(p1 >> 32) ^ c1[i] ^ k0;  // no v_xor3_b32 on gfx950: two v_xor_b32
      c1[i] = (uint32_t)p1;
      c2[i] = (uint32_t)(p0 >> 32) ^ c3[i] ^ k1;
      c3[i] = (uint32_t)p0;
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
#pragma unroll
  for (int i = 0; i < B; ++i) out[i] = make_uint4(c0[i], c1[i], c2[i], c3[i]);
}

struct Uniforms {
  const float* inj;  // injected plane (indexed like x) or null
  uint64_t seed, counter;

  // u for elements g .. g+3, g % 4 == 0
  __device__ __forceinline__ float4 group(int64_t g) const {
    if (inj) return *reinterpret_cast<const float4*>(inj + g);
    const uint4 w = philox4x32(counter + (uint64_t)(g >> 2), seed);
    return make_float4(u24(w.x), u24(w.y), u24(w.z), u24(w.w));
  }
  __device__ __forceinline__ float one(int64_t g) const {
    if (inj) return inj[g];
    const uint4 w = philox4x32(counter + (uint64_t)(g >> 2), seed);
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

// Every element rule below comes in two forms:
//  * an EXACT form — the reference's fp32 arithmetic, including every special case (NaN, inf, overflow,
//    caller-supplied tiny norms), with correctly rounded __fdiv_rn divisions;
//  * a FAST form — branch-free, the same result wherever it sets no `bad` flag. The kernels evaluate the
//    fast form for a float4 group, and if any lane of the wave flagged its group (a wave-uniform ballot)
//    that wave recomputes the flagged lanes with the exact form. Per-element exec-mask branching on rare
//    cases made the kernels issue-bound (267 saveexec / 196 branches for 32 elements per lane).
//
// Division. The fast form uses a per-tensor reciprocal (Markstein): y = RN(1/b), q = RN(a*y),
// r = RN(a - b*q) (exact), q' = RN(q + r*y) = RN(a/b) while every intermediate stays normal; it is valid
// for b in [2^-60, 2^60] (block-uniform) and |a| in {0} U [2^-60, 2^60]. 4.4 vs 12.1 lane-cycles per
// quotient, and 0 of 1.7e10 random operand pairs differ from __fdiv_rn (tools/microbench_stoch.hip,
// profiles/r01/microbench_stoch.txt).
struct Div {
  float b, y;
  bool fast;
};

__device__ __forceinline__ Div make_div(float b) {
  Div d;
  d.b = b;
  d.y = __fdiv_rn(1.0f, b);
  d.fast = b >= 0x1p-60f && b <= 0x1p60f;
  return d;
}

__device__ __forceinline__ float div_fast(float a, const Div& d, bool& bad) {
  const float aa = __builtin_fabsf(a);
  bad |= !(aa <= 0x1p60f && (aa >= 0x1p-60f || aa == 0.0f));
  const float q = a * d.y;
  const float r = __builtin_fmaf(-d.b, q, a);
  return __builtin_fmaf(r, d.y, q);  // +0 for a = +0 (a is never -0 on these paths)
}

// QSGD / RQSGD level (quant.py:230-236): s * |x| / norm in fp32, floor, stochastic round up, u8.
__device__ __forceinline__ uint32_t qsgd_level_exact(float x, float s, float norm, float u) {
  const float scaled = __fdiv_rn(s * __builtin_fabsf(x), norm);
  const float l = __builtin_floorf(scaled);
  return low_byte(l + (u < scaled - l ? 1.0f : 0.0f));
}

// Fast form: for 0 <= scaled < 2^24 (every level of bits <= 16 against its own norm) the floor is an
// integer truncation and l + 1 is exact in fp32.
__device__ __forceinline__ uint32_t qsgd_level_fast(float x, float s, const Div& d, float u, bool& bad) {
  const float scaled = div_fast(s * __builtin_fabsf(x), d, bad);
  bad |= !(scaled < 16777216.0f);                          // also catches NaN
  const float sc = __builtin_fminf(scaled, 16777215.0f);   // keep the conversion defined when flagged
  const int l = (int)sc;
  return (uint32_t)(l + (u < sc - (float)l ? 1 : 0)) & 0xffu;
}

__device__ __forceinline__ float pow2i(int k) {  // 2^k for k in [-126, 128] (128 -> inf), exact
  return __uint_as_float((uint32_t)(k + 127) << 23);
}

// CNAT exponent byte (quant.py:516-532). v = fl(|x| + eps) >= 2^-23 is normal, so its binary exponent e and
// the band table give floor / ceil of fl32(log2 v) exactly. Integer clamp and low byte = torch's float
// clamp_ then .to(int8) of an integral value.
__device__ __forceinline__ uint32_t cnat_exp_exact(float x, float u, int min_e, int max_e) {
  if (x == 0.0f) return (uint32_t)min_e & 0xffu;  // final_exponents[x == 0] = min_exp
  const float xa = __builtin_fabsf(x);
  const float v = xa + 0x1p-23f;
  if (__builtin_isnan(v)) return 0u;                        // ceil NaN, clamp keeps NaN, int8(NaN) = 0
  if (__builtin_isinf(v)) return (uint32_t)max_e & 0xffu;   // prob = NaN -> ceil = inf -> max_exp
  const uint32_t bits = __float_as_uint(v);
  const int e = (int)(bits >> 23) - 127;
  const uint32_t m = bits & 0x7fffffu;
  int f = e, c = e + 1;
  if (m <= kCnatBand[e - kCnatKMin].above) {
    c = e;
  } else if (0x800000u - m <= kCnatBand[e + 1 - kCnatKMin].below) {
    f = e + 1;
  }
  // (2^c - |x|) / 2^f: dividing by a power of two is exact here (the quotient is 0, normal or inf), so an
  // ldexp replaces the division; 2^128 = inf as a divisor (f = 128) makes the quotient NaN, as in torch.
  const float a = pow2i(c) - xa;
  const float prob = f < 128 ? __builtin_ldexpf(a, -f) : __builtin_nanf("");
  const int r = (u < prob) ? f : c;
  return (uint32_t)min(max(r, min_e), max_e) & 0xffu;
}

// Fast form: finite non-zero x whose mantissa is outside every power of two's band (no band is wider
// than kCnatMaxAbove / kCnatMaxBelow ulps): floor / ceil are e / e + 1. Zeros are handled inline.
// prob = (2^(e+1) - |x|) / 2^e is formed as 2 - |x| * 2^-e: both are exact scalings of one rounding of the
// same difference (every intermediate is normal on this path), so the bits are the exact form's, in two
// fewer instructions. The band test is one unsigned range check on the mantissa (m <= A or m >= 2^23 - B
// <=> (m + B) mod 2^23 <= A + B).
__device__ __forceinline__ uint32_t cnat_exp_fast(float x, float u, int min_e, int max_e, bool& bad) {
  const float xa = __builtin_fabsf(x);
  const float v = xa + 0x1p-23f;
  const uint32_t bits = __float_as_uint(v);
  const int ex = (int)(bits >> 23);
  const int e = ex - 127;
  bad |= (x != 0.0f) & (!(v < 0x1p127f) | (((bits + kCnatMaxBelow) & 0x7fffffu) <= kCnatMaxAbove + kCnatMaxBelow));
  const float prob = 2.0f - __builtin_ldexpf(xa, 127 - ex);
  int r = e + (u < prob ? 0 : 1);
  r = min(max(r, min_e), max_e);
  return (uint32_t)(x == 0.0f ? min_e : r) & 0xffu;
}

// decoders (d divides by levels)
__device__ __forceinline__ float qsgd_value_exact(uint32_t l, uint32_t sgn, float norm, float s) {
  return __fdiv_rn(norm * (float)l, s) * (float)(int8_t)sgn;
}

__device__ __forceinline__ float qsgd_value_fast(uint32_t l, uint32_t sgn, float norm, const Div& d, bool& bad) {
  return div_fast(norm * (float)l, d, bad) * (float)(int8_t)sgn;
}

__device__ __forceinline__ float rqsgd_value_exact(uint32_t l, uint32_t sgn, float norm, float mn, float s) {
  const float sf = (float)(int8_t)sgn;
  return l == 0u ? mn * sf : __fdiv_rn((norm * sf) * (float)l, s);
}

__device__ __forceinline__ float rqsgd_value_fast(uint32_t l, uint32_t sgn, float norm, float mn, const Div& d,
                                                  bool& bad) {
  const float sf = (float)(int8_t)sgn;
  bool b2 = false;
  const float v = div_fast((norm * sf) * (float)l, d, b2);
  bad |= b2 & (l != 0u);
  return l == 0u ? mn * sf : v;
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

// streaming (non-temporal) 16-byte load: x is read once per pass and must not evict the payload planes
__device__ __forceinline__ float4 load4_nt(const float4* p) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// elements [0, head) of a chunk are done one by one, up to the first 4-element boundary of the bucket
__device__ __forceinline__ int chunk_head4(int64_t start, int len) {
  const int h = (int)((4 - (start & 3)) & 3);
  return h < len ? h : len;
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
// Work layout: one block per chunk (<= 8192 elements; a 1 GiB tensor is 32768 blocks). Inside a chunk
// every thread first issues all its loads (at most kPer = 8192 / 4 / 256 = 8 float4 or plane dwords),
// then computes. Measured alternatives (profiles/r01/stoch_*): a loop that consumes each load before
// issuing the next is latency-bound; blocks that walk a range of chunks serialise them and were slower
// still (fresh blocks overlap one another's loads and compute).
constexpr int kPer = ADFL_SLQ_CHUNK_ELEMS / 4 / kBlock;
constexpr int kPbQuantize = 4;  // Philox blocks per batch in the multi-launch quantize kernels
constexpr int kPbResident = 2;  // ... and in the resident encodes (their VGPRs hold two chunks per lane)
// k_qsgd_encode_resident: sign bytes stored before the norm barrier (true) or with the levels (false). A/B on
// C3, tools/microbench_stoch_res.hip: 29.2 vs 28.5 us flushed — the product stores them with the levels.
constexpr bool kEarlySigns = false;
constexpr int64_t kKeepBytes = 192ll << 20;  // x tail the norm pass leaves in the Infinity Cache
constexpr int64_t kKeepChunks = kKeepBytes / (4 * ADFL_SLQ_CHUNK_ELEMS);

// Per-element head / tail of a chunk: the < 4 elements before the first 4-element boundary and after the
// last; thread t < head takes head element t, the next threads the tail elements. Returns -1 if none.
__device__ __forceinline__ int edge_elem_t(int t, int head, int tail, int len) {
  if (t < head) return t;
  return (t - head < len - tail) ? tail + t - head : -1;
}

__device__ __forceinline__ int edge_elem(int head, int tail, int len) { return edge_elem_t(threadIdx.x, head, tail, len); }

template <int MODE>
struct NormAcc {
  double s = 0.0;
  uint32_t mx = 0u, mn = 0xffffffffu;
  __device__ __forceinline__ void add(float v) {
    if (MODE == ADFL_NORM_L2) {
      s += sq(v);
    } else {
      mx = max(mx, abs_bits(v));
      mn = min(mn, abs_bits(v));
    }
  }
  __device__ __forceinline__ void add4(float4 v) {
    if (MODE == ADFL_NORM_L2) {
      s += (sq(v.x) + sq(v.y)) + (sq(v.z) + sq(v.w));
    } else {
      const uint32_t a = abs_bits(v.x), b = abs_bits(v.y), d = abs_bits(v.z), e = abs_bits(v.w);
      mx = max(mx, max(max(a, b), max(d, e)));
      mn = min(mn, min(min(a, b), min(d, e)));
    }
  }
  // block-reduce and write slot `ci` (every thread calls it: it synchronises)
  __device__ __forceinline__ void flush(void* partials, int64_t ci) {
    if (MODE == ADFL_NORM_L2) {
      const double r = block_sum(s);
      if (threadIdx.x == 0) reinterpret_cast<double*>(partials)[ci] = r;
    } else {
      const uint2 r = block_maxmin(mx, mn);
      if (threadIdx.x == 0) reinterpret_cast<uint2*>(partials)[ci] = r;
    }
    *this = NormAcc();
  }
};

// Norm partials, one block per chunk: the chunk's fp64 sum of fp32 squares (L2) or {max, min} |x| bits
// (LINF) into its slot. Fixed assignment and order: deterministic.
// Chunks from `keep_from` on are read with allocating loads, the rest non-temporally: the bucket's last
// kKeepBytes stay in the 256 MiB Infinity Cache for the quantize pass, which walks the chunks in reverse.
// A/B in the config bench (profiles/r01/stoch/keep_policy_ab.txt): 5% faster C3 encode than all
// non-temporal, 1% at C2.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_norm_partials(const float* __restrict__ x,
                                                          const adfl_slq_chunk* __restrict__ chunks,
                                                          int64_t keep_from, void* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  const int head = chunk_head4(c.start, c.len);
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
  const int n4 = (c.len - head) >> 2;
  const bool keep = (int64_t)blockIdx.x >= keep_from;
  float4 v[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = threadIdx.x + j * kBlock;
    if (k < n4) v[j] = keep ? x4[k] : load4_nt(x4 + k);
  }
  NormAcc<MODE> acc;
  const int i = edge_elem(head, head + (n4 << 2), c.len);
  if (i >= 0) acc.add(xc[i]);
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if ((int)threadIdx.x + j * kBlock < n4) acc.add4(v[j]);
  acc.flush(partials, blockIdx.x);
}

// Per-tensor finalize, one launch in two roles over the same table (every table entry is read by one thread, in
// parallel). Small tensors (<= kSmallChunks chunks): the thread that meets the first chunk sums the slots
// itself. Large tensors: a 1024-thread block sums them with 16 independent accumulators per thread,
// combined in a fixed tree. Both write norm = fp32 sqrt of the sum rounded once to fp32 (L2), or the
// max / min |x| with NaN propagated (LINF).
constexpr int kSmallChunks = 16;
constexpr int kBigBlock = 1024;

template <int MODE>
__device__ __forceinline__ void write_norm(const adfl_slq_chunk& c, double s, uint32_t mx, uint32_t mn,
                                           float* __restrict__ norms, float* __restrict__ mins) {
  if (MODE == ADFL_NORM_L2) {
    norms[c.tensor] = (float)__builtin_sqrt((double)(float)s);
  } else {
    const bool nan = mx > 0x7f800000u;  // NaN anywhere: torch's max and min both propagate it
    norms[c.tensor] = nan ? __builtin_nanf("") : __uint_as_float(mx);
    if (mins) mins[c.tensor] = nan ? __builtin_nanf("") : __uint_as_float(mn);
  }
}

template <int MODE>
__device__ __forceinline__ void finalize_small(const adfl_slq_chunk* __restrict__ chunks, int64_t nchunks,
                                               const void* __restrict__ partials, float* __restrict__ norms,
                                               float* __restrict__ mins, int64_t ci) {
  if (ci >= nchunks) return;
  const adfl_slq_chunk c = chunks[ci];
  if (c.first_chunk != ci || c.nchunks > kSmallChunks) return;
  // All kSmallChunks loads issued before the first use (the index clamped to the tensor's last slot), then
  // summed in slot order with the absent slots masked out: a loop of `k < c.nchunks` loads compiled to one
  // load + wait per slot, a chain of dependent memory latencies.
  const int last = c.nchunks - 1;
  double s = 0.0;
  uint32_t mx = 0u, mn = 0xffffffffu;
  if (MODE == ADFL_NORM_L2) {
    double p[kSmallChunks];
#pragma unroll
    for (int k = 0; k < kSmallChunks; ++k) p[k] = reinterpret_cast<const double*>(partials)[ci + min(k, last)];
#pragma unroll
    for (int k = 0; k < kSmallChunks; ++k) s += k <= last ? p[k] : 0.0;  // sums are >= +0: adding +0 is exact
  } else {
    uint2 p[kSmallChunks];
#pragma unroll
    for (int k = 0; k < kSmallChunks; ++k) p[k] = reinterpret_cast<const uint2*>(partials)[ci + min(k, last)];
#pragma unroll
    for (int k = 0; k < kSmallChunks; ++k) {  // repeats of the last slot change neither max nor min
      mx = max(mx, p[k].x);
      mn = min(mn, p[k].y);
    }
  }
  write_norm<MODE>(c, s, mx, mn, norms, mins);
}

// One launch for both: blocks [0, nsmall) take the small tensors (one table entry per thread), blocks
// [nsmall, ...) the large ones (a launch saved per encode; the empty role costs one table read).
template <int MODE>
__global__ __launch_bounds__(kBigBlock) void k_norm_finalize(const adfl_slq_chunk* __restrict__ chunks,
                                                             int64_t nchunks, int64_t nsmall,
                                                             const void* __restrict__ partials,
                                                             float* __restrict__ norms, float* __restrict__ mins) {
  if ((int64_t)blockIdx.x < nsmall) {
    finalize_small<MODE>(chunks, nchunks, partials, norms, mins, (int64_t)blockIdx.x * kBigBlock + threadIdx.x);
    return;
  }
  constexpr int U = 16, W = kBigBlock / 64;
  __shared__ int64_t firsts[kBigBlock];
  __shared__ int nfirst;
  __shared__ double red_s[W];
  __shared__ uint32_t red_mx[W], red_mn[W];
  if (threadIdx.x == 0) nfirst = 0;
  __syncthreads();
  const int64_t me = ((int64_t)blockIdx.x - nsmall) * kBigBlock + threadIdx.x;
  if (me < nchunks) {
    const adfl_slq_chunk c = chunks[me];
    if (c.first_chunk == me && c.nchunks > kSmallChunks) firsts[atomicAdd(&nfirst, 1)] = me;
  }
  __syncthreads();
  for (int f = 0; f < nfirst; ++f) {  // block-uniform loop; tensors are independent, so order is free
    const int64_t ci = firsts[f];
    const adfl_slq_chunk c = chunks[ci];
    double a[U];
    uint32_t mx = 0u, mn = 0xffffffffu;
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = 0.0;
    const int last = c.nchunks - 1;
    for (int k0 = threadIdx.x; k0 < c.nchunks; k0 += U * kBigBlock) {  // U loads in flight, as in finalize_small
      if (MODE == ADFL_NORM_L2) {
        double p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = reinterpret_cast<const double*>(partials)[ci + min(k0 + u * kBigBlock, last)];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += k0 + u * kBigBlock <= last ? p[u] : 0.0;
      } else {
        uint2 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = reinterpret_cast<const uint2*>(partials)[ci + min(k0 + u * kBigBlock, last)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          mx = max(mx, p[u].x);
          mn = min(mn, p[u].y);
        }
      }
    }
    double s = 0.0;
    if (MODE == ADFL_NORM_L2) {
#pragma unroll
      for (int w = U / 2; w > 0; w >>= 1)
#pragma unroll
        for (int u = 0; u < w; ++u) a[u] += a[u + w];
      s = a[0];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    } else {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
      }
    }
    if ((threadIdx.x & 63) == 0) {
      red_s[threadIdx.x >> 6] = s;
      red_mx[threadIdx.x >> 6] = mx;
      red_mn[threadIdx.x >> 6] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      uint32_t tx = 0u, tn = 0xffffffffu;
      for (int w = 0; w < W; ++w) {
        t += red_s[w];
        tx = max(tx, red_mx[w]);
        tn = min(tn, red_mn[w]);
      }
      write_norm<MODE>(c, t, tx, tn, norms, mins);
    }
    __syncthreads();
  }
}

// torch.linalg.vector_norm(x, ord=2) bit for bit as torch 2.10's CPU kernel computes it (the reference's
// QSGD / CNAT norm, quant.py:226,512; restated and pinned to every golden norm in oracle/slq_oracle.c
// oracle_torch_l2_norm): 8 fp32 lane accumulators acc[j] = fma(x[8i+j], x[8i+j], acc[j]) over i in order,
// a left-to-right sum of the 8 lanes, then the n % 8 tail with fma; below 8 elements plain b + x*x.
// The chains are sequential (n / 8 dependent FMAs per lane): ADFL_NORM_L2_TORCH runs one block per tensor
// (adfl_tn::k_norm_walk: four waves stream the tensor through LDS ahead of the FMA chain); the tile-parallel
// phased kernels (adfl_torch_norms, torch_norm.hip) give the same bits for long tensors.
__device__ __forceinline__ void fill_zero_norm(uint8_t* __restrict__ lv, int8_t* __restrict__ sg, int len,
                                               int t = threadIdx.x) {
  for (int i = t; i < len; i += kBlock) {
    lv[i] = 0;
    sg[i] = 1;
  }
}

__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }

// Quantize a chunk's float4 groups held in registers: v[j] is group tg + j * kBlock of the chunk (tg = the
// thread's index in its 256-thread group). Per group the level / exponent bytes (fast form; exact form for
// the wave if any lane flagged its group) and the sign bytes, stored as one dword each (contiguous across
// the wave). `all_exact` is uniform over the group.
// Philox uniforms are generated PB groups at a time (philox4x32_batch); injected uniforms (a test path)
// are loaded group by group.
// pre (LDS, or null): Philox words generated ahead of time, group j's at pre[j * pre_stride]. s4 null: the
// caller stores the sign bytes itself.
template <int PB, class F, class E, class A>
__device__ __forceinline__ void quantize_regs(const float4 (&v)[kPer], int tg, int n4, int64_t g0, const Uniforms& U,
                                              uint32_t* __restrict__ l4, uint32_t* __restrict__ s4, F fast, E exact,
                                              bool all_exact, A* acc, const uint4* pre = nullptr,
                                              int pre_stride = 0) {
  static_assert(kPer % PB == 0, "batches tile a chunk's groups");
#pragma unroll
  for (int jb = 0; jb < kPer; jb += PB) {
    if (jb * kBlock >= n4) break;  // group-uniform: no thread has group jb or later
    uint4 w[PB];
    if (!U.inj && pre) {
#pragma unroll
      for (int i = 0; i < PB; ++i) w[i] = pre[(jb + i) * pre_stride];
    } else if (!U.inj) {
      uint64_t ctr[PB];
#pragma unroll
      for (int i = 0; i < PB; ++i) ctr[i] = U.counter + (uint64_t)((g0 >> 2) + tg + (jb + i) * kBlock);
      philox4x32_batch(ctr, U.seed, w);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int j = jb + i;
      const int k = tg + j * kBlock;
      if (j * kBlock >= n4) break;  // group-uniform
      const bool live = k < n4;
      float4 uj;
      if (!U.inj)
        uj = make_float4(u24(w[i].x), u24(w[i].y), u24(w[i].z), u24(w[i].w));
      else
        uj = U.group(g0 + 4 * (int64_t)(live ? k : 0));
      bool bad = all_exact;
      uint32_t q = pack4(fast(v[j].x, uj.x, bad), fast(v[j].y, uj.y, bad), fast(v[j].z, uj.z, bad),
                         fast(v[j].w, uj.w, bad));
      // the whole wave takes the exact form when any live lane flagged (equal results where the fast form
      // holds): `bad` is then only a wave-wide OR of compare masks, never a per-lane value
      if (wave_any(bad && live))
        q = pack4(exact(v[j].x, uj.x), exact(v[j].y, uj.y), exact(v[j].z, uj.z), exact(v[j].w, uj.w));
      if (live) {
        l4[k] = q;
        if (s4) s4[k] = pack4(sign_byte(v[j].x), sign_byte(v[j].y), sign_byte(v[j].z), sign_byte(v[j].w));
        if (acc) acc->add4(v[j]);
      }
    }
  }
}

__device__ __forceinline__ void load_chunk_regs(const float4* __restrict__ x4, int n4, int tg, float4 (&v)[kPer]) {
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = tg + j * kBlock;
    if (k < n4) v[j] = load4_nt(x4 + k);
  }
}

// The vector part of a quantize chunk: x loaded up front, then quantize_regs.
template <int PB, class F, class E, class A>
__device__ __forceinline__ void quantize_chunk_vec(const float4* __restrict__ x4, int n4, int64_t g0, const Uniforms& U,
                                                   uint32_t* __restrict__ l4, uint32_t* __restrict__ s4, F fast,
                                                   E exact, bool all_exact, A* acc) {
  float4 v[kPer];
  load_chunk_regs(x4, n4, threadIdx.x, v);
  quantize_regs<PB>(v, threadIdx.x, n4, g0, U, l4, s4, fast, exact, all_exact, acc);
}

// PB: Philox blocks generated per batch (philox4x32_batch); the product's choice is kPbQuantize.
template <int PB>
__global__ __launch_bounds__(kBlock) void k_qsgd_quantize(const float* __restrict__ x,
                                                          const adfl_slq_chunk* __restrict__ chunks, float s,
                                                          const float* __restrict__ norms, Uniforms U,
                                                          uint8_t* __restrict__ levels, int8_t* __restrict__ signs) {
  const adfl_slq_chunk c = chunks[gridDim.x - 1 - blockIdx.x];  // reverse: start on the cached tail of x
  const float norm = norms[c.tensor];
  uint8_t* lv = levels + c.start;
  int8_t* sg = signs + c.start;
  if (norm == 0.0f) {  // quant.py:227-228
    fill_zero_norm(lv, sg, c.len);
    return;
  }
  const Div d = make_div(norm);
  const float* xc = x + c.start;
  const int head = chunk_head4(c.start, c.len);
  const int n4 = (c.len - head) >> 2;
  const auto fast = [&](float xv, float uv, bool& bad) { return qsgd_level_fast(xv, s, d, uv, bad); };
  const auto exact = [&](float xv, float uv) { return qsgd_level_exact(xv, s, norm, uv); };
  quantize_chunk_vec<PB>(reinterpret_cast<const float4*>(xc + head), n4, c.start + head, U,
                         reinterpret_cast<uint32_t*>(lv + head), reinterpret_cast<uint32_t*>(sg + head), fast, exact,
                         !d.fast, (NormAcc<ADFL_NORM_L2>*)nullptr);
  const int i = edge_elem(head, head + (n4 << 2), c.len);
  if (i >= 0) {
    lv[i] = (uint8_t)exact(xc[i], U.one(c.start + i));
    sg[i] = (int8_t)sign_byte(xc[i]);
  }
}

// CNAT: exponents + signs + the chunk's L2 partial in one read of x.
template <int PB>
__global__ __launch_bounds__(kBlock) void k_cnat_quantize(const float* __restrict__ x,
                                                          const adfl_slq_chunk* __restrict__ chunks, int min_e,
                                                          int max_e, Uniforms U, int8_t* __restrict__ exps,
                                                          int8_t* __restrict__ signs, double* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  int8_t* ex = exps + c.start;
  int8_t* sg = signs + c.start;
  const int head = chunk_head4(c.start, c.len);
  const int n4 = (c.len - head) >> 2;
  const auto fast = [=](float xv, float uv, bool& bad) { return cnat_exp_fast(xv, uv, min_e, max_e, bad); };
  const auto exact = [=](float xv, float uv) { return cnat_exp_exact(xv, uv, min_e, max_e); };
  NormAcc<ADFL_NORM_L2> acc;
  quantize_chunk_vec<PB>(reinterpret_cast<const float4*>(xc + head), n4, c.start + head, U,
                         reinterpret_cast<uint32_t*>(ex + head), reinterpret_cast<uint32_t*>(sg + head), fast, exact,
                         false, &acc);
  const int i = edge_elem(head, head + (n4 << 2), c.len);
  if (i >= 0) {
    const float v = xc[i];
    ex[i] = (int8_t)exact(v, U.one(c.start + i));
    sg[i] = (int8_t)sign_byte(v);
    acc.add(v);
  }
  acc.flush(partials, blockIdx.x);
}

// CNAT norm == 0 (an all-zero tensor): the reference returns u8 zeros and int8 ones (quant.py:513-514).
// One THREAD per chunk checks its tensor's norm; a wave then fills its zero-norm chunks one at a time, all
// 64 lanes on each. Nearly every launch only reads a norm per chunk and exits: one block per chunk made it
// a launch of 32,768 tiny dependent read chains at C2 (7.8-8.2 us at 256 or 64 threads per block,
// profiles/r03/rocprof_head/stoch_kernel_stats.csv); here it is 128 blocks.
__global__ __launch_bounds__(kBlock) void k_cnat_zero_fixup(const adfl_slq_chunk* __restrict__ chunks,
                                                            int64_t nchunks, const float* __restrict__ norms,
                                                            int8_t* __restrict__ exps, int8_t* __restrict__ signs) {
  const int64_t wave0 = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63);
  const int64_t ci = wave0 + (threadIdx.x & 63);
  const bool zero = ci < nchunks && norms[chunks[ci].tensor] == 0.0f;
  uint64_t m = __ballot(zero);
  while (m) {  // wave-uniform: the wave's zero-norm chunks, lowest lane first
    const int l = __builtin_ctzll(m);
    m &= m - 1;
    const adfl_slq_chunk c = chunks[wave0 + l];
    uint8_t* lv = reinterpret_cast<uint8_t*>(exps) + c.start;
    int8_t* sg = signs + c.start;
    for (int i = threadIdx.x & 63; i < c.len; i += 64) {
      lv[i] = 0;
      sg[i] = 1;
    }
  }
}

// ---- one-launch encodes of a bucket of small tensors (a whole tensor per 1024-thread block) -------------
// When every tensor of the bucket has at most ADFL_SLQ_RESIDENT_CHUNKS (8) chunks (the work list of
// adfl_slq_build_encode_work holds each tensor's first chunk), one 1024-thread block takes one whole
// tensor — 4 groups of 256 threads, group g takes chunks g and g + 4 — so the tensor's norm is a block
// reduction and the encode is ONE launch instead of three:
//  * QSGD / RQSGD (k_qsgd_encode_resident): the levels need the norm, so the block holds its whole tensor
//    in VGPRs (16 float4 per lane), reduces the norm, then quantizes from the registers: x read once
//    (6 B per element instead of 10);
//  * CNAT (k_cnat_encode_resident): the exponents do not depend on the norm, so each group streams its
//    chunks as k_cnat_quantize does (exponents + signs stored as they are made), and only an all-zero
//    norm rewrites the tensor's bytes after the reduction — no finalize and no fix-up launch.
// The outputs equal the multi-launch path's bit for bit: each group forms its chunks' L2 partials with
// the same 256-thread arithmetic as k_norm_partials (QSGD: edge element first) or k_cnat_quantize (CNAT:
// edge element last), the partials are summed in chunk order from 0.0 as finalize_small does, and the
// Philox groups are indexed by bucket element as everywhere else.
constexpr int kResBlock = 1024;
constexpr int kResGroups = kResBlock / kBlock;                        // 4
constexpr int kResPerGroup = ADFL_SLQ_RESIDENT_CHUNKS / kResGroups;  // 2
constexpr int kResWaves = kResBlock / 64;
static_assert(kResPerGroup * kResGroups == ADFL_SLQ_RESIDENT_CHUNKS, "groups cover a resident tensor");
static_assert(ADFL_SLQ_RESIDENT_CHUNKS <= kSmallChunks, "partials summed in finalize_small's order");

// The block's L2 norm from the per-wave partial sums red[r][wave] of chunk grp + 4r: each chunk's
// partial as block_sum forms it over its group's 4 waves, summed in chunk order (finalize_small).
__device__ __forceinline__ float resident_l2(const double (&red)[kResPerGroup][kResWaves], int nchunks) {
  double t = 0.0;
  for (int kc = 0; kc < nchunks; ++kc) {
    const double* p = &red[kc / kResGroups][(kc % kResGroups) * kWaves];
    t += (p[0] + p[1]) + (p[2] + p[3]);
  }
  return (float)__builtin_sqrt((double)(float)t);
}

// EARLY_SIGNS: the sign bytes (which do not depend on the norm) are stored while the loads drain, before the
// block's norm barrier, instead of after it with the levels.
template <int MODE, int PB, bool EARLY_SIGNS>  // MODE ADFL_NORM_L2 (QSGD) or ADFL_NORM_LINF (RQSGD)
__global__ __launch_bounds__(kResBlock) void k_qsgd_encode_resident(
    const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, const int32_t* __restrict__ work,
    float lev, Uniforms U, uint8_t* __restrict__ levels, int8_t* __restrict__ signs, float* __restrict__ norms,
    float* __restrict__ mins) {
  __shared__ double red_s[kResPerGroup][kResWaves];
  __shared__ uint32_t red_mx[kResWaves], red_mn[kResWaves];
  __shared__ uint4 pre[kPer][kResBlock];  // 128 KiB: the first chunk's Philox words, made while x streams in
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk ct = chunks[ci];
  if (ct.nchunks > ADFL_SLQ_RESIDENT_CHUNKS) {  // not a resident work list: NaN norm, nothing written
    if (threadIdx.x == 0) norms[ct.tensor] = __builtin_nanf("");
    return;
  }
  // group and wave are wave-uniform: in SGPRs, so the chunk metadata below is scalar
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x / kBlock);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = threadIdx.x % kBlock, lane = threadIdx.x & 63;
  float4 v[kResPerGroup][kPer];
  float ev[kResPerGroup];
  int ei[kResPerGroup], n4s[kResPerGroup];
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    ei[r] = -1;
    n4s[r] = 0;
    ev[r] = 0.0f;
    if (kc < ct.nchunks) {  // group-uniform
      const adfl_slq_chunk c = chunks[ci + kc];
      const int head = chunk_head4(c.start, c.len);
      n4s[r] = (c.len - head) >> 2;
      load_chunk_regs(reinterpret_cast<const float4*>(x + c.start + head), n4s[r], tg, v[r]);
      ei[r] = edge_elem_t(tg, head, head + (n4s[r] << 2), c.len);
      if (ei[r] >= 0) ev[r] = x[c.start + ei[r]];
    }
  }
  // The quantize needs the norm, so without this the Philox work of the whole tensor would sit between the
  // norm and the stores (about a third of the kernel on C3, tools/microbench_stoch_res.hip). Made here it
  // overlaps the loads in flight; the first chunk's share fits the LDS (the second chunk's is made later).
  if (!U.inj && grp < ct.nchunks) {
    const adfl_slq_chunk c = chunks[ci + grp];
    const int64_t q0 = (c.start + chunk_head4(c.start, c.len)) >> 2;
#pragma unroll
    for (int jb = 0; jb < kPer; jb += PB) {
      if (jb * kBlock >= n4s[0]) break;  // group-uniform
      uint64_t ctr[PB];
      uint4 w[PB];
#pragma unroll
      for (int i = 0; i < PB; ++i) ctr[i] = U.counter + (uint64_t)(q0 + tg + (jb + i) * kBlock);
      philox4x32_batch(ctr, U.seed, w);
#pragma unroll
      for (int i = 0; i < PB; ++i) pre[jb + i][threadIdx.x] = w[i];
    }
  }
  if (EARLY_SIGNS) {
#pragma unroll
    for (int r = 0; r < kResPerGroup; ++r) {
      const int kc = grp + r * kResGroups;
      if (kc >= ct.nchunks) continue;  // group-uniform
      const adfl_slq_chunk c = chunks[ci + kc];
      int8_t* sg = signs + c.start;
      uint32_t* s4 = reinterpret_cast<uint32_t*>(sg + chunk_head4(c.start, c.len));
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int k = tg + j * kBlock;
        if (k < n4s[r])
          s4[k] = pack4(sign_byte(v[r][j].x), sign_byte(v[r][j].y), sign_byte(v[r][j].z), sign_byte(v[r][j].w));
      }
      if (ei[r] >= 0) sg[ei[r]] = (int8_t)sign_byte(ev[r]);
    }
  }
  float norm, mn = 0.0f;
  if (MODE == ADFL_NORM_LINF) {  // max / min |x|: order-free
    uint32_t mx = 0u, mi = 0xffffffffu;
#pragma unroll
    for (int r = 0; r < kResPerGroup; ++r) {
      if (ei[r] >= 0) {
        mx = max(mx, abs_bits(ev[r]));
        mi = min(mi, abs_bits(ev[r]));
      }
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (tg + j * kBlock < n4s[r]) {
          const float4 a = v[r][j];
          mx = max(mx, max(max(abs_bits(a.x), abs_bits(a.y)), max(abs_bits(a.z), abs_bits(a.w))));
          mi = min(mi, min(min(abs_bits(a.x), abs_bits(a.y)), min(abs_bits(a.z), abs_bits(a.w))));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      mi = min(mi, (uint32_t)__shfl_xor((int)mi, o, 64));
    }
    if (lane == 0) {
      red_mx[wave] = mx;
      red_mn[wave] = mi;
    }
    __syncthreads();
    mx = red_mx[0];
    mi = red_mn[0];
#pragma unroll
    for (int w = 1; w < kResWaves; ++w) {
      mx = max(mx, red_mx[w]);
      mi = min(mi, red_mn[w]);
    }
    const bool nan = mx > 0x7f800000u;
    norm = nan ? __builtin_nanf("") : __uint_as_float(mx);
    mn = nan ? __builtin_nanf("") : __uint_as_float(mi);
  } else {  // L2: k_norm_partials' per-chunk arithmetic (edge element first)
#pragma unroll
    for (int r = 0; r < kResPerGroup; ++r) {
      double a = 0.0;
      if (ei[r] >= 0) a += sq(ev[r]);
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (tg + j * kBlock < n4s[r]) a += (sq(v[r][j].x) + sq(v[r][j].y)) + (sq(v[r][j].z) + sq(v[r][j].w));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
      if (lane == 0) red_s[r][wave] = a;
    }
    __syncthreads();
    norm = resident_l2(red_s, ct.nchunks);
  }
  if (threadIdx.x == 0) {
    norms[ct.tensor] = norm;
    if (MODE == ADFL_NORM_LINF) mins[ct.tensor] = mn;
  }
  const Div d = make_div(norm);
  const auto fast = [&](float xv, float uv, bool& bad) { return qsgd_level_fast(xv, lev, d, uv, bad); };
  const auto exact = [&](float xv, float uv) { return qsgd_level_exact(xv, lev, norm, uv); };
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    if (kc >= ct.nchunks) continue;  // group-uniform
    const adfl_slq_chunk c = chunks[ci + kc];
    uint8_t* lv = levels + c.start;
    int8_t* sg = signs + c.start;
    if (norm == 0.0f) {  // quant.py:227-228
      fill_zero_norm(lv, sg, c.len, tg);
      continue;
    }
    const int head = chunk_head4(c.start, c.len);
    quantize_regs<PB>(v[r], tg, n4s[r], c.start + head, U, reinterpret_cast<uint32_t*>(lv + head),
                      EARLY_SIGNS ? nullptr : reinterpret_cast<uint32_t*>(sg + head), fast, exact, !d.fast,
                      (NormAcc<ADFL_NORM_L2>*)nullptr, r == 0 ? &pre[0][threadIdx.x] : nullptr, kResBlock);
    if (ei[r] >= 0) {
      lv[ei[r]] = (uint8_t)exact(ev[r], U.one(c.start + ei[r]));
      if (!EARLY_SIGNS) sg[ei[r]] = (int8_t)sign_byte(ev[r]);
    }
  }
}

template <int PB>
__global__ __launch_bounds__(kResBlock) void k_cnat_encode_resident(
    const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, const int32_t* __restrict__ work,
    int min_e, int max_e, Uniforms U, int8_t* __restrict__ exps, int8_t* __restrict__ signs,
    float* __restrict__ norms) {
  __shared__ double red_s[kResPerGroup][kResWaves];
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk ct = chunks[ci];
  if (ct.nchunks > ADFL_SLQ_RESIDENT_CHUNKS) {  // not a resident work list: NaN norm, nothing written
    if (threadIdx.x == 0) norms[ct.tensor] = __builtin_nanf("");
    return;
  }
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x / kBlock);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = threadIdx.x % kBlock, lane = threadIdx.x & 63;
  const auto fast = [=](float xv, float uv, bool& bad) { return cnat_exp_fast(xv, uv, min_e, max_e, bad); };
  const auto exact = [=](float xv, float uv) { return cnat_exp_exact(xv, uv, min_e, max_e); };
  // both chunks' loads issued up front: the second chunk streams in while the first one is quantized
  float4 v[kResPerGroup][kPer];
  int n4s[kResPerGroup];
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    n4s[r] = 0;
    if (kc < ct.nchunks) {  // group-uniform
      const adfl_slq_chunk c = chunks[ci + kc];
      const int head = chunk_head4(c.start, c.len);
      n4s[r] = (c.len - head) >> 2;
      load_chunk_regs(reinterpret_cast<const float4*>(x + c.start + head), n4s[r], tg, v[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {  // k_cnat_quantize per chunk, its partial kept in LDS
    const int kc = grp + r * kResGroups;
    NormAcc<ADFL_NORM_L2> acc;
    if (kc < ct.nchunks) {
      const adfl_slq_chunk c = chunks[ci + kc];
      const float* xc = x + c.start;
      int8_t* ex = exps + c.start;
      int8_t* sg = signs + c.start;
      const int head = chunk_head4(c.start, c.len);
      quantize_regs<PB>(v[r], tg, n4s[r], c.start + head, U, reinterpret_cast<uint32_t*>(ex + head),
                        reinterpret_cast<uint32_t*>(sg + head), fast, exact, false, &acc);
      const int i = edge_elem_t(tg, head, head + (n4s[r] << 2), c.len);
      if (i >= 0) {
        const float e = xc[i];
        ex[i] = (int8_t)exact(e, U.one(c.start + i));
        sg[i] = (int8_t)sign_byte(e);
        acc.add(e);
      }
    }
    double a = acc.s;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (lane == 0) red_s[r][wave] = a;
  }
  __syncthreads();  // also orders this block's byte stores before the zero-norm rewrite below
  const float norm = resident_l2(red_s, ct.nchunks);
  if (threadIdx.x == 0) norms[ct.tensor] = norm;
  if (norm != 0.0f) return;  // block-uniform
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {  // quant.py:513-514: u8 zeros, int8 ones
    const int kc = grp + r * kResGroups;
    if (kc >= ct.nchunks) continue;
    const adfl_slq_chunk c = chunks[ci + kc];
    fill_zero_norm(reinterpret_cast<uint8_t*>(exps) + c.start, signs + c.start, c.len, tg);
  }
}

__device__ __forceinline__ void store4_nt(float4* p, float4 d) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v v = {d.x, d.y, d.z, d.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
}

// Decoders. KIND 0 = QSGD, 1 = RQSGD, 2 = CNAT.
template <int KIND>
__device__ __forceinline__ float decode_exact(uint32_t l, uint32_t sgn, float norm, float mn, float s) {
  if (KIND == 0) return qsgd_value_exact(l, sgn, norm, s);
  if (KIND == 1) return rqsgd_value_exact(l, sgn, norm, mn, s);
  return cnat_value(l, sgn, norm);
}

template <int KIND>
__device__ __forceinline__ float decode_fast(uint32_t l, uint32_t sgn, float norm, float mn, const Div& d, bool& bad) {
  if (KIND == 0) return qsgd_value_fast(l, sgn, norm, d, bad);
  if (KIND == 1) return rqsgd_value_fast(l, sgn, norm, mn, d, bad);
  return cnat_value(l, sgn, norm);
}

// Four decoded values from one dword of levels and one of signs. The fast division path falls back to the
// exact one for the whole wave if any live lane's quotient is in doubt (every lane must call this).
template <int KIND>
__device__ __forceinline__ float4 decode4(uint32_t l, uint32_t g, float norm, float mn, const Div& d, float s,
                                          bool live) {
  bool bad = KIND != 2 && !d.fast;
  float4 r;
  r.x = decode_fast<KIND>(l & 0xffu, g & 0xffu, norm, mn, d, bad);
  r.y = decode_fast<KIND>((l >> 8) & 0xffu, (g >> 8) & 0xffu, norm, mn, d, bad);
  r.z = decode_fast<KIND>((l >> 16) & 0xffu, (g >> 16) & 0xffu, norm, mn, d, bad);
  r.w = decode_fast<KIND>(l >> 24, g >> 24, norm, mn, d, bad);
  if (KIND != 2 && wave_any(bad && live)) {
    r.x = decode_exact<KIND>(l & 0xffu, g & 0xffu, norm, mn, s);
    r.y = decode_exact<KIND>((l >> 8) & 0xffu, (g >> 8) & 0xffu, norm, mn, s);
    r.z = decode_exact<KIND>((l >> 16) & 0xffu, (g >> 16) & 0xffu, norm, mn, s);
    r.w = decode_exact<KIND>(l >> 24, g >> 24, norm, mn, s);
  }
  return r;
}

// Decode in wave tiles of 1024 elements, the SLQ decode's shape (slq_codec.hip dequantize_tile): lane l
// loads 16 level bytes and 16 sign bytes (16-byte accesses, 1 KiB per wave-instruction per plane), a 1 KiB
// per-wave LDS transpose per plane hands lane l dwords j*64+l (j = 0..3), and the four float4 results are
// 16-byte stores contiguous across the wave. A wave issues all its tiles' loads (at most 2 per chunk)
// before consuming the first. The < 16 elements before the first 16-element boundary and the < 1024 after
// the last whole tile go per dword / per element. Measured on C2 (2^28 elements): 4-byte plane loads per
// lane, the previous shape, decoded QSGD in 0.303 ms and CNAT in 0.325 ms (0.66 / 0.62 of 8 TB/s at 6 B
// per element).
constexpr int kDecTile = 1024;
constexpr int kDecTilesPerWave = ADFL_SLQ_CHUNK_ELEMS / kDecTile / kWaves;

template <int KIND>
__global__ __launch_bounds__(kBlock) void k_stoch_dequantize(const uint8_t* __restrict__ levels,
                                                             const int8_t* __restrict__ signs,
                                                             const adfl_slq_chunk* __restrict__ chunks,
                                                             const float* __restrict__ norms,
                                                             const float* __restrict__ mins, float s,
                                                             float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][2][kDecTile / 4];
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float norm = norms[c.tensor];
  const float mn = KIND == 1 ? mins[c.tensor] : 0.0f;
  float* oc = out + c.start;
  if (norm == 0.0f) {  // quant.py:248-249 / :390-391 / :542-543
    for (int i = threadIdx.x; i < c.len; i += kBlock) oc[i] = 0.0f;
    return;
  }
  const Div d = make_div(s);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint8_t* lv = levels + c.start;
  const uint8_t* sg = reinterpret_cast<const uint8_t*>(signs) + c.start;
  const int h16 = (int)((16 - (c.start & 15)) & 15);
  const int head = h16 < c.len ? h16 : c.len;
  const int ntiles = (c.len - head) / kDecTile;
  // two tiles per wave at most (named registers: an indexed array here was promoted to LDS by the compiler)
  static_assert(kDecTilesPerWave == 2, "k_stoch_dequantize: one chunk is two tiles per wave");
  const int t0 = wave, t1 = wave + kWaves;
  uint4 L0, G0, L1, G1;
  if (t0 < ntiles) {
    L0 = reinterpret_cast<const uint4*>(lv + head + t0 * kDecTile)[lane];
    G0 = reinterpret_cast<const uint4*>(sg + head + t0 * kDecTile)[lane];
  }
  if (t1 < ntiles) {
    L1 = reinterpret_cast<const uint4*>(lv + head + t1 * kDecTile)[lane];
    G1 = reinterpret_cast<const uint4*>(sg + head + t1 * kDecTile)[lane];
  }
  auto tile = [&](int t, const uint4& L, const uint4& G) {
    reinterpret_cast<uint4*>(lds[wave][0])[lane] = L;
    reinterpret_cast<uint4*>(lds[wave][1])[lane] = G;
    __builtin_amdgcn_wave_barrier();
    uint32_t lw[4], gw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lw[j] = lds[wave][0][j * 64 + lane];
      gw[j] = lds[wave][1][j * 64 + lane];
    }
    __builtin_amdgcn_wave_barrier();
    float4* o4 = reinterpret_cast<float4*>(oc + head + t * kDecTile);
#pragma unroll
    for (int j = 0; j < 4; ++j) store4_nt(o4 + j * 64 + lane, decode4<KIND>(lw[j], gw[j], norm, mn, d, s, true));
  };
  if (t0 < ntiles) tile(t0, L0, G0);  // wave-uniform
  if (t1 < ntiles) tile(t1, L1, G1);
  // after the last whole tile: < 1024 elements, one dword of each plane per thread
  const int rs = head + ntiles * kDecTile;
  const int n4 = (c.len - rs) >> 2;
  if (n4 > 0) {  // block-uniform
    const int k = threadIdx.x;
    const bool live = k < n4;
    uint32_t l = 0u, g = 0u;
    if (live) {
      l = reinterpret_cast<const uint32_t*>(lv + rs)[k];
      g = reinterpret_cast<const uint32_t*>(sg + rs)[k];
    }
    const float4 r = decode4<KIND>(l, g, norm, mn, d, s, live);
    if (live) store4_nt(reinterpret_cast<float4*>(oc + rs) + k, r);
  }
  const int i = edge_elem(head, rs + (n4 << 2), c.len);
  if (i >= 0) oc[i] = decode_exact<KIND>(lv[i], sg[i], norm, mn, s);
}

// Server-side mean of K clients' payloads: simple_aggregate (Src/ADFL/model.py:221-234) over the K decodes
// (quant.py:243-252 / :385-398 / :537-545), the synchronous server's aggregate of K updates:
//   out[i] = fp32(torch-order sum over r of d_r[i]) / K   (the division correctly rounded)
// in torch's CPU summation order for sum(stack(...), dim=0) (torch_sum_order.h: per tensor, the order depends
// on the element's index in its tensor; SEQ columns from +0, cascaded every 16 rows), with d_r the decode of
// row r's level / exponent and sign bytes under row r's norm (+0 where that norm is 0, as the decoder returns
// zeros). Row r's planes are levels / signs + r * row_stride (one bucket payload each, one chunk table), its
// norms norms + r * norm_stride (RQSGD's minima likewise). The sum starts from +0 as torch's does, so a column
// of -0 decodes (level 0, sign -1) sums to +0. One block per chunk; each thread's dword groups of SEQ columns
// (after the < 4-element head), all of a row's loads issued before its decodes; the < 4-element head and the
// elements past the tensor's last SEQ column element-wise in their own order. DEEP: K >= 256.
template <int KIND>
__device__ __forceinline__ float mean_term(uint32_t l, uint32_t g, float norm, float mn, float s) {
  return norm == 0.0f ? 0.0f : decode_exact<KIND>(l, g, norm, mn, s);
}

template <int KIND, bool DEEP>
__global__ __launch_bounds__(kBlock) void k_stoch_dequantize_mean(const uint8_t* __restrict__ levels,
                                                                  const uint8_t* __restrict__ signs,
                                                                  int64_t row_stride, int k,
                                                                  const adfl_slq_chunk* __restrict__ chunks,
                                                                  const float* __restrict__ norms,
                                                                  const float* __restrict__ mins, int64_t norm_stride,
                                                                  float s, float* __restrict__ out) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const int64_t t_start = chunks[c.first_chunk].start;
  const int64_t t_n = (int64_t)(c.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[c.first_chunk + c.nchunks - 1].len;
  const int head = chunk_head4(c.start, c.len);
  int64_t lim = t_start + adfl_sum::seq_end(t_n) - c.start;  // chunk-relative end of the SEQ columns
  lim = lim < c.len ? lim : c.len;
  const int n4 = lim > head ? (int)((lim - head) >> 2) : 0;  // dword groups wholly in SEQ columns
  const double dk = (double)k;
  adfl_sum::SeqTile<kPer, DEEP> acc;
  acc.init();
  for (int r = 0; r < k; ++r) {
    const float norm = norms[r * norm_stride + c.tensor];
    const float mn = KIND == 1 ? mins[r * norm_stride + c.tensor] : 0.0f;
    const uint8_t* lv = levels + r * row_stride + c.start;
    const uint8_t* sg = signs + r * row_stride + c.start;
    const uint32_t* l4 = reinterpret_cast<const uint32_t*>(lv + head);
    const uint32_t* g4 = reinterpret_cast<const uint32_t*>(sg + head);
    uint32_t L[kPer], G[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int q = threadIdx.x + j * kBlock;
      L[j] = q < n4 ? l4[q] : 0u;
      G[j] = q < n4 ? g4[q] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if ((int)threadIdx.x + j * kBlock < n4)
        acc.add(j, make_float4(mean_term<KIND>(L[j] & 0xffu, G[j] & 0xffu, norm, mn, s),
                               mean_term<KIND>((L[j] >> 8) & 0xffu, (G[j] >> 8) & 0xffu, norm, mn, s),
                               mean_term<KIND>((L[j] >> 16) & 0xffu, (G[j] >> 16) & 0xffu, norm, mn, s),
                               mean_term<KIND>(L[j] >> 24, G[j] >> 24, norm, mn, s)));
    }
    acc.step();
  }
  float* oc = out + c.start;
  float4* o4 = reinterpret_cast<float4*>(oc + head);
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int q = threadIdx.x + j * kBlock;
    if (q < n4) {
      const float4 a = acc.result(j);
      store4_nt(o4 + q, make_float4((float)((double)a.x / dk), (float)((double)a.y / dk), (float)((double)a.z / dk),
                                    (float)((double)a.w / dk)));
    }
  }
  // head elements and those past the SEQ groups: each in its own order
  const int rest = c.len - (head + (n4 << 2));
  for (int t = threadIdx.x; t < head + rest; t += kBlock) {
    const int i = t < head ? t : head + (n4 << 2) + (t - head);
    auto get = [&](int r) -> float {
      const float norm = norms[r * norm_stride + c.tensor];
      const float mn = KIND == 1 ? mins[r * norm_stride + c.tensor] : 0.0f;
      return mean_term<KIND>(levels[r * row_stride + c.start + i], signs[r * row_stride + c.start + i], norm, mn, s);
    };
    const int64_t j = c.start + i - t_start;
    oc[i] = (float)((double)adfl_sum::sum_elem(get, k, adfl_sum::mode_of(j, t_n, k)) / dk);
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


template <int MODE>
inline int launch_finalize(const adfl_slq_chunk* d_chunks, int64_t nchunks, const void* d_ws, float* d_norms,
                           float* d_mins, hipStream_t st) {
  const int64_t blocks = (nchunks + kBigBlock - 1) / kBigBlock;  // per role
  hipLaunchKernelGGL(k_norm_finalize<MODE>, dim3((unsigned)(2 * blocks)), dim3(kBigBlock), 0, st, d_chunks, nchunks,
                     blocks, d_ws, d_norms, d_mins);
  return launch_status();
}

// KIND 0 QSGD, 1 RQSGD, 2 CNAT (d_a = levels, or CNAT's exponent bytes)
template <int KIND>
inline int launch_resident(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, const int32_t* d_work,
                           int64_t nwork, int bits, const float* d_uniforms, uint64_t seed, uint64_t counter,
                           uint8_t* d_a, int8_t* d_signs, float* d_norms, float* d_mins, void* stream) {
  if (!d_x || !d_work || !d_a || !d_signs || !d_norms || (KIND == 1 && !d_mins) || bad_table(d_chunks, nchunks) ||
      nwork < 1 || nwork > nchunks)
    return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_a) || !aligned16(d_signs) || (d_uniforms && !aligned16(d_uniforms)))
    return ADFL_E_ALIGN;
  const Uniforms U{d_uniforms, seed, counter};
  const dim3 grid((unsigned)nwork), block(kResBlock);
  hipStream_t st = (hipStream_t)stream;
  if (KIND == 2) {
    const int min_e = -(1 << (bits - 1)), max_e = (1 << (bits - 1)) - 1;  // quant.py:519-520
    hipLaunchKernelGGL(k_cnat_encode_resident<kPbResident>, grid, block, 0, st, d_x, d_chunks, d_work, min_e, max_e, U,
                       reinterpret_cast<int8_t*>(d_a), d_signs, d_norms);
  } else {
    constexpr int mode = KIND == 1 ? ADFL_NORM_LINF : ADFL_NORM_L2;
    hipLaunchKernelGGL((k_qsgd_encode_resident<mode, kPbResident, kEarlySigns>), grid, block, 0, st, d_x, d_chunks,
                       d_work, levels_f(bits), U, d_a, d_signs, d_norms, d_mins);
  }
  return launch_status();
}

}  // namespace

namespace adfl_tn {
// The in-order walker for fp32 tensors of at most kWalkMax elements, for adfl_torch_norms (torch_norm.hip).
int launch_walk(const float* x, const adfl_slq_chunk* chunks, int64_t nchunks, float* n32, double* n64,
                hipStream_t st) {
  hipLaunchKernelGGL(k_norm_walk, dim3((unsigned)nchunks), dim3(kWalkThreads), 0, st, x, chunks, kWalkMax, n32, n64);
  return (int)hipGetLastError();
}
}  // namespace adfl_tn

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int64_t adfl_stoch_workspace_bytes(int64_t nchunks) { return nchunks < 1 ? kPartialBytes : nchunks * kPartialBytes; }

int adfl_stoch_norms_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int mode,
                             void* d_workspace, int64_t workspace_bytes, float* d_norms, float* d_mins,
                             void* stream) {
  if (!d_x || !d_norms || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (mode != ADFL_NORM_L2 && mode != ADFL_NORM_LINF && mode != ADFL_NORM_L2_TORCH) return ADFL_E_ARG;
  if (!aligned16(d_x)) return ADFL_E_ALIGN;
  hipStream_t st = (hipStream_t)stream;
  if (mode == ADFL_NORM_L2_TORCH) {  // no workspace: one block per tensor
    hipLaunchKernelGGL(adfl_tn::k_norm_walk, dim3((unsigned)nchunks), dim3(adfl_tn::kWalkThreads), 0, st, d_x, d_chunks,
                       INT64_MAX, d_norms, nullptr);
    return launch_status();
  }
  if (int s = check_ws(d_workspace, workspace_bytes, nchunks)) return s;
  if (mode == ADFL_NORM_L2) {
    hipLaunchKernelGGL(k_norm_partials<ADFL_NORM_L2>, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks,
                       nchunks - kKeepChunks, d_workspace);
    if (int s = launch_status()) return s;
    return launch_finalize<ADFL_NORM_L2>(d_chunks, nchunks, d_workspace, d_norms, d_mins, st);
  }
  hipLaunchKernelGGL(k_norm_partials<ADFL_NORM_LINF>, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks,
                     nchunks - kKeepChunks, d_workspace);
  if (int s = launch_status()) return s;
  return launch_finalize<ADFL_NORM_LINF>(d_chunks, nchunks, d_workspace, d_norms, d_mins, st);
}


int adfl_qsgd_quantize_batched(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int bits,
                               const float* d_norms, const float* d_uniforms, uint64_t seed, uint64_t counter,
                               uint8_t* d_levels, int8_t* d_signs, void* stream) {
  if (!d_x || !d_norms || !d_levels || !d_signs || bad_table(d_chunks, nchunks)) return ADFL_E_ARG;
  if (int s = check_bits(bits)) return s;
  if (!aligned16(d_x) || !aligned16(d_levels) || !aligned16(d_signs) || (d_uniforms && !aligned16(d_uniforms)))
    return ADFL_E_ALIGN;
  const Uniforms U{d_uniforms, seed, counter};
  hipLaunchKernelGGL(k_qsgd_quantize<kPbQuantize>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, d_x, d_chunks,
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
  const int min_e = -(1 << (bits - 1)), max_e = (1 << (bits - 1)) - 1;  // quant.py:519-520
  hipLaunchKernelGGL(k_cnat_quantize<kPbQuantize>, dim3((unsigned)nchunks), dim3(kBlock), 0, st, d_x, d_chunks, min_e, max_e, U,
                     d_exps, d_signs, (double*)d_workspace);
  if (int s = launch_status()) return s;
  if (int s = launch_finalize<ADFL_NORM_L2>(d_chunks, nchunks, d_workspace, d_norms, nullptr, st)) return s;
  hipLaunchKernelGGL(k_cnat_zero_fixup, dim3((unsigned)((nchunks + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     d_chunks, nchunks, (const float*)d_norms, d_exps, d_signs);
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

int adfl_qsgd_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                  const int32_t* d_work, int64_t nwork, int bits, const float* d_uniforms,
                                  uint64_t seed, uint64_t counter, void* d_workspace, int64_t workspace_bytes,
                                  uint8_t* d_levels, int8_t* d_signs, float* d_norms, void* stream) {
  if (nwork == 0)
    return adfl_qsgd_encode_batched(d_x, d_chunks, nchunks, bits, d_uniforms, seed, counter, d_workspace,
                                    workspace_bytes, d_levels, d_signs, d_norms, stream);
  return launch_resident<0>(d_x, d_chunks, nchunks, d_work, nwork, bits, d_uniforms, seed, counter, d_levels, d_signs,
                            d_norms, nullptr, stream);
}

int adfl_rqsgd_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                   const int32_t* d_work, int64_t nwork, int bits, const float* d_uniforms,
                                   uint64_t seed, uint64_t counter, void* d_workspace, int64_t workspace_bytes,
                                   uint8_t* d_levels, int8_t* d_signs, float* d_norms, float* d_mins, void* stream) {
  if (nwork == 0)
    return adfl_rqsgd_encode_batched(d_x, d_chunks, nchunks, bits, d_uniforms, seed, counter, d_workspace,
                                     workspace_bytes, d_levels, d_signs, d_norms, d_mins, stream);
  return launch_resident<1>(d_x, d_chunks, nchunks, d_work, nwork, bits, d_uniforms, seed, counter, d_levels, d_signs,
                            d_norms, d_mins, stream);
}

int adfl_cnat_encode_batched_work(const float* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                                  const int32_t* d_work, int64_t nwork, int bits, const float* d_uniforms,
                                  uint64_t seed, uint64_t counter, void* d_workspace, int64_t workspace_bytes,
                                  int8_t* d_exps, int8_t* d_signs, float* d_norms, void* stream) {
  if (nwork == 0)
    return adfl_cnat_encode_batched(d_x, d_chunks, nchunks, bits, d_uniforms, seed, counter, d_workspace,
                                    workspace_bytes, d_exps, d_signs, d_norms, stream);
  return launch_resident<2>(d_x, d_chunks, nchunks, d_work, nwork, bits, d_uniforms, seed, counter,
                            reinterpret_cast<uint8_t*>(d_exps), d_signs, d_norms, nullptr, stream);
}

int adfl_stoch_dequantize_mean_batched(int32_t codec, const uint8_t* d_levels, const int8_t* d_signs,
                                       int64_t row_stride_bytes, int32_t k, const adfl_slq_chunk* d_chunks,
                                       int64_t nchunks, int bits, const float* d_norms, const float* d_mins,
                                       int64_t norm_stride, float* d_out, void* stream) {
  if (codec != ADFL_CODEC_QSGD && codec != ADFL_CODEC_RQSGD && codec != ADFL_CODEC_CNAT) return ADFL_E_ARG;
  if (!d_levels || !d_signs || !d_norms || !d_out || (codec == ADFL_CODEC_RQSGD && !d_mins) ||
      bad_table(d_chunks, nchunks) || k < 1 || k > adfl_sum::kMaxRows || row_stride_bytes < 0 || norm_stride < 0 ||
      (k > 1 && (row_stride_bytes == 0 || norm_stride == 0)))
    return ADFL_E_ARG;
  if (codec != ADFL_CODEC_CNAT)
    if (int s = check_bits(bits)) return s;
  if (!aligned16(d_levels) || !aligned16(d_signs) || !aligned16(d_out) || (row_stride_bytes & 15)) return ADFL_E_ALIGN;
  const float s = codec == ADFL_CODEC_CNAT ? 1.0f : levels_f(bits);
  const auto* sg = reinterpret_cast<const uint8_t*>(d_signs);
  const dim3 grid((unsigned)nchunks), block(kBlock);
  hipStream_t st = (hipStream_t)stream;
  const bool deep = k >= 256;
  auto kern = codec == ADFL_CODEC_QSGD
                  ? (deep ? k_stoch_dequantize_mean<0, true> : k_stoch_dequantize_mean<0, false>)
                  : codec == ADFL_CODEC_RQSGD ? (deep ? k_stoch_dequantize_mean<1, true> : k_stoch_dequantize_mean<1, false>)
                                              : (deep ? k_stoch_dequantize_mean<2, true> : k_stoch_dequantize_mean<2, false>);
  hipLaunchKernelGGL(kern, grid, block, 0, st, d_levels, sg, row_stride_bytes, k, d_chunks, d_norms, d_mins, norm_stride,
                     s, d_out);
  return launch_status();
}

int adfl_philox_rounds(void) { return adfl::kPhiloxRounds; }

int adfl_philox_uniforms(float* d_out, int64_t n, int64_t start, uint64_t seed, uint64_t counter, void* stream) {
  if (!d_out || n < 1 || start < 0) return ADFL_E_ARG;
  const Uniforms U{nullptr, seed, counter};
  const int64_t g = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_philox_uniforms, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(kBlock), 0, (hipStream_t)stream,
                     d_out, n, start, U);
  return launch_status();
}

}  // extern "C"
