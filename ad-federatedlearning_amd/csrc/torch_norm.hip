// torch_norm.hip — torch 2.10's CPU L2 norm (torch.linalg.vector_norm(x, ord=2), the reference's QSGD / CNAT
// scale: Src/ADFL/Channel/quant.py:226,512) of fp32 / bf16 / fp16 / fp64 tensors, bit for bit, in phases with
// no cross-block waits.
//
// The orders (oracle/slq_oracle.c restates each; tests/test_torch_norm_dtypes.py pins them to torch itself):
//   fp32  8 fp32 chains, element e into chain e % 8 for e < n - n % 8, acc = fmaf(x, x, acc) in order; lane
//         sum left to right; the n % 8 tail as torch's compiled scalar loop runs it (a group of 4 rounded
//         squares added in order when there are 4 or more, the rest with fmaf); fp32 sqrt.
//   bf16  the same 8 fp32 chains over e < n - n % 16 (16-element vectors), tail with fmaf; sqrt, to bf16.
//   fp16  at::parallel_for's split: nt = min(threads, ceil(n / 32768)) chunks (1 below 32768 elements or
//         with one thread) of ceil(n / nt) elements, each one fp32 chain from 0; the chain sums added in
//         order; sqrt, to fp16. `threads` is the caller's torch.get_num_threads().
//   fp64  4 fp64 chains (e % 4, e < n - n % 4) with fma; lane sum; the tail with fma; fp64 sqrt.
//   Every dtype: a one-element tensor's norm is |x| (no square, so no underflow).
// Squares of fp16 / bf16 / fp32 values are exact in fp64 (and fp16 / bf16 ones in fp32), so every chain step
// is acc <- RN(acc + p) with p exact: fp32 accumulators for fp32 / bf16 / fp16, fp64 ones for fp64.
//
// The integer model. While acc stays in one binade it is A * u (u the binade's ulp, A an integer below
// 2^24 — 2^53 for fp64 — and above 2^23 / 2^52 unless the binade is the subnormal one) and a step that does
// not leave the binade is A <- A + R(p / u), R = round half to even. A step whose p / u is not a tie adds
// a constant k. A tie, p / u = f + 1/2, gives A + f rounded up to even: it depends on A's parity only.
// So a run of steps is a pair of constants (Ke, Ko) — what it adds to an even / an odd A — and runs
// compose associatively: (a then b).e = a.e + (a.e odd ? b.o : b.e), .o = a.o + (a.o even ? b.o : b.e).
// A run is exact from A if A + its increment stays below 2^24 (increments are >= 0, so every partial sum
// does too). Only a step that leaves the binade (a "crossing", about log2 of the norm's growth per chain),
// a non-finite value, or a step of 2^24 ulps or more is not covered: the reference arithmetic (fma) runs it.
//
// Phases (long tensors: more than kShortMax elements), one launch each, every block independent:
//   A  k_tn_sums: per 8192-element chunk and chain (fp16: piece), the fp64 sum S of x^2 (one read of x;
//      fp32 / bf16 / fp16, k_tn_sums_sampled: of a 1/16 sample, weighted 16 — their phase C totals are exact, so S only
//      predicts binades and flags nothing);
//   B  k_tn_winsums + k_tn_grids: per window of 512 tiles the sum of S, then per tile the exclusive prefix P
//      (earlier windows + a wave scan) predicts the binade of the accumulator at the tile's start:
//      g = binade(P (1 + 2^-8)) — a prediction only (a miss leaves the tile uncovered, resolved in D);
//   C  k_tn_maps: per tile, its integer totals on g and g - 1, order-free (k = rint(hi), rint(2 hi)); a
//      chunk whose squares may hide a tie is listed for k_tn_maps_exact, which stages it chain-major through
//      LDS and composes each lane's 16 steps as (Ke, Ko) maps in order (second read of x); fp32: k_tn_maps_f32
//      (exact fp32 increments); bf16 / fp16, whose ties are real: every chunk straight to k_tn_maps_exact;
//   C2 k_tn_windows: per window, the composition of its tiles' maps for the two binades it can start in;
//   D  k_tn_chains: one wave per chain: windows 64 at a time on the exact accumulator's binade, the first one
//      not covered tile by tile, the first tile not covered in segments of 1024 steps (lane sums or maps on
//      G and G + 1, scanned; the lane that crosses runs its steps with fma); then k_tn_finish: the lane sum
//      (fp16: piece sums in order), the tail, sqrt and the rounding to the dtype. fp32 runs its segments with
//      k_tn_short's short_segment and its window / tile scans in fp32 by DPP (integer totals below 2^24).
// Short tensors, one block per tensor in one launch: fp32 up to kShortMaxF32 elements k_tn_short (ADFL_TN_WALKER
// builds: the in-order walker, torch_norm_walk.h), bf16 up to the same k_tn_short_bf16, fp16 up to kShortMax
// k_tn_short_f16; short fp64 tensors go straight to D with every tile resolved in detail. DESIGN.md §10.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <type_traits>

#include "adfl_slq.h"
#include "adfl_stoch.h"

namespace adfl_tn {
int launch_walk(const float* x, const adfl_slq_chunk* chunks, int64_t nchunks, float* n32, double* n64, hipStream_t st);
}

namespace adfl_tnx {

#ifdef ADFL_TN_STATS  // tools/ref_norm_prof.py --stats builds: phase D counters per wave, printed per launch
__device__ unsigned long long g_tn_stats[8][12];  // window descents, tiles in detail, segment rounds, cycles, cycles in
// detail, cycles waiting for segment loads, cycles in window descents, window scans, exact-path segment rounds,
// cycles in segments, cycles waiting for a window's records, cycles in window scans up to a tile in detail
#define TN_STAT(i, v) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_tn_stats[blockIdx.y & 7][i], (unsigned long long)(v)); } while (0)
// k_tn_short's counters, summed over its waves: segments, rounds, exact-map rounds, lanes run with fma, G + 1
// continuations that finished the segment, cycles in short_segment, cycles per wave, (unused), waves, cycles in
// stage() (its load waits included), cycles in barriers
__device__ unsigned long long g_sh_stats[11];
// one block's timeline (tools: stats builds): per wave, up to 48 (event, clock) pairs — 1 stage start, 2 stage
// end, 3 run start (LDS read issued), 4 segment start (values in registers), 5 run end, 6 barrier end
__device__ long long g_sh_tl[8][48][2];
__device__ int g_sh_tln[8];
#define SH_TL(e) do { if (shn < 48) { if ((threadIdx.x & 63) == 0) { s_tl[threadIdx.x >> 6][shn][0] = (e); \
  s_tl[threadIdx.x >> 6][shn][1] = clock64(); } ++shn; } } while (0)  // in LDS: no vmcnt waits added
#define SH_STAT(i, v) do { shs[i] += (unsigned long long)(v); } while (0)  // per wave, added once at the end
#define SH_ARG , unsigned long long (&shs)[11]
#define SH_PASS , shs
#else
#define TN_STAT(i, v) do { } while (0)
#define SH_STAT(i, v) do { } while (0)
#define SH_ARG
#define SH_PASS
#define SH_TL(e) do { } while (0)
#endif

constexpr int kChunk = ADFL_SLQ_CHUNK_ELEMS;      // 8192: a tile is a chunk's steps of one chain
constexpr int kSlots = 8;                         // records per chunk: one per chain (strided) or piece (fp16)
constexpr int kLane = 16;                         // steps per lane
constexpr int kSeg = 64 * kLane;                  // 1024 steps: one wave's segment
constexpr int64_t kShortMax = 1 << 16;            // tensors up to this size skip phases A-C (fp16 / bf16 / fp64)
#ifndef ADFL_TN_SHORT_MAX_F32
#define ADFL_TN_SHORT_MAX_F32 (1 << 19)
#endif
constexpr int64_t kShortMaxF32 = ADFL_TN_SHORT_MAX_F32;  // fp32: k_tn_short (one block per tensor) up to this size
template <int DT> constexpr int64_t short_max() {  // fp32 / bf16: k_tn_short(_bf16); fp16: k_tn_short_f16; fp64: D
  return DT == ADFL_DTYPE_F32 || DT == ADFL_DTYPE_BF16 ? kShortMaxF32 : kShortMax;
}
constexpr int64_t kGrain = 32768;                 // at::internal::GRAIN_SIZE
constexpr int kMaxChains = 512;                   // fp16: chains (torch threads) per tensor the combine holds
constexpr double kMagic = 6755399441055744.0;     // 1.5 * 2^52: (v + kMagic) - kMagic = rint(v), 0 <= v < 2^51
constexpr int kTPL = 8;                           // phase D: tiles per lane
constexpr int kWinTiles = 64 * kTPL;              // phase D: tiles per window

__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ double pow2(int k) { return __longlong_as_double((long long)(k + 1023) << 52); }
__device__ __forceinline__ bool odd(double v) { return floor(v * 0.5) * 2.0 != v; }  // v an integer

// ---- accumulator types
template <bool W> struct Acc;
template <> struct Acc<false> {
  using T = float;
  static constexpr int kM = 23, kGmin = -126, kGmax = 127;
  static constexpr double kTop = 16777216.0;  // 2^24
};
template <> struct Acc<true> {
  using T = double;
  static constexpr int kM = 52, kGmin = -1022, kGmax = 1023;
  static constexpr double kTop = 9007199254740992.0;  // 2^53
};

__device__ __forceinline__ int grid_of(float a) {
  const uint32_t ef = __float_as_uint(a) >> 23;
  return ef <= 1u ? -126 : (int)ef - 127;
}
__device__ __forceinline__ int grid_of(double a) {
  const uint64_t ef = (uint64_t)__double_as_longlong(a) >> 52;
  return ef <= 1u ? -1022 : (int)ef - 1023;
}
__device__ __forceinline__ double a_of(float a) {  // the integer A of a finite accumulator >= 0 on its grid
  const uint32_t b = __float_as_uint(a), m = b & 0x7fffffu;
  return (double)((b >> 23) ? (m | 0x800000u) : m);
}
__device__ __forceinline__ double a_of(double a) {
  const uint64_t b = (uint64_t)__double_as_longlong(a), m = b & ((1ull << 52) - 1);
  return (double)(long long)((b >> 52) ? (m | (1ull << 52)) : m);
}
template <bool W> __device__ __forceinline__ typename Acc<W>::T rebuild(double A, int g);
template <> __device__ __forceinline__ float rebuild<false>(double A, int g) { return (float)(A * pow2(g - 23)); }
template <> __device__ __forceinline__ double rebuild<true>(double A, int g) { return (A * 0x1p-52) * pow2(g); }

// the binade an accumulator near the exact value v >= 0 is predicted in
template <bool W> __device__ __forceinline__ int grid_pred(double v) {
  v *= 1.0 + 0x1p-8;
  if (!(v < 0x1p127) && !W) return 127;
  if (!W && v < 0x1p-125) return -126;
  if (W && !(v < 0x1p1023)) return 1023;
  if (W && v < 0x1p-1021) return -1022;
  return (int)(((uint64_t)__double_as_longlong(v) >> 52) & 0x7ff) - 1023;
}

// ---- maps: what a run of steps adds to an even / an odd A
struct Map {
  double e, o;
};
__device__ __forceinline__ Map compose(Map a, Map b) {  // a, then b
  return Map{a.e + (odd(a.e) ? b.o : b.e), a.o + (odd(a.o) ? b.e : b.o)};
}
__device__ __forceinline__ double apply(Map m, double A) { return A + (odd(A) ? m.o : m.e); }
__device__ __forceinline__ Map shfl_up(Map m, int o) { return Map{__shfl_up(m.e, o, 64), __shfl_up(m.o, o, 64)}; }
__device__ __forceinline__ Map shfl_xor(Map m, int o) { return Map{__shfl_xor(m.e, o, 64), __shfl_xor(m.o, o, 64)}; }

// every lane: the composition of all 64 lanes' maps in lane order
__device__ __forceinline__ Map wave_compose(Map m, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const Map p = shfl_xor(m, o);
    m = (lane & o) ? compose(p, m) : compose(m, p);
  }
  return m;
}
// exclusive prefix (composition of the lanes before this one; identity on lane 0)
__device__ __forceinline__ Map wave_excl(Map m, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const Map p = shfl_up(m, o);
    if (lane >= o) m = compose(p, m);
  }
  const Map x = shfl_up(m, 1);
  return lane == 0 ? Map{0.0, 0.0} : x;
}
__device__ __forceinline__ double wave_excl_sum(double v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double p = __shfl_up(v, o, 64);
    if (lane >= o) v += p;
  }
  const double x = __shfl_up(v, 1, 64);
  return lane == 0 ? 0.0 : x;
}

template <int CTRL, int RM>
__device__ __forceinline__ float dpp0(float v) {  // the DPP-moved value, +0 where the lane has no source
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, RM, 0xf, false));
}
__device__ __forceinline__ bool odd_f(float v) { return __builtin_amdgcn_fractf(v * 0.5f) != 0.0f; }  // v an integer
template <int CTRL, int RM>
__device__ __forceinline__ void dpp_compose(float& e, float& o) {  // (e, o) <- (the moved lane's map) then (e, o)
  const float pe = dpp0<CTRL, RM>(e), po = dpp0<CTRL, RM>(o);   // identity (0, 0) where no lane moves in
  const float ne = pe + (odd_f(pe) ? o : e), no = po + (odd_f(po) ? e : o);
  e = ne;
  o = no;
}
// every lane: the composition of all 64 lanes' maps in lane order, as fp32 pairs by DPP — for maps of integers
// (exact-square inputs): exact below 2^24, at least 2^24 above (every term >= 0), which is all a consumer of a
// fp32-accumulator map tests (Acc<false>::kTop); +inf stays +inf
__device__ __forceinline__ float lane63_f(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63)); }
__device__ __forceinline__ Map wave_compose_f(Map m) {
  float e = (float)m.e, o = (float)m.o;
  dpp_compose<0x111, 0xf>(e, o);  // row_shr:1
  dpp_compose<0x112, 0xf>(e, o);  // row_shr:2
  dpp_compose<0x114, 0xf>(e, o);  // row_shr:4
  dpp_compose<0x118, 0xf>(e, o);  // row_shr:8
  dpp_compose<0x142, 0xa>(e, o);  // row_bcast:15
  dpp_compose<0x143, 0xc>(e, o);  // row_bcast:31
  return Map{(double)lane63_f(e), (double)lane63_f(o)};
}

// ---- one step's increment on grid with ulp 2^-s (s = kM - g): k and whether it is a tie (then k = floor)
__device__ __forceinline__ void inc_exact(float x, double sc, double& k, bool& tie) {
  const double d = (double)x;
  const double v = d * (d * sc);              // x^2 / u, exact (48 bits)
  const double kd = (v + kMagic) - kMagic;    // rint; v >= 2^51 makes kd huge (not covered) — fine
  const double fr = v - kd;
  tie = __builtin_fabs(fr) == 0.5;
  k = tie && fr < 0.0 ? kd - 1.0 : kd;
}
__device__ __forceinline__ void inc_exact(double x, double sc_unused, double& k, bool& tie, int s) {
  // x^2 * 2^s as hi + lo without overflow or underflow of the scale: x' = x 2^(s >> 1), x'' = x' 2^(s & 1)
  const double xa = x * pow2(s >> 1);
  const double xb = (s & 1) ? xa * 2.0 : xa;
  const double hi = xa * xb, lo = __fma_rn(xa, xb, -hi);
  double kd = (hi + kMagic) - kMagic;
  const double fr = hi - kd;
  tie = false;
  if (__builtin_fabs(fr) == 0.5) {
    if (lo == 0.0) tie = true;
    else if ((fr > 0.0) == (lo > 0.0)) kd += fr > 0.0 ? 1.0 : -1.0;
  }
  k = tie && fr < 0.0 ? kd - 1.0 : kd;
  (void)sc_unused;
}

// A lane's map of its steps v[0..n) in order on grid g (exact tie handling): the slow path.
template <bool W, typename E>
__device__ __forceinline__ Map lane_map_exact(const E (&v)[kLane], int g) {
  const int s = Acc<W>::kM - g;
  const double sc = W ? 0.0 : pow2(s);
  double se = 0.0, so = 1.0;
#pragma unroll
  for (int i = 0; i < kLane; ++i) {
    double k;
    bool tie;
    if constexpr (W) inc_exact((double)v[i], sc, k, tie, s);
    else inc_exact((float)v[i], sc, k, tie);
    se += k;
    so += k;
    if (tie) {
      se += odd(se) ? 1.0 : 0.0;
      so += odd(so) ? 1.0 : 0.0;
    }
  }
  return Map{se, so - 1.0};
}

// Lane maps on grids g and g + d (d = +1 or -1) in one pass. SQ (bf16 / fp16 inputs): x^2 has at most 22
// significant bits, so hi = x^2 / u is exact in fp32 and its fraction decides ties: fp32 / int32 arithmetic,
// no fp64 (a square that underflows is far below 1/2: no tie, increment 0). Otherwise lane_map_exact twice.
__device__ __forceinline__ float pow2f(int k) { return __int_as_float((k + 127) << 23); }  // -126 <= k <= 128
// 2^k for -149 <= k <= 127, subnormal powers included (half-ulps of low binades: 2^(G-24) down to G = -125)
__device__ __forceinline__ float pow2fs(int k) { return k >= -126 ? pow2f(k) : __int_as_float(1 << (k + 149)); }
__device__ __forceinline__ void sq_step(float h, int& e, int& o) {
  const float k = (h + 12582912.0f) - 12582912.0f;  // rint, |h| < 2^22
  const float fr = h - k;
  const bool tie = __builtin_fabsf(fr) == 0.5f;
  const int ki = (int)k - ((tie && fr < 0.0f) ? 1 : 0);
  e += ki;
  o += ki;
  if (tie) {
    e += e & 1;
    o += o & 1;
  }
}
template <bool W, bool SQ, typename E>
__device__ __forceinline__ void lane_maps_pair(const E (&v)[kLane], int g, int d, Map& m0, Map& m1) {
  if constexpr (!W && SQ) {
    const int s = 23 - g;
    const float sa = pow2f(s >> 1), sb = (s & 1) ? 2.0f : 1.0f, sd = d > 0 ? 0.5f : 2.0f;
    int e0 = 0, o0 = 1, e1 = 0, o1 = 1;
    bool big0 = false, big1 = false;
#pragma unroll
    for (int i = 0; i < kLane; ++i) {
      const float xs = (float)v[i] * sa;
      const float h0 = xs * xs * sb, h1 = h0 * sd;
      big0 |= !(h0 < 0x1p21f);  // NaN / inf too: not covered
      big1 |= !(h1 < 0x1p21f);
      sq_step(big0 ? 0.0f : h0, e0, o0);
      sq_step(big1 ? 0.0f : h1, e1, o1);
    }
    const double inf = __builtin_inf();
    m0 = big0 ? Map{inf, inf} : Map{(double)e0, (double)(o0 - 1)};
    m1 = (big1 || g + d < Acc<W>::kGmin || g + d > Acc<W>::kGmax) ? Map{inf, inf} : Map{(double)e1, (double)(o1 - 1)};
  } else {
    m0 = lane_map_exact<W>(v, g);
    m1 = (g + d < Acc<W>::kGmin || g + d > Acc<W>::kGmax) ? Map{__builtin_inf(), __builtin_inf()} : lane_map_exact<W>(v, g + d);
  }
}

// ---- dtype traits
template <int DT> struct Dt;
template <> struct Dt<ADFL_DTYPE_F32> {
  using S = float;
  using E = float;
  static constexpr int NC = 8, VB = 8;
  static constexpr bool kContig = false, kWide = false, kSq = false;
  __device__ static E ld(const void* x, int64_t i) { return ((const float*)x)[i]; }
};
template <> struct Dt<ADFL_DTYPE_BF16> {
  using S = uint16_t;
  using E = float;
  static constexpr int NC = 8, VB = 16;
  static constexpr bool kContig = false, kWide = false, kSq = true;
  __device__ static E ld(const void* x, int64_t i) { return __uint_as_float((uint32_t)((const uint16_t*)x)[i] << 16); }
};
template <> struct Dt<ADFL_DTYPE_F16> {
  using S = uint16_t;
  using E = float;
  static constexpr int NC = 1, VB = 1;
  static constexpr bool kContig = true, kWide = false, kSq = true;
  __device__ static E ld(const void* x, int64_t i) { return __half2float(__ushort_as_half(((const uint16_t*)x)[i])); }
};
template <> struct Dt<ADFL_DTYPE_F64> {
  using S = double;
  using E = double;
  static constexpr int NC = 4, VB = 4;
  static constexpr bool kContig = false, kWide = true, kSq = false;
  __device__ static E ld(const void* x, int64_t i) { return ((const double*)x)[i]; }
};

// A tensor and its chains, from the chunk table.
struct Tensor {
  int64_t base;  // first element in the flat buffer
  int64_t n;
  int64_t nall;  // chunks in the table (records are chain-major: slot = k * nall + chunk)
  int first;     // first chunk
  int nch;       // chunks
  int tensor;
};
__device__ __forceinline__ Tensor tensor_of(const adfl_slq_chunk* chunks, int ci, int64_t nall) {
  const adfl_slq_chunk ch = chunks[ci];
  Tensor t;
  t.nall = nall;
  t.first = ch.first_chunk;
  t.nch = ch.nchunks;
  t.tensor = ch.tensor;
  t.base = ch.start - (int64_t)(ci - ch.first_chunk) * kChunk;
  t.n = (int64_t)(ch.nchunks - 1) * kChunk + chunks[ch.first_chunk + ch.nchunks - 1].len;
  return t;
}

// fp16: at::parallel_for's split of n elements over `threads`
struct Split {
  int64_t nt, cs;
};
__device__ __forceinline__ Split split_of(int64_t n, int threads) {
  int64_t nt = 1;
  if (n >= kGrain && threads > 1) {
    nt = (n + kGrain - 1) / kGrain;
    if (nt > threads) nt = threads;
  }
  return Split{nt, (n + nt - 1) / nt};
}

// Record slot of chunk ci's chain (strided) or piece (fp16) k: chain-major, so a chain's tiles are contiguous.
__device__ __forceinline__ int64_t slot_of(int64_t ci, int k, int64_t nall) { return (int64_t)k * nall + ci; }

// Chain c's tile t (strided: chunk t; fp16: the t-th chunk the chain touches): its record slot and steps.
struct Tile {
  int64_t slot, s0, s1;  // steps [s0, s1) of the chain
};
template <int DT>
__device__ __forceinline__ int64_t chain_len(const Tensor& T, int c, Split sp) {
  if constexpr (Dt<DT>::kContig) {
    const int64_t a = (int64_t)c * sp.cs, b = a + sp.cs < T.n ? a + sp.cs : T.n;
    return b > a ? b - a : 0;
  } else {
    return T.n >= Dt<DT>::VB ? (T.n - T.n % Dt<DT>::VB) / Dt<DT>::NC : 0;
  }
}
template <int DT>
__device__ __forceinline__ int64_t chain_tiles(const Tensor& T, int c, Split sp) {
  const int64_t L = chain_len<DT>(T, c, sp);
  if (L == 0) return 0;
  if constexpr (Dt<DT>::kContig) {
    const int64_t a = (int64_t)c * sp.cs;
    return (a + L - 1) / kChunk - a / kChunk + 1;
  } else {
    constexpr int spc = kChunk / Dt<DT>::NC;
    return (L + spc - 1) / spc;
  }
}
template <int DT>
__device__ __forceinline__ Tile tile_of(const Tensor& T, int c, Split sp, int64_t t) {
  Tile r;
  if constexpr (Dt<DT>::kContig) {
    const int64_t a = (int64_t)c * sp.cs, b = a + sp.cs < T.n ? a + sp.cs : T.n;
    const int64_t kc = a / kChunk + t;
    const int64_t lo = kc * kChunk > a ? kc * kChunk : a, hi = (kc + 1) * kChunk < b ? (kc + 1) * kChunk : b;
    r.slot = slot_of(T.first + kc, a > kc * kChunk ? 1 : 0, T.nall);
    r.s0 = lo - a;
    r.s1 = hi - a;
  } else {
    constexpr int spc = kChunk / Dt<DT>::NC;
    const int64_t L = chain_len<DT>(T, c, sp);
    r.slot = slot_of(T.first + t, c, T.nall);
    r.s0 = t * spc;
    r.s1 = (t + 1) * spc < L ? (t + 1) * spc : L;
  }
  return r;
}
template <int DT>
__device__ __forceinline__ int64_t elem_of(const Tensor& T, int c, Split sp, int64_t s) {
  if constexpr (Dt<DT>::kContig) return T.base + (int64_t)c * sp.cs + s;
  else return T.base + s * Dt<DT>::NC + c;
}

// ---- records
// Per chunk and chain (strided) or piece (fp16) — a "tile" of a chain: the predicted binade g (phase B) and
// the tile's totals on g and g - 1 (phase C): k0 / k1 as fp32 integers (exact below 2^24; +inf where a step
// is too large for the fast path — the tile is then resolved in detail), or, when the tile may hold a tie
// (flag kSide), its exact maps in the side table (double4 {e0, o0, e1, o1}).
struct Rec {
  uint32_t w0, w1;
};
static_assert(sizeof(Rec) == 8, "record layout");
constexpr uint32_t kSide = 1u;      // exact maps in the side table
constexpr uint32_t kPad = 2u;       // phase D: past the chain's end (identity)
constexpr uint32_t kNaN = 4u;       // fp32 (whose S is sampled): the tile holds a NaN
constexpr uint32_t kNoK = 0xffffffu;  // a total of 2^24 - 1 or more (not covered)
// fp32 accumulators: w0 = k0 | flags << 24, w1 = k1 | (g + 128) << 24; fp64 ones: w0 = flags << 24, w1 = g + 2048
template <bool W> __device__ __forceinline__ Rec make_rec(double k0, double k1, int g, uint32_t flags) {
  if constexpr (W) {
    return Rec{flags << 24, (uint32_t)(g + 2048)};
  } else {
    const uint32_t a = k0 < (double)kNoK ? (uint32_t)k0 : kNoK, b = k1 < (double)kNoK ? (uint32_t)k1 : kNoK;
    return Rec{a | (flags << 24), b | ((uint32_t)(g + 128) << 24)};
  }
}
template <bool W> __device__ __forceinline__ int rec_g(Rec r) {
  return W ? (int)(r.w1 & 0xfffu) - 2048 : (int)(r.w1 >> 24) - 128;
}
__device__ __forceinline__ uint32_t rec_flags(Rec r) { return r.w0 >> 24; }
__device__ __forceinline__ double rec_k(Rec r, int j) {  // j = 0 / 1: the total on g / g - 1 (fp32 accumulators)
  const uint32_t k = (j ? r.w1 : r.w0) & kNoK;
  return k == kNoK ? __builtin_inf() : (double)k;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
// x streams through phases A and C once each (1 GiB on C2, beyond the Infinity Cache): non-temporal loads
// (measured: phase A 190 -> 171 us on C2)
// (global address space, so they are global_load, not flat_load, and do not count on lgkmcnt)
__device__ __forceinline__ u32x4 ld_x(const u32x4* p) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)p);
}

// A chunk's elements as 16-byte vectors from the aligned block holding its first element: element e of the
// chunk is position (e + delta) % EPV of vector (e + delta) / EPV (tensors of compact buckets start anywhere).
template <int DT> struct View {
  using St = typename Dt<DT>::S;
  static constexpr int EPV = 16 / (int)sizeof(St);
  static constexpr int NV = (kChunk / EPV + 1 + 255) / 256;  // vectors per thread (256 threads)
  const u32x4* vb;
  int delta, nvec;
  __device__ View(const void* x, int64_t first, int lim) {
    const uintptr_t a = (uintptr_t)((const St*)x + first);
    delta = (int)((a & 15) / sizeof(St));
    vb = (const u32x4*)(a - (a & 15));
    nvec = (delta + lim + EPV - 1) / EPV;
  }
  __device__ static typename Dt<DT>::E elem(const u32x4& r, int p) {
    St el[EPV];
    __builtin_memcpy(el, &r, 16);
    if constexpr (DT == ADFL_DTYPE_F32 || DT == ADFL_DTYPE_F64) return el[p];
    else if constexpr (DT == ADFL_DTYPE_BF16) return __uint_as_float((uint32_t)el[p] << 16);
    else return __half2float(__ushort_as_half(el[p]));
  }
};

// chunk geometry shared by phases A and C
struct ChunkGeo {
  int kc, len, lim, bnd;  // chunk index in the tensor, elements, elements that are chain steps, fp16 piece edge
  int64_t c0e;
};
template <int DT>
__device__ __forceinline__ ChunkGeo geo_of(const Tensor& T, int ci, Split sp) {
  ChunkGeo g;
  g.kc = ci - T.first;
  g.c0e = (int64_t)g.kc * kChunk;
  g.len = (int)(T.n - g.c0e < kChunk ? T.n - g.c0e : kChunk);
  g.bnd = kChunk;
  if constexpr (Dt<DT>::kContig) {
    g.lim = g.len;
    const int64_t b = (g.c0e / sp.cs + 1) * sp.cs - g.c0e;
    g.bnd = b < g.len ? (int)b : kChunk;
  } else {
    const int64_t nv = T.n - T.n % Dt<DT>::VB;
    g.lim = (int)(nv - g.c0e < g.len ? nv - g.c0e : g.len);
  }
  return g;
}

template <int DT>
__device__ __forceinline__ void load_chunk(const View<DT>& v, int tid, u32x4 (&r)[View<DT>::NV]) {
#pragma unroll
  for (int i = 0; i < View<DT>::NV; ++i) {
    const int f = tid + 256 * i;
    const u32x4 q = ld_x(v.vb + (f < v.nvec ? f : v.nvec - 1));  // unconditional (index clamped): all loads in flight
    r[i] = f < v.nvec ? q : u32x4{0u, 0u, 0u, 0u};
  }
}

// ---- phase A: per chunk and chain (piece), the fp64 sum of x^2; also tfirst[t] = t's first chunk
template <int DT>
__global__ __launch_bounds__(256) void k_tn_sums(const void* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                 int threads, int* __restrict__ tfirst, double* __restrict__ S) {
  using D = Dt<DT>;
  using V = View<DT>;
  constexpr int EPV = V::EPV, NV = V::NV;
  __shared__ double s_red[4][8];
  const int ci = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tensor T = tensor_of(chunks, ci, nall);
  if (tid == 0 && ci == T.first) tfirst[T.tensor] = ci;
  if (T.n <= short_max<DT>()) return;
  const Split sp = split_of(T.n, threads);
  const ChunkGeo G = geo_of<DT>(T, ci, sp);
  if (G.lim <= 0) return;  // a chunk of tail elements only: no tile
  const V v(x, T.base + G.c0e, G.lim);
  u32x4 r[NV];
  load_chunk<DT>(v, tid, r);
  double acc[EPV], acc1 = 0.0;  // strided: per vector position; fp16: acc[0] / acc1 = piece 0 / 1
#pragma unroll
  for (int p = 0; p < EPV; ++p) acc[p] = 0.0;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int f = tid + 256 * i;
#pragma unroll
    for (int p = 0; p < EPV; ++p) {
      const int e = f * EPV + p - v.delta;
      const double d = (e >= 0 && e < G.lim) ? (double)V::elem(r[i], p) : 0.0;
      if constexpr (D::kContig) {
        if (e < G.bnd) acc[0] = __fma_rn(d, d, acc[0]);
        else acc1 = __fma_rn(d, d, acc1);
      } else {
        acc[p] = __fma_rn(d, d, acc[p]);
      }
    }
  }
  if constexpr (D::kContig) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      acc[0] += __shfl_xor(acc[0], o, 64);
      acc1 += __shfl_xor(acc1, o, 64);
    }
    if (lane == 0) {
      s_red[wave][0] = acc[0];
      s_red[wave][1] = acc1;
    }
    __syncthreads();
    if (tid < 2 && (tid == 0 || G.bnd < G.len))
      S[slot_of(ci, tid, T.nall)] = s_red[0][tid] + s_red[1][tid] + s_red[2][tid] + s_red[3][tid];
  } else {
    // lanes whose positions map to the same chains: tid % (NC / EPV) (NC / EPV = 2, or 1 for bf16)
    constexpr int kCls = D::NC / EPV;
#pragma unroll
    for (int p = 0; p < EPV; ++p)
#pragma unroll
      for (int o = kCls; o < 64; o <<= 1) acc[p] += __shfl_xor(acc[p], o, 64);
    if (lane < kCls) {
#pragma unroll
      for (int p = 0; p < EPV; ++p) {
        const int c = ((lane * EPV + p - v.delta) % D::NC + D::NC) % D::NC;
        s_red[wave][c] = acc[p];
      }
    }
    __syncthreads();
    if (tid < D::NC)
      S[slot_of(ci, tid, T.nall)] = s_red[0][tid] + s_red[1][tid] + s_red[2][tid] + s_red[3][tid];
  }
}

// fp32 / bf16 phase A: the same sample (16 of a chunk's 256 lines, weighted 16) and tfirst, one wave per chunk and
// kSumsCPW chunks per wave with every load issued first — a block per chunk issued 2 KB and waited (66 us on C2,
// latency-bound); lane l loads vectors f0 = 8 (16 (l / 8) + rot) + l % 8 and f0 + 1024 (lines l / 8 and
// l / 8 + 8 of the sample), so the lanes of one parity hold the same chains and no LDS or barrier is needed.
#ifndef ADFL_TN_SUMS_CPW
#define ADFL_TN_SUMS_CPW 2
#endif
constexpr int kSumsCPW = ADFL_TN_SUMS_CPW;  // chunks per wave in the sampled phase A
// (bf16 — 2-byte elements, 8 to a vector, each vector one element of every chain — takes the same sample: 8 of
// its chunk's 128 lines, lane l loading vector f0 only, and every lane holding all 8 chains)
// (fp16: the same 8 lines; a lane's 8 elements are summed into the chunk's two pieces, split at the piece edge)
template <int DT>
__global__ __launch_bounds__(256) void k_tn_sums_sampled(const void* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks,
                                                         int64_t nall, int threads, int* __restrict__ tfirst,
                                                         double* __restrict__ S) {
  using V = View<DT>;
  constexpr bool kC = Dt<DT>::kContig;
  constexpr int EPV = V::EPV;            // 4 (fp32) / 8 (bf16)
  constexpr int NH = EPV == 4 ? 2 : 1;   // vectors per lane: 16 sampled lines of 256 (fp32) / 8 of 128 (bf16)
  constexpr int kCls = 8 / EPV;          // lanes of one class hold the same chains
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c0 = ((int64_t)blockIdx.x * 4 + wave) * kSumsCPW;
  const u32x4* const x0 = (const u32x4*)((uintptr_t)x & ~(uintptr_t)15);  // a valid address for idle lanes
  u32x4 r[kSumsCPW][NH];
  bool live[kSumsCPW];
  int delta[kSumsCPW], lim[kSumsCPW], f0[kSumsCPW], bnd[kSumsCPW], len[kSumsCPW];
#pragma unroll
  for (int j = 0; j < kSumsCPW; ++j) {
    const int64_t ci = c0 + j;
    live[j] = false;
    delta[j] = lim[j] = f0[j] = bnd[j] = len[j] = 0;
    const u32x4* p[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) p[h] = x0;
    if (ci < nall) {
      const Tensor T = tensor_of(chunks, (int)ci, nall);
      if (lane == 0 && ci == T.first) tfirst[T.tensor] = (int)ci;
      const ChunkGeo G = geo_of<DT>(T, (int)ci, kC ? split_of(T.n, threads) : Split{1, T.n});
      if (T.n > short_max<DT>() && G.lim > 0) {
        const V v(x, T.base + G.c0e, G.lim);
        live[j] = true;
        delta[j] = v.delta;
        lim[j] = G.lim;
        bnd[j] = G.bnd;
        len[j] = G.len;
        f0[j] = 8 * (16 * (lane >> 3) + (int)((ci * 7) & 15)) + (lane & 7);
#pragma unroll
        for (int h = 0; h < NH; ++h) p[h] = v.vb + (f0[j] + 1024 * h < v.nvec ? f0[j] + 1024 * h : v.nvec - 1);
      }
    }
#pragma unroll
    for (int h = 0; h < NH; ++h) r[j][h] = ld_x(p[h]);
  }
#pragma unroll
  for (int j = 0; j < kSumsCPW; ++j) {
    if (!live[j]) continue;  // uniform over the wave
    if constexpr (kC) {  // fp16: two pieces at most, every lane holding both
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int q = 0; q < EPV; ++q) {
        const int e = f0[j] * EPV + q - delta[j];
        const double d = (e >= 0 && e < lim[j]) ? (double)V::elem(r[j][0], q) : 0.0;
        if (e < bnd[j]) a0 = __fma_rn(d, d, a0);
        else a1 = __fma_rn(d, d, a1);
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        a0 += __shfl_xor(a0, o, 64);
        a1 += __shfl_xor(a1, o, 64);
      }
      if (lane == 0) {
        S[slot_of(c0 + j, 0, nall)] = a0 * 16.0;
        if (bnd[j] < len[j]) S[slot_of(c0 + j, 1, nall)] = a1 * 16.0;
      }
      continue;
    }
    double acc[EPV];
#pragma unroll
    for (int q = 0; q < EPV; ++q) acc[q] = 0.0;
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int q = 0; q < EPV; ++q) {
        const int e = (f0[j] + 1024 * h) * EPV + q - delta[j];
        const double d = (e >= 0 && e < lim[j]) ? (double)V::elem(r[j][h], q) : 0.0;
        acc[q] = __fma_rn(d, d, acc[q]);
      }
    // reduce-scatter over the lanes of a class: halve the values a lane holds at lane bits 5, 4 (, 3), then
    // sum the one left over the remaining bits down to kCls — 10 (bf16) / 6 (fp32) shuffles instead of 48 / 20
    int qb = 0;  // the first value index this lane still holds
#pragma unroll
    for (int o = 32, n = EPV; n > 1; o >>= 1) {
      n >>= 1;
      const bool hi = (lane & o) != 0;
#pragma unroll
      for (int i = 0; i < n; ++i) {
        const double give = hi ? acc[i] : acc[i + n], keep = hi ? acc[i + n] : acc[i];
        acc[i] = keep + __shfl_xor(give, o, 64);
      }
      if (hi) qb += n;
    }
    constexpr int kLow = 64 / EPV;  // lane bits below this: still to be summed (down to kCls)
#pragma unroll
    for (int o = kLow / 2; o >= kCls; o >>= 1) acc[0] += __shfl_xor(acc[0], o, 64);
    if ((lane & (kLow - 1)) < kCls) {  // one lane per (class, value)
      const int cls = lane & (kCls - 1);
      S[slot_of(c0 + j, ((cls * EPV + qb - delta[j]) % 8 + 8) % 8, nall)] = acc[0] * 16.0;
    }
  }
}

// ---- phase B: per chain, the exclusive prefix P of S at each tile -> the tile's predicted binade (rec.g).
// P is only a prediction (a tile whose binade it misses is not covered and is resolved in detail), so its
// summation order is free: B1 sums each window's S, B2 adds the windows before it to a scan inside the
// window. One wave per window (lane l: tiles l * kTPL ..), grid (tensors, 8, 8): blockIdx.y strides the
// chains, blockIdx.z and the wave the windows.
template <int DT>
__global__ __launch_bounds__(256) void k_tn_winsums(const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                    const int* __restrict__ tfirst, int threads,
                                                    const double* __restrict__ S, double* __restrict__ wsum) {
  using D = Dt<DT>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tensor T = tensor_of(chunks, tfirst[blockIdx.x], nall);
  if (T.n <= short_max<DT>()) return;
  const Split sp = split_of(T.n, threads);
  const int nchains = D::kContig ? (int)sp.nt : D::NC;
  const int wstride = gridDim.z * 4;
  for (int c = blockIdx.y; c < nchains; c += gridDim.y) {
    const int64_t nt = chain_tiles<DT>(T, c, sp);
    const int64_t nw = (nt + kWinTiles - 1) / kWinTiles;
    for (int64_t w = blockIdx.z * 4 + wave; w < nw; w += wstride) {
      const int64_t w0 = w * kWinTiles;
      double a = 0.0;
#pragma unroll
      for (int k = 0; k < kTPL; ++k) {
        const int64_t t = w0 + lane * kTPL + k;
        const double v = S[tile_of<DT>(T, c, sp, t < nt ? t : nt - 1).slot];  // clamped: loads in flight
        a += t < nt ? v : 0.0;
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
      if (lane == 0) wsum[tile_of<DT>(T, c, sp, w0).slot] = a;
    }
  }
}

template <int DT>
__global__ __launch_bounds__(256) void k_tn_grids(const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                  const int* __restrict__ tfirst, int threads, const double* __restrict__ S,
                                                  const double* __restrict__ wsum, Rec* __restrict__ recs) {
  using D = Dt<DT>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tensor T = tensor_of(chunks, tfirst[blockIdx.x], nall);
  if (T.n <= short_max<DT>()) return;
  const Split sp = split_of(T.n, threads);
  const int nchains = D::kContig ? (int)sp.nt : D::NC;
  const int wstride = gridDim.z * 4;
  for (int c = blockIdx.y; c < nchains; c += gridDim.y) {
    const int64_t nt = chain_tiles<DT>(T, c, sp);
    const int64_t nw = (nt + kWinTiles - 1) / kWinTiles;
    for (int64_t w = blockIdx.z * 4 + wave; w < nw; w += wstride) {
      const int64_t w0 = w * kWinTiles;
      double y[kTPL], a = 0.0;
#pragma unroll
      for (int k = 0; k < kTPL; ++k) {
        const int64_t t = w0 + lane * kTPL + k;
        const double v = S[tile_of<DT>(T, c, sp, t < nt ? t : nt - 1).slot];  // clamped: loads in flight
        y[k] = t < nt ? v : 0.0;
        a += y[k];
      }
      double base = 0.0;  // the windows before this one
      for (int64_t j = lane; j < w; j += 64) base += wsum[tile_of<DT>(T, c, sp, j * kWinTiles).slot];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) base += __shfl_xor(base, o, 64);
      double P = base + wave_excl_sum(a, lane);
#pragma unroll
      for (int k = 0; k < kTPL; ++k) {
        const int64_t t = w0 + lane * kTPL + k;
        // fp32's, bf16's and fp16's S is sampled: P is raised by a margin that covers the sample's error (a Gaussian tile's sampled
        // sum is within about 18% of its own, a prefix of t tiles within 18% / sqrt(t)); P may overshoot the
        // accumulator by up to 2x and still predict it (the maps are on g and g - 1), not undershoot it
        const double Pm = !D::kWide ? P * (1.0 + fmin(0.9, 1.0 / __builtin_sqrt((double)t + 1.0))) : P;
        if (t < nt) recs[tile_of<DT>(T, c, sp, t).slot] = make_rec<D::kWide>(0.0, 0.0, grid_pred<D::kWide>(Pm), 0u);
        P += y[k];
      }
    }
  }
}

// ---- phase C: per chunk and chain (piece), the totals on the predicted binades g and g - 1
// Fast path, order-free: with hi = RN(x^2 / u) in the accumulator's type, k = rint(hi) is R(x^2 / u)
// unless hi - k = +-1/2 (where the exact value decides, and a tie is possible) — and on g - 1, R(2 x^2 / u)
// = 2 k + rint(2 (hi - k)), exact unless hi - k = +-1/4. A chunk where any lane meets one of those is listed
// for k_tn_maps_exact: staged chain-major through LDS, each lane's 16 steps composed in order as maps.
template <int DT>
__global__ __launch_bounds__(256) void k_tn_maps(const void* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                 int threads, Rec* __restrict__ recs, double4* __restrict__ maps,
                                                 int* __restrict__ exact_list) {
  using D = Dt<DT>;
  using V = View<DT>;
  constexpr bool W = D::kWide;
  using A_t = typename Acc<W>::T;
  constexpr int EPV = V::EPV, NV = V::NV;
  constexpr A_t kM = W ? (A_t)6755399441055744.0 : (A_t)12582912.0f;   // 1.5 * 2^52 / 1.5 * 2^23
  constexpr A_t kBig = W ? (A_t)0x1p50 : (A_t)0x1p21;                   // hi at or above: rint(2 hi) by kM fails
  // the largest square (NaN: not covered): fp32 as its bit pattern (squares are >= +0, NaN's pattern is above
  // +inf's, so an unsigned max propagates it in one instruction); fp64 by value, NaN replaced by +inf
  using M_t = typename std::conditional<W, double, uint32_t>::type;
  __shared__ A_t s_k[4][8][2];
  __shared__ M_t s_mx[4][8];
  __shared__ int s_g[8], s_slow, s_fl[4][8];
  const int ci = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tensor T = tensor_of(chunks, ci, nall);
  if (T.n <= short_max<DT>()) return;
  const Split sp = split_of(T.n, threads);
  const ChunkGeo G = geo_of<DT>(T, ci, sp);
  if (G.lim <= 0) return;
  const int npieces = D::kContig ? (G.bnd < G.len ? 2 : 1) : D::NC;
  const V v(x, T.base + G.c0e, G.lim);
  u32x4 r[NV];
  load_chunk<DT>(v, tid, r);  // first: the record load below must not hold the chunk's loads back
  if (tid < npieces) s_g[tid] = rec_g<W>(recs[slot_of(ci, tid, T.nall)]);
  __syncthreads();
  // per position (strided) or piece (fp16): scale of x so hi = x^2 / u on g: xs = x 2^(s >> 1), hi = xs xs (2)
  constexpr int kP = D::kContig ? 2 : EPV;
  A_t sa[kP], sb[kP];
#pragma unroll
  for (int p = 0; p < kP; ++p) {
    const int c = D::kContig ? (p < npieces ? p : 0) : ((tid * EPV + p - v.delta) % D::NC + D::NC) % D::NC;
    const int s = Acc<W>::kM - s_g[c];
    sa[p] = (A_t)pow2(s >> 1);
    sb[p] = (s & 1) ? (A_t)2 : (A_t)1;
  }
  // per element: k = rint(hi) and k1 = rint(2 hi) (the totals on g and g - 1), the largest hi, and whether
  // |hi - k| is 1/2 or 1/4 (a tie on g or g - 1 the rounding of hi may hide: the chunk goes to the exact path)
  A_t K0[kP], K1[kP];
  M_t mx[kP];
  bool fl[kP];
#pragma unroll
  for (int p = 0; p < kP; ++p) {
    K0[p] = K1[p] = (A_t)0;
    mx[p] = (M_t)0;
    fl[p] = false;
  }
  const auto step = [&](A_t xv, int q) {
    const A_t xs = xv * sa[q];
    const A_t hi = xs * xs * sb[q];
    const A_t k = (hi + kM) - kM;
    const A_t rr = hi - k;
    const A_t ar = __builtin_fabs(rr);
    K0[q] += k;
    K1[q] += (hi * (A_t)2 + kM) - kM;
    if constexpr (W) mx[q] = (hi == hi) ? __builtin_fmax(mx[q], hi) : (M_t)__builtin_inf();
    else mx[q] = max(mx[q], __float_as_uint(hi));
    fl[q] |= (ar == (A_t)0.5) | (ar == (A_t)0.25);
  };
  if (v.delta == 0 && G.lim == kChunk && G.bnd >= G.len) {  // a whole chunk of one piece: no masks
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int p = 0; p < EPV; ++p) step((A_t)V::elem(r[i], p), D::kContig ? 0 : p);
  } else {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
#pragma unroll
      for (int p = 0; p < EPV; ++p) {
        const int e = f * EPV + p - v.delta;
        step((e >= 0 && e < G.lim) ? (A_t)V::elem(r[i], p) : (A_t)0, D::kContig ? (e < G.bnd ? 0 : 1) : p);
      }
    }
  }
  if (tid == 0) s_slow = 0;
  const auto mx_max = [](M_t a, M_t b) -> M_t {
    if constexpr (W) return __builtin_fmax(a, b);
    else return max(a, b);
  };
  if constexpr (D::kContig) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        K0[p] += __shfl_xor(K0[p], o, 64);
        K1[p] += __shfl_xor(K1[p], o, 64);
        mx[p] = mx_max(mx[p], __shfl_xor(mx[p], o, 64));
      }
      fl[p] = __ballot(fl[p]) != 0ull;
    }
    if (lane < 2) {
      s_k[wave][lane][0] = lane ? K0[1] : K0[0];
      s_k[wave][lane][1] = lane ? K1[1] : K1[0];
      s_mx[wave][lane] = lane ? mx[1] : mx[0];
      s_fl[wave][lane] = lane ? fl[1] : fl[0];
    }
  } else {
    constexpr int kCls = D::NC / EPV;
#pragma unroll
    for (int p = 0; p < EPV; ++p) {
#pragma unroll
      for (int o = kCls; o < 64; o <<= 1) {
        K0[p] += __shfl_xor(K0[p], o, 64);
        K1[p] += __shfl_xor(K1[p], o, 64);
        mx[p] = mx_max(mx[p], __shfl_xor(mx[p], o, 64));
      }
      // lanes of one class (lane % kCls) hold the same chains: the flag per class from the wave's ballot
      const unsigned long long b = __ballot(fl[p]);
      fl[p] = (b & (kCls == 1 ? ~0ull : (0x5555555555555555ull << (lane & 1)))) != 0ull;
    }
    if (lane < kCls) {
#pragma unroll
      for (int p = 0; p < EPV; ++p) {
        const int c = ((lane * EPV + p - v.delta) % D::NC + D::NC) % D::NC;
        s_k[wave][c][0] = K0[p];
        s_k[wave][c][1] = K1[p];
        s_mx[wave][c] = mx[p];
        s_fl[wave][c] = fl[p];
      }
    }
  }
  __syncthreads();
  if (tid < npieces) {
    A_t k0 = 0, k1 = 0;
    M_t m = 0;
    bool f = false;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      k0 += s_k[w][tid][0];
      k1 += s_k[w][tid][1];
      m = mx_max(m, s_mx[w][tid]);
      f |= s_fl[w][tid] != 0;
    }
    const int g = s_g[tid];
    bool big;
    if constexpr (W) big = !(m < kBig);
    else big = m >= __float_as_uint(kBig);
    const double inf = __builtin_inf();
    const double e0 = big ? inf : (double)k0;
    const double e1 = (!big && g - 1 >= Acc<W>::kGmin) ? (double)k1 : inf;
    // a possible tie matters only where a total can still be covered (below 2^24 / 2^53)
    if (f && (e0 < Acc<W>::kTop || e1 < Acc<W>::kTop)) s_slow = 1;
    const int64_t slot = slot_of(ci, tid, T.nall);
    if constexpr (W) {
      maps[slot] = make_double4(e0, e0, e1, e1);
      recs[slot] = make_rec<W>(0.0, 0.0, g, kSide);
    } else {
      recs[slot] = make_rec<W>(e0, e1, g, 0u);
    }
  }
  __syncthreads();
  if (tid == 0 && s_slow) exact_list[atomicAdd(exact_list - 1, 1)] = ci;  // the count sits just before the list
}

// fp32 phase C: a tile's totals on its predicted binade g and on g - 1 as exact increments, order-free: on a
// normal grid G (ulp u = 2^(G-23)) a step adds fma(x, x, 2^G) - 2^G (k_tn_short's argument: exact unless x^2 is
// at or above 2^G, which then makes the total at least 2^23 u — never covered from A >= 2^23), summed in fp32
// (exact below 2^24 u, at least that above). A tie leaves the residual x^2 - k at exactly +-u/2, which
// fma(-x, x, k) returns exactly, so a chunk where some |residual| equals u/2 (rarely a rounding, not a tie) goes
// to k_tn_maps_exact; so does a chunk with a chain predicted on the subnormal grid. A NaN sets its tile's kNaN
// (S is sampled for fp32, so it cannot tell phase D). One read of x; no fp64.
__global__ __launch_bounds__(256) void k_tn_maps_f32(const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks,
                                                     int64_t nall, Rec* __restrict__ recs, int* __restrict__ exact_list) {
  using V = View<ADFL_DTYPE_F32>;
  constexpr int EPV = V::EPV, NV = V::NV;
  __shared__ float s_k[4][8][2];
  __shared__ int s_g[8], s_slow, s_fl[4][8];
  const int ci = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tensor T = tensor_of(chunks, ci, nall);
  if (T.n <= kShortMaxF32) return;
  const ChunkGeo G = geo_of<ADFL_DTYPE_F32>(T, ci, Split{1, T.n});
  if (G.lim <= 0) return;
  const V v(x, T.base + G.c0e, G.lim);
  u32x4 r[NV];
  load_chunk<ADFL_DTYPE_F32>(v, tid, r);  // first: the record load below must not hold the chunk's loads back
  if (tid < 8) s_g[tid] = rec_g<false>(recs[slot_of(ci, tid, T.nall)]);
  if (tid == 0) s_slow = 0;
  __syncthreads();
  // per position p: its chain's grids g and g - 1 as one pair (packed fp32: B = 2^g, 2^(g-1); h = the half-ulps)
  f2v B[EPV], h[EPV];
#pragma unroll
  for (int p = 0; p < EPV; ++p) {
    const int g = s_g[((tid * EPV + p - v.delta) % 8 + 8) % 8];
    B[p] = f2v{pow2f(g), pow2f(g - 1 < -126 ? -126 : g - 1)};  // (g - 1 < -126: not a grid; e1 is +inf below)
    h[p] = f2v{pow2fs(g - 24 < -149 ? -149 : g - 24), pow2fs(g - 25 < -149 ? -149 : g - 25)};
  }
  // per element: k = fma(x, x, B) - B and the residual fma(-x, x, k) on both grids (two packed fmas, a packed
  // add, a packed accumulate); a half-ulp residual is a wave mask accumulated in scalar registers (one compare
  // per grid). A NaN is left to propagate into K (every k >= 0, so K is NaN exactly when an input was).
  f2v K[EPV];
  unsigned long long fm[EPV];
#pragma unroll
  for (int p = 0; p < EPV; ++p) {
    K[p] = f2v{0.0f, 0.0f};
    fm[p] = 0ull;
  }
  const auto step = [&](float xv, int p) {
    const f2v xx = f2v{xv, xv};
    const f2v k = __builtin_elementwise_fma(xx, xx, B[p]) - B[p];
    K[p] += k;
    const f2v rr = __builtin_elementwise_fma(-xx, xx, k);
    fm[p] |= __ballot(__builtin_fabsf(rr.x) == h[p].x);
    fm[p] |= __ballot(__builtin_fabsf(rr.y) == h[p].y);
  };
  if (v.delta == 0 && G.lim == kChunk) {  // a whole aligned chunk: no masks
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int p = 0; p < EPV; ++p) step(V::elem(r[i], p), p);
  } else {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
#pragma unroll
      for (int p = 0; p < EPV; ++p) {
        const int e = f * EPV + p - v.delta;
        step((e >= 0 && e < G.lim) ? V::elem(r[i], p) : 0.0f, p);
      }
    }
  }
  // lanes of one parity hold the same chains (positions p -> chains (4 tid + p - delta) % 8)
#pragma unroll
  for (int p = 0; p < EPV; ++p) {
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) {
      K[p].x += __shfl_xor(K[p].x, o, 64);
      K[p].y += __shfl_xor(K[p].y, o, 64);
    }
  }
  if (lane < 2) {
#pragma unroll
    for (int p = 0; p < EPV; ++p) {
      const int c = ((lane * EPV + p - v.delta) % 8 + 8) % 8;
      s_k[wave][c][0] = K[p].x;
      s_k[wave][c][1] = K[p].y;
      s_fl[wave][c] = (fm[p] & (0x5555555555555555ull << lane)) != 0ull;
    }
  }
  __syncthreads();
  if (tid < 8) {
    float k0 = 0.0f, k1 = 0.0f;
    int f = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      k0 += s_k[w][tid][0];
      k1 += s_k[w][tid][1];
      f |= s_fl[w][tid];
    }
    const int g = s_g[tid];
    // the totals in ulps of g and g - 1, exact integers below 2^24 (kNoK: not covered; NaN / inf included)
    const double inf = __builtin_inf();
    const double q0 = (double)k0 * pow2(23 - g), q1 = (double)k1 * pow2(24 - g);
    const double e0 = q0 < (double)kNoK ? q0 : inf;
    const double e1 = (g - 1 >= -126 && q1 < (double)kNoK) ? q1 : inf;
    // a residual on the subnormal grid (g - 1 = -126) cannot show a tie: such a chain goes to the exact path
    if ((f || g - 1 <= -126) && (e0 < Acc<false>::kTop || e1 < Acc<false>::kTop)) s_slow = 1;
    recs[slot_of(ci, tid, T.nall)] = make_rec<false>(e0, e1, g, (k0 != k0 || k1 != k1) ? kNaN : 0u);
  }
  __syncthreads();
  if (tid == 0 && s_slow) exact_list[atomicAdd(exact_list - 1, 1)] = ci;  // the count sits just before the list
}

// The listed chunks (bf16 / fp16: every long tensor's chunk), exactly: chain-major staging (16 steps per lane
// block, +1 pad), maps composed in order.
template <int DT>
__global__ __launch_bounds__(256) void k_tn_maps_exact(const void* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                       int threads, Rec* __restrict__ recs, double4* __restrict__ maps,
                                                       const int* __restrict__ exact_list) {
  using D = Dt<DT>;
  using V = View<DT>;
  using E = typename D::E;
  constexpr bool W = D::kWide;
  constexpr int EPV = V::EPV, NV = V::NV;
  constexpr int kLS = kLane + 1;
  __shared__ E st[8 * 64 * kLS];  // 8 rows of 1024 steps (strided: chain-major; fp16: the chunk in order)
  __shared__ double s_m[4][2][4];
  __shared__ int s_g[8];
  __shared__ uint32_t s_nf[8];
  // bf16 / fp16 (whose S is a sample that may miss a NaN): whether the chunk holds a NaN, double-buffered by iteration
  // (set while staging, read after the barrier, the other buffer cleared for the next iteration)
  __shared__ int s_anynan[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr bool kNanScan = DT == ADFL_DTYPE_BF16 || DT == ADFL_DTYPE_F16;
  if (kNanScan && tid == 0) s_anynan[0] = s_anynan[1] = 0;
  if (kNanScan) __syncthreads();
  // exact_list NULL: every chunk of a long tensor (exact-square dtypes, whose ties are real and frequent: phase
  // C's order-free pass listed nearly every chunk anyway, so it is skipped)
  const int count = exact_list ? exact_list[-1] : (int)nall;
  int it = 0;
  for (int li = blockIdx.x; li < count; li += gridDim.x) {
    const int ci = exact_list ? exact_list[li] : li;
    const Tensor T = tensor_of(chunks, ci, nall);
    const Split sp = split_of(T.n, threads);
    const ChunkGeo G = geo_of<DT>(T, ci, sp);
    if (!exact_list && (T.n <= short_max<DT>() || G.lim <= 0)) continue;  // (block-uniform)
    const int npieces = D::kContig ? (G.bnd < G.len ? 2 : 1) : D::NC;
    if (tid < npieces) {
      const Rec q = recs[slot_of(ci, tid, T.nall)];
      s_g[tid] = rec_g<W>(q);
      s_nf[tid] = rec_flags(q) & kNaN;
    }
    const V v(x, T.base + G.c0e, G.lim);
    u32x4 r[NV];
    load_chunk<DT>(v, tid, r);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
#pragma unroll
      for (int p = 0; p < EPV; ++p) {
        const int e = f * EPV + p - v.delta;
        if (e >= 0 && e < G.lim) {
          int row, sl;
          if constexpr (D::kContig) {
            row = e / kSeg;
            sl = e % kSeg;
          } else {  // steps per chain in a chunk: 1024 (NC 8) or 2048 (NC 4)
            const int c = e % D::NC, s = e / D::NC;
            row = D::NC == 8 ? c : c * 2 + s / kSeg;
            sl = s % kSeg;
          }
          const E el = V::elem(r[i], p);
          if constexpr (kNanScan) {
            if (el != el) s_anynan[it & 1] = 1;
          }
          st[row * 64 * kLS + (sl / kLane) * kLS + sl % kLane] = el;
        }
      }
    }
    __syncthreads();
    // fp16: wave w composes rows 2w, 2w + 1 (elements [2048 w, 2048 w + 2048)) for each piece; strided: the
    // rows w and w + 4 (fp32 / bf16: chains w, w + 4; fp64: halves of chains)
    Map acc0[2] = {Map{0.0, 0.0}, Map{0.0, 0.0}}, acc1[2] = {Map{0.0, 0.0}, Map{0.0, 0.0}};
    for (int h = 0; h < 2; ++h) {
      const int row = D::kContig ? wave * 2 + h : wave + 4 * h;
      E w[kLane];
#pragma unroll
      for (int i = 0; i < kLane; ++i) {
        const int e = row * kSeg + lane * kLane + i;  // fp16: the chunk element; strided: the row's step
        w[i] = (!D::kContig || e < G.lim) ? st[row * 64 * kLS + lane * kLS + i] : (E)0;
      }
      if constexpr (D::kContig) {
        for (int pc = 0; pc < npieces; ++pc) {  // steps outside a piece are zeros (identity); one piece: one pass
          E z[kLane];
#pragma unroll
          for (int i = 0; i < kLane; ++i) {
            const int e = row * kSeg + lane * kLane + i;
            z[i] = (pc == 0 ? e < G.bnd : e >= G.bnd) ? w[i] : (E)0;
          }
          const int g = s_g[pc < npieces ? pc : 0];
          Map l0, l1;
          lane_maps_pair<W, D::kSq>(z, g, -1, l0, l1);
          if constexpr (D::kSq) {  // integer maps: fp32 DPP composition (round 6)
            acc0[pc] = compose(acc0[pc], wave_compose_f(l0));
            acc1[pc] = compose(acc1[pc], wave_compose_f(l1));
          } else {
            acc0[pc] = compose(acc0[pc], wave_compose(l0, lane));
            acc1[pc] = compose(acc1[pc], wave_compose(l1, lane));
          }
        }
      } else {
        const int g = s_g[D::NC == 8 ? row : row / 2];
        // rows past the chunk's steps are zeros: LDS left from an earlier chunk must not count
        const int c = D::NC == 8 ? row : row / 2, s0 = (D::NC == 8 ? 0 : (row % 2) * kSeg);
#pragma unroll
        for (int i = 0; i < kLane; ++i) {
          const int e = (s0 + lane * kLane + i) * D::NC + c;
          if (e >= G.lim) w[i] = (E)0;
        }
        Map l0, l1;
        lane_maps_pair<W, D::kSq>(w, g, -1, l0, l1);
        Map m0, m1;
        if constexpr (D::kSq) {  // integer maps: fp32 DPP composition (round 6)
          m0 = wave_compose_f(l0);
          m1 = wave_compose_f(l1);
        } else {
          m0 = wave_compose(l0, lane);
          m1 = wave_compose(l1, lane);
        }
        if (lane == 0) {
          s_m[wave][h][0] = m0.e;
          s_m[wave][h][1] = m0.o;
          s_m[wave][h][2] = m1.e;
          s_m[wave][h][3] = m1.o;
        }
      }
    }
    if constexpr (D::kContig) {
      if (lane == 0)
        for (int pc = 0; pc < 2; ++pc) {
          s_m[wave][pc][0] = acc0[pc].e;
          s_m[wave][pc][1] = acc0[pc].o;
          s_m[wave][pc][2] = acc1[pc].e;
          s_m[wave][pc][3] = acc1[pc].o;
        }
    }
    __syncthreads();
    if (tid < npieces) {
      Map a0{0.0, 0.0}, a1{0.0, 0.0};
      if constexpr (D::kContig) {
        for (int w = 0; w < 4; ++w) {
          a0 = compose(a0, Map{s_m[w][tid][0], s_m[w][tid][1]});
          a1 = compose(a1, Map{s_m[w][tid][2], s_m[w][tid][3]});
        }
      } else if (D::NC == 8) {  // chain c = row c: wave c % 4, half c / 4
        a0 = Map{s_m[tid % 4][tid / 4][0], s_m[tid % 4][tid / 4][1]};
        a1 = Map{s_m[tid % 4][tid / 4][2], s_m[tid % 4][tid / 4][3]};
      } else {  // NC 4: chain c = rows 2c, 2c + 1
        const int r0 = 2 * tid, r1 = 2 * tid + 1;
        a0 = compose(Map{s_m[r0 % 4][r0 / 4][0], s_m[r0 % 4][r0 / 4][1]}, Map{s_m[r1 % 4][r1 / 4][0], s_m[r1 % 4][r1 / 4][1]});
        a1 = compose(Map{s_m[r0 % 4][r0 / 4][2], s_m[r0 % 4][r0 / 4][3]}, Map{s_m[r1 % 4][r1 / 4][2], s_m[r1 % 4][r1 / 4][3]});
      }
      const int g = s_g[tid];
      if (g - 1 < Acc<W>::kGmin) a1 = Map{__builtin_inf(), __builtin_inf()};
      const int64_t slot = slot_of(ci, tid, T.nall);
      maps[slot] = make_double4(a0.e, a0.o, a1.e, a1.o);
      const uint32_t nf = s_nf[tid] | ((kNanScan && s_anynan[it & 1]) ? kNaN : 0u);
      recs[slot] = make_rec<W>(0.0, 0.0, g, kSide | nf);
    }
    if (kNanScan && tid == 0) s_anynan[(it + 1) & 1] = 0;
    ++it;
    __syncthreads();
  }
}

// ---- phase C2: window summaries. A window is kWinTiles consecutive tiles of a chain; its summary is the
// composition of its tiles' maps on G = gw (every tile predicted on gw) and on gw - 1 (every tile predicted on
// gw or gw - 1), gw the window's highest predicted binade; a map that does not exist is +inf. One wave per
// window; grid (tensors, 8, 8): blockIdx.y strides chains, blockIdx.z and the wave stride windows.
template <int DT>
__global__ __launch_bounds__(256) void k_tn_windows(const adfl_slq_chunk* __restrict__ chunks, int64_t nall, const int* __restrict__ tfirst,
                                                    int threads, const Rec* __restrict__ recs, const double4* __restrict__ maps,
                                                    int* __restrict__ wing, double4* __restrict__ winmaps) {
  using D = Dt<DT>;
  constexpr bool W = D::kWide;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Tensor T = tensor_of(chunks, tfirst[blockIdx.x], nall);
  if (T.n <= short_max<DT>()) return;
  const Split sp = split_of(T.n, threads);
  const int nchains = D::kContig ? (int)sp.nt : D::NC;
  const int wstride = gridDim.z * 4;
  for (int c = blockIdx.y; c < nchains; c += gridDim.y) {
    const int64_t nt = chain_tiles<DT>(T, c, sp);
    const int64_t nw = (nt + kWinTiles - 1) / kWinTiles;
    for (int64_t w = blockIdx.z * 4 + wave; w < nw; w += wstride) {
      const int64_t w0 = w * kWinTiles;
      Rec r[kTPL];
      int gmax = -0x7fffffff;
#pragma unroll
      for (int k = 0; k < kTPL; ++k) {
        const int64_t t = w0 + lane * kTPL + k;
        const Rec q = recs[tile_of<DT>(T, c, sp, t < nt ? t : nt - 1).slot];  // clamped: loads in flight
        r[k] = t < nt ? q : Rec{kPad << 24, 0u};
        if (t < nt) gmax = max(gmax, rec_g<W>(r[k]));
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) gmax = max(gmax, __shfl_xor(gmax, o, 64));
      Map a{0.0, 0.0}, b{0.0, 0.0};
#pragma unroll
      for (int k = 0; k < kTPL; ++k) {
        const Rec q = r[k];
        const uint32_t fl = rec_flags(q);
        if (fl & kPad) continue;
        const int g = rec_g<W>(q);
        Map m0, m1;  // the tile's maps on g and g - 1
        if (fl & kSide) {
          const double4 m = maps[tile_of<DT>(T, c, sp, w0 + lane * kTPL + k).slot];
          m0 = Map{m.x, m.y};
          m1 = Map{m.z, m.w};
        } else {
          const double k0 = rec_k(q, 0), k1 = rec_k(q, 1);
          m0 = Map{k0, k0};
          m1 = Map{k1, k1};
        }
        const Map inf{__builtin_inf(), __builtin_inf()};
        a = compose(a, g == gmax ? m0 : inf);                        // on gmax: j = g - gmax must be 0
        b = compose(b, g == gmax ? m1 : (g == gmax - 1 ? m0 : inf));  // on gmax - 1: j = 1 or 0
      }
      a = wave_compose(a, lane);
      b = wave_compose(b, lane);
      if (lane == 0) {
        const int64_t slot = tile_of<DT>(T, c, sp, w0).slot;
        wing[slot] = gmax;
        winmaps[slot] = make_double4(a.e, a.o, b.e, b.o);
      }
    }
  }
}

// ---- short fp32 tensors: k_tn_short, one block per tensor, one wave per chain, one launch
// The fp32 form of the binade model, with no fp64 and no integer conversion. On binade G (ulp u = 2^(G-23),
// A = acc / u in [2^23, 2^24); G = -126 also holds the subnormals) a step adds R(x^2 / u) * u, which is exactly
// fma(x, x, B) - B for B = 2^G (A = 2^23, even) whenever x^2 < 2^G — the fma rounds B + x^2 on G's own grid —
// and for B = +0 on G = -126 (RN(x^2) is then on the subnormal grid). Increments and their sums are multiples of
// u, exact in fp32 below 2^24 u; above it every sum still rounds to at least 2^24 u (RN is monotone and the terms
// are >= 0), so acc + the sum of a run stays below 2^(G+1) exactly when the run is covered, and a step of
// x^2 >= 2^G (whose fma leaves the binade) is never covered. The increment agrees with the even-A rounding of the
// step; odd A differs only on a tie (x^2 / u = f + 1/2), and a tie on G or on G + 1 needs x^2 to be a multiple
// of u / 2: 2 lsb(x) >= G - 24, with lsb(x) = E - 150 + ctz(mantissa | 2^23) for x's biased exponent E (a
// subnormal x squares far below u / 2). A lane whose 16 steps cannot rule that out sends its round down the
// exact map path (lane_map_exact, fp64). Measured against k_norm_walk (the chains run in order) and torch
// itself: tests/test_gpu_torch_norm.py, test_gpu_torch_norm_dt.py.
constexpr int kShThreads = 512;                 // wave c runs chain c
#ifndef ADFL_TN_SHORT_SL
#define ADFL_TN_SHORT_SL 16
#endif
constexpr int kSL = ADFL_TN_SHORT_SL;           // steps per lane's run (a segment: 64 kSL steps of each chain)
constexpr int kShSeg = 8 * 64 * kSL;            // elements per segment (16384)
constexpr int kShLS = kSL + 4;                  // floats per lane's run in LDS (+4: 16-byte reads, no conflicts)
constexpr int kShRow = 64 * kShLS + 8;          // floats per chain (+8: chains c and c + 4 alone share banks)
constexpr int kShVec = kShSeg / 4 / kShThreads; // 16-byte loads per thread per segment

// the n % 8 tail after the lane sum (and the whole sum below 8 elements) as torch's compiled scalar loop runs
// it: 4 rounded squares added in order when there are 4 or more, the rest with fma (as k_norm_walk's tail_sum)
__device__ __forceinline__ float tail32(const float* x, int64_t d, int64_t n, float b) {
  if (n - d >= 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float sq = x[d + k] * x[d + k];
      b = b + sq;
    }
    d += 4;
  }
  for (int64_t i = d; i < n; ++i) b = __builtin_fmaf(x[i], x[i], b);
  return b;
}

// inclusive wave scan in fp32 by DPP (row shifts, then the row broadcasts 15 and 31): exact on multiples of u
// whose sums stay below 2^24 u, a lower bound of 2^24 u otherwise (any summation tree of terms >= 0)
__device__ __forceinline__ float wave_incl_f(float v) {
  v += dpp0<0x111, 0xf>(v);  // row_shr:1
  v += dpp0<0x112, 0xf>(v);  // row_shr:2
  v += dpp0<0x114, 0xf>(v);  // row_shr:4
  v += dpp0<0x118, 0xf>(v);  // row_shr:8
  v += dpp0<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp0<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double lane_d(double v, int l) {  // readlane, so the compiler sees a uniform value
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// A lane's 16 steps on binade G (B = 2^G, or +0 for G = -126; h = u / 2): the sum of their increments and whether
// one of them may be a tie. A tie x^2 / u = f + 1/2 puts B + x^2 exactly halfway between two neighbours, so the
// residual x^2 - k of the increment k = fma(x, x, B) - B is exactly +-u / 2, which fma(x, x, -k) returns exactly;
// any other residual rounds to +-u / 2 only within 2^-24 of it (rare false positives, which only cost time). On
// G = -126, u / 2 = 2^-150 is not a float: there a residual of 0 from a nonzero x flags the lane instead (exact
// squares on the subnormal grid included).
template <bool SUB>
__device__ __forceinline__ float lane_incs(const float (&v)[kSL], float B, float h, unsigned long long& ties) {
  float Ka = 0.0f, Kb = 0.0f;
  unsigned long long t = 0ull;  // wave masks straight from the compares (as bools the compiler rebuilt bit vectors)
#pragma unroll
  for (int i = 0; i < kSL; i += 2) {
    const float ka = __builtin_fmaf(v[i], v[i], B) - B, kb = __builtin_fmaf(v[i + 1], v[i + 1], B) - B;
    Ka += ka;
    Kb += kb;
    const float ra = __builtin_fmaf(-v[i], v[i], ka), rb = __builtin_fmaf(-v[i + 1], v[i + 1], kb);  // k - x^2
    if constexpr (SUB) {  // h is +0 here, from an empty asm: these compares stay in this (rare) branch
      t |= __ballot(ra == 0.0f && v[i] != h) | __ballot(rb == 0.0f && v[i + 1] != h);
    } else {
      t |= __ballot(__builtin_fabsf(ra) == h) | __ballot(__builtin_fabsf(rb) == h);
    }
  }
  ties = t;
  return Ka + Kb;
}
__device__ __forceinline__ float lane_incs(const float (&v)[kSL], int G, unsigned long long& ties) {
  if (G > -126) return lane_incs<false>(v, pow2f(G), pow2fs(G - 24), ties);
  float z = 0.0f;  // through an empty asm: the loop-invariant subnormal-grid sums must not be hoisted out of the
  __asm__ volatile("" : "+v"(z));  // round loop into every segment
  return lane_incs<true>(v, z, z, ties);
}

// The lane that leaves the binade runs its steps with fma from its exact start a = acc + (the lanes before it).
__device__ __forceinline__ float lane_fma(const float (&v)[kSL], float a, int lane, int ls) {
  if (lane == ls) {
#pragma unroll
    for (int i = 0; i < kSL; ++i) a = __builtin_fmaf(v[i], v[i], a);
  }
  return lane_f(a, ls);
}

// A round by exact maps (what each lane's run adds to an even / an odd A), for a wave where a tie is possible.
// Kept out of the fast path: the steps pass an empty asm first, so the fp64 conversions are not hoisted into
// every round. Returns the new acc; `start` moves past the lane that left the binade (64: segment done).
__device__ float short_exact_round(const float (&v)[kSL], float acc, int G, int lane, int& start) {
  float w[kSL];
#pragma unroll
  for (int i = 0; i < kSL; ++i) {
    w[i] = v[i];
    __asm__ volatile("" : "+v"(w[i]));
  }
  Map m{0.0, 0.0};
#pragma unroll
  for (int h = 0; h < kSL / kLane; ++h) {  // 16 steps at a time (lane_map_exact), composed in order
    float u[kLane];
#pragma unroll
    for (int i = 0; i < kLane; ++i) u[i] = w[h * kLane + i];
    m = compose(m, lane_map_exact<false>(u, G));
  }
  if (lane < start) m = Map{0.0, 0.0};
  const double Al = apply(wave_excl(m, lane), a_of(acc));
  const double out = apply(m, Al);
  const unsigned long long ball = __ballot(lane >= start && !(out < Acc<false>::kTop));
  if (ball == 0ull) {
    start = 64;
    return rebuild<false>(lane_d(out, 63), G);
  }
  const int ls = __builtin_ctzll(ball);
  start = ls + 1;
  return lane_fma(w, rebuild<false>(lane_d(Al, ls), G), lane, ls);
}

// The same round for exact-square inputs (fp16 / bf16 values: x^2 has at most 22 significant bits), with no fp64:
// on grid G, h = x^2 / u is exact in fp32, so k = rint(h) and a tie (h - k = +-1/2) are exact, and a lane's map
// (what its steps add to an even / an odd A, sq_step) is an integer pair. The maps are scanned as fp32 pairs by
// DPP, composed in lane order: exact below 2^24, and at least 2^24 above (every term >= 0), which is all a
// covered run needs; a lane with a step of h >= 2^21 is not covered (+inf).
__device__ float short_sq_round(const float (&v)[kSL], float acc, int G, int lane, int& start) {
  float w[kSL];
#pragma unroll
  for (int i = 0; i < kSL; ++i) {  // through an empty asm: the rare path's work is not hoisted into every round
    w[i] = v[i];
    __asm__ volatile("" : "+v"(w[i]));
  }
  const int s = 23 - G;
  const float sa = pow2f(s >> 1), sb = (s & 1) ? 2.0f : 1.0f;
  int ie = 0, io = 1;
  bool big = false;
#pragma unroll
  for (int i = 0; i < kSL; ++i) {
    const float xs = w[i] * sa;
    const float h = xs * xs * sb;
    big |= !(h < 0x1p21f);  // NaN / inf too
    sq_step(big ? 0.0f : h, ie, io);
  }
  float e = big ? __builtin_inff() : (float)ie, o = big ? __builtin_inff() : (float)(io - 1);
  if (lane < start) e = o = 0.0f;
  dpp_compose<0x111, 0xf>(e, o);  // row_shr:1
  dpp_compose<0x112, 0xf>(e, o);  // row_shr:2
  dpp_compose<0x114, 0xf>(e, o);  // row_shr:4
  dpp_compose<0x118, 0xf>(e, o);  // row_shr:8
  dpp_compose<0x142, 0xa>(e, o);  // row_bcast:15
  dpp_compose<0x143, 0xc>(e, o);  // row_bcast:31
  const float A = (float)a_of(acc);
  const float out = A + (odd_f(A) ? o : e);  // A through lanes 0 .. lane
  const unsigned long long ball = __ballot(lane >= start && !(out < 0x1p24f));
  if (ball == 0ull) {
    start = 64;
    return rebuild<false>((double)lane_f(out, 63), G);
  }
  const int ls = __builtin_ctzll(ball);
  start = ls + 1;
  return lane_fma(w, rebuild<false>((double)(ls > 0 ? lane_f(out, ls - 1) : A), G), lane, ls);
}

#ifndef ADFL_TN_SERIAL_STEPS
#define ADFL_TN_SERIAL_STEPS 256
#endif
constexpr int kSerial = ADFL_TN_SERIAL_STEPS / ADFL_TN_SHORT_SL;  // lanes (256 steps) run in order at a chain's start (short_segment)

// One segment of a chain (lane l: steps 16 l .. 16 l + 15, in order) from the exact accumulator acc (wave-uniform).
// SQ: exact-square inputs (fp16 / bf16), whose tie rounds take short_sq_round instead of the fp64 maps.
template <bool SQ = false>
__device__ __forceinline__ float short_segment(const float (&v)[kSL], float acc, int lane SH_ARG) {
  int start = 0;
  SH_STAT(0, 1);
  if (acc == 0.0f) {
    // A chain's start: the accumulator doubles about every time the step count does (binade crossings at lanes 1,
    // 3, 7, 15, 31, 63), and a crossing round costs about as much as 256 dependent fma: the first kSerial lanes
    // run their steps with fma one after the other.
#pragma unroll 1
    for (int l = 0; l < kSerial; ++l) acc = lane_fma(v, acc, lane, l);
    start = kSerial;
  }
  while (start < 64) {
    SH_STAT(1, 1);
    if (!__builtin_isfinite(acc)) {  // inf stays inf unless a NaN follows; NaN stays NaN
      unsigned long long nan = 0ull;
#pragma unroll
      for (int i = 0; i < kSL; ++i) {  // through an empty asm: not hoisted into every segment
        float w = v[i];
        __asm__ volatile("" : "+v"(w));
        nan |= __ballot(__builtin_isnan(w));
      }
      if (nan >> start) acc = __builtin_nanf("");
      return acc;
    }
    const int G = grid_of(acc);
    unsigned long long ties;
    float K0 = lane_incs(v, G, ties);
    if (ties >> start) {  // a possible tie in a lane still to run
      SH_STAT(2, 1);
      if constexpr (SQ) acc = short_sq_round(v, acc, G, lane, start);
      else acc = short_exact_round(v, acc, G, lane, start);
      continue;
    }
    if (lane < start) K0 = 0.0f;
    const float top = pow2f(G + 1);  // +inf above the top binade
    const float I0 = wave_incl_f(K0), out = acc + I0;
    const unsigned long long ball = __ballot(lane >= start && !(out < top));
    if (ball == 0ull) return lane_f(out, 63);
    const int ls = __builtin_ctzll(ball);
    SH_STAT(3, 1);
    acc = lane_fma(v, acc + (ls > 0 ? lane_f(I0, ls - 1) : 0.0f), lane, ls);
    start = ls + 1;
    if (start == 64 || !__builtin_isfinite(acc) || grid_of(acc) != G + 1) continue;
    // on from lane ls + 1 on G + 1, where acc went (the usual crossing): one more scan, no new round
    unsigned long long ties1;
    const float K1 = lane_incs<false>(v, top, pow2fs(G - 23), ties1);
    if (ties1 >> start) continue;  // start = ls + 1 < 64
    const float I1 = wave_incl_f(lane > ls ? K1 : 0.0f), out1 = acc + I1;
    const unsigned long long b1 = __ballot(lane > ls && !(out1 < pow2f(G + 2)));
    if (b1 == 0ull) {
      SH_STAT(4, 1);
      return lane_f(out1, 63);
    }
    const int l1 = __builtin_ctzll(b1);
    SH_STAT(3, 1);
    acc = lane_fma(v, acc + lane_f(I1, l1 - 1), lane, l1);
    start = l1 + 1;
  }
  return acc;
}

// ---- phase D
// A segment (<= 1024 steps, lane l holding steps 16 l .. 16 l + 15) run from the exact accumulator acc
// (fp64 accumulators; fp32 / bf16 / fp16 ones take short_segment, resolve_tile).
// fp32 accumulators, no tie possible in the wave: each lane's steps add a constant on the binade G and one
// on G + 1 — both summed in one pass and scanned together, so the usual segment (one crossing) costs one
// round: the first lane that leaves G runs its steps with fma, and the lanes after it are checked on G + 1
// from the sums' differences. Otherwise (ties, two crossings, non-finite values) maps, lane by lane.
template <int DT>
__device__ __forceinline__ typename Acc<Dt<DT>::kWide>::T resolve_segment(const typename Dt<DT>::E (&v)[kLane],
                                                                           typename Acc<Dt<DT>::kWide>::T acc, int lane) {
  constexpr bool W = Dt<DT>::kWide;
  using A_t = typename Acc<W>::T;
  int start = 0;
  for (;;) {
    if (!__builtin_isfinite(acc)) {  // inf stays inf unless a NaN follows; NaN stays NaN
      bool nan = false;
#pragma unroll
      for (int i = 0; i < kLane; ++i) nan |= __builtin_isnan(v[i]);
      if (__ballot(nan && lane >= start)) acc = (A_t)__builtin_nan("");
      return acc;
    }
    TN_STAT(2, 1);
    const int G = grid_of(acc);
    const double A = a_of(acc);
    if constexpr (!W && Dt<DT>::kSq) {  // exact-square inputs: the lane maps on G and G + 1 in one pass
      Map m0, m1;
      lane_maps_pair<W, true>(v, G, +1, m0, m1);
      if (lane < start) m0 = Map{0.0, 0.0};
      const double Al = apply(wave_excl(m0, lane), A);
      const double out = apply(m0, Al);
      const unsigned long long ball = __ballot(lane >= start && !(out < Acc<W>::kTop));
      if (ball == 0ull) return rebuild<W>(__shfl(out, 63, 64), G);
      const int ls = __builtin_ctzll(ball);
      A_t a = rebuild<W>(__shfl(Al, ls, 64), G);
      if (lane == ls) {
#pragma unroll
        for (int i = 0; i < kLane; ++i) a = fma_t(v[i], v[i], a);
      }
      acc = __shfl(a, ls, 64);
      start = ls + 1;
      if (start == 64) return acc;
      if (__builtin_isfinite(acc) && grid_of(acc) == G + 1) {  // on from lane ls + 1 with the maps on G + 1
        const Map n1 = lane > ls ? m1 : Map{0.0, 0.0};
        const double Al1 = apply(wave_excl(n1, lane), a_of(acc));
        const double out1 = apply(n1, Al1);
        if (__ballot(lane > ls && !(out1 < Acc<W>::kTop)) == 0ull) return rebuild<W>(__shfl(out1, 63, 64), G + 1);
      }
      continue;
    }
    if constexpr (!W) {
      const double sc = pow2(23 - G);
      double K0 = 0.0, K1 = 0.0;
      bool maybe = false;
#pragma unroll
      for (int i = 0; i < kLane; ++i) {
        const double d = (double)v[i];
        const double x2 = d * (d * sc), h = x2 * 0.5, w = x2 * 2.0;
        K0 += (x2 + kMagic) - kMagic;
        K1 += (h + kMagic) - kMagic;
        maybe |= ((w + kMagic) - kMagic) == w && w != 0.0;  // 2v an integer: a tie is possible (on G or G + 1)
      }
      if (__ballot(maybe) == 0ull) {
        if (lane < start) K0 = K1 = 0.0;
        double I0 = K0, I1 = K1;  // inclusive scans
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const double p0 = __shfl_up(I0, o, 64), p1 = __shfl_up(I1, o, 64);
          if (lane >= o) {
            I0 += p0;
            I1 += p1;
          }
        }
        const double out = A + I0, Al = out - K0;
        const unsigned long long ball = __ballot(lane >= start && !(out < Acc<W>::kTop));
        if (ball == 0ull) return rebuild<W>(__shfl(out, 63, 64), G);
        const int ls = __builtin_ctzll(ball);
        A_t a = rebuild<W>(__shfl(Al, ls, 64), G);
        if (lane == ls) {
#pragma unroll
          for (int i = 0; i < kLane; ++i) a = fma_t(v[i], v[i], a);
        }
        acc = __shfl(a, ls, 64);
        start = ls + 1;
        if (start == 64) return acc;
        // on from lane ls + 1 on G + 1: the K1 sums of lanes ls + 1 .. (exact while the total is below 2^53)
        if (__builtin_isfinite(acc) && grid_of(acc) == G + 1 && G + 1 <= Acc<W>::kGmax &&
            __shfl(I1, 63, 64) < 0x1p52) {
          const double out1 = a_of(acc) + (I1 - __shfl(I1, ls, 64));
          if (__ballot(lane > ls && !(out1 < Acc<W>::kTop)) == 0ull) return rebuild<W>(__shfl(out1, 63, 64), G + 1);
        }
        continue;
      }
    }
    TN_STAT(8, 1);
    Map m = lane_map_exact<W>(v, G);
    if (lane < start) m = Map{0.0, 0.0};
    const Map ex = wave_excl(m, lane);
    const double Al = apply(ex, A);
    const double out = apply(m, Al);
    const bool bad = lane >= start && !(out < Acc<W>::kTop);
    const unsigned long long ball = __ballot(bad);
    if (ball == 0ull) return rebuild<W>(__shfl(out, 63, 64), G);
    const int ls = __builtin_ctzll(ball);
    const double As = __shfl(Al, ls, 64);
    A_t a = rebuild<W>(As, G);
    if (lane == ls) {
#pragma unroll
      for (int i = 0; i < kLane; ++i) a = fma_t(v[i], v[i], a);
    }
    acc = __shfl(a, ls, 64);
    start = ls + 1;
    if (start == 64) return acc;
  }
}

template <int DT>
__device__ __forceinline__ void load_seg(const void* x, const Tensor& T, int c, Split sp, int64_t s0, int64_t s1,
                                         int lane, typename Dt<DT>::E (&v)[kLane]) {
#pragma unroll
  for (int i = 0; i < kLane; ++i) {
    const int64_t s = s0 + lane * kLane + i;
    const typename Dt<DT>::E e = Dt<DT>::ld(x, elem_of<DT>(T, c, sp, s < s1 ? s : s1 - 1));  // clamped
    v[i] = s < s1 ? e : (typename Dt<DT>::E)0;
  }
}

template <int DT>
__device__ typename Acc<Dt<DT>::kWide>::T resolve_tile(const void* x, const Tensor& T, int c, Split sp, const Tile& tl,
                                                       typename Acc<Dt<DT>::kWide>::T acc, int lane) {
  typename Dt<DT>::E v[kLane];
  TN_STAT(1, 1);
#ifdef ADFL_TN_STATS
  const long long c0 = clock64();
#endif
  for (int64_t s0 = tl.s0; s0 < tl.s1; s0 += kSeg) {
    load_seg<DT>(x, T, c, sp, s0, s0 + kSeg < tl.s1 ? s0 + kSeg : tl.s1, lane, v);
#ifdef ADFL_TN_STATS
    {
      const long long l0 = clock64();
      float z = 0.0f;
#pragma unroll
      for (int i = 0; i < kLane; ++i) z += (float)v[i];
      __asm__ volatile("" ::"v"(z));
      TN_STAT(5, clock64() - l0);
    }
#endif
#ifdef ADFL_TN_STATS
    const long long r0 = clock64();
#endif
    if constexpr (!Dt<DT>::kWide && kSL == kLane) {  // k_tn_short's fp32 rounds (no fp64, DPP scans), same answer;
                                                      // bf16 / fp16 (exact squares) with their fp32 tie rounds
#ifdef ADFL_TN_STATS
      unsigned long long shs[11] = {};
#endif
      acc = short_segment<Dt<DT>::kSq>(v, acc, lane SH_PASS);
    } else {
      acc = resolve_segment<DT>(v, acc, lane);
    }
#ifdef ADFL_TN_STATS
    TN_STAT(9, clock64() - r0);
#endif
  }
#ifdef ADFL_TN_STATS
  TN_STAT(4, clock64() - c0);
#endif
  return acc;
}

// One window (kWinTiles tiles of chain c from tile w0; lane l holds tiles l * kTPL ..) from the exact acc:
// scan the tiles' maps on acc's binade; the first tile not covered (a crossing, a miss of the predictor, a
// large step) is resolved in detail; and on from the tile after it.
template <int DT>
__device__ typename Acc<Dt<DT>::kWide>::T resolve_window(const void* x, const Tensor& T, int c, Split sp,
                                                         const double* S, const Rec* recs, const double4* maps,
                                                         int64_t w0, int64_t nt, typename Acc<Dt<DT>::kWide>::T acc,
                                                         int lane) {
  constexpr bool W = Dt<DT>::kWide;
  using A_t = typename Acc<W>::T;
  Rec r[kTPL];
  double4 mp[kTPL];  // the side maps (read for every tile, so the loads are all in flight; used where kSide)
#pragma unroll
  for (int k = 0; k < kTPL; ++k) {
    const int64_t t = w0 + lane * kTPL + k;
    const int64_t slot = tile_of<DT>(T, c, sp, t < nt ? t : nt - 1).slot;  // clamped: loads in flight
    const Rec q = recs[slot];
    mp[k] = maps[slot];
    r[k] = t < nt ? q : Rec{kPad << 24, 0u};
  }
#ifdef ADFL_TN_STATS
  {
    const long long l0 = clock64();
    uint32_t z = 0;
#pragma unroll
    for (int k = 0; k < kTPL; ++k) z ^= r[k].w0 ^ r[k].w1 ^ (uint32_t)__double_as_longlong(mp[k].x);
    __asm__ volatile("" ::"v"(z));
    TN_STAT(10, clock64() - l0);
  }
#endif
  // the records decoded once per window (every scan re-selects from them by the accumulator's binade): flags,
  // predicted binade, and (fp32) the totals on g and g - 1 as fp32 integers (+inf where not covered)
  uint32_t flk[kTPL];
  int gk[kTPL];
  float K0f[kTPL], K1f[kTPL];
#pragma unroll
  for (int k = 0; k < kTPL; ++k) {
    flk[k] = rec_flags(r[k]);
    gk[k] = rec_g<W>(r[k]);
    if constexpr (!W) {
      K0f[k] = (float)rec_k(r[k], 0);
      K1f[k] = (float)rec_k(r[k], 1);
    }
  }
  int start = 0;  // window tiles before it are done
  const int wlen = nt - w0 < kWinTiles ? (int)(nt - w0) : kWinTiles;
  while (start < wlen) {
    TN_STAT(7, 1);
#ifdef ADFL_TN_STATS
    const long long sc0 = clock64();
#endif
    if (!__builtin_isfinite(acc)) {  // inf stays inf unless a NaN follows: the remaining tiles' sums say
      bool nan = false;
      for (int64_t u = w0 + start + lane; u < nt; u += 64) {
        const int64_t sl = tile_of<DT>(T, c, sp, u).slot;
        nan |= __builtin_isnan(S[sl]) || (rec_flags(recs[sl]) & kNaN);
      }
      if (__ballot(nan)) acc = (A_t)__builtin_nan("");
      return acc;
    }
    const int G = grid_of(acc);
    const double A = a_of(acc);
    bool side = false;
#pragma unroll
    for (int k = 0; k < kTPL; ++k) side |= (flk[k] & kSide) && lane * kTPL + k >= start;
    const bool any_side = __ballot(side) != 0ull;
    const auto tile_map = [&](int k) -> Map {
      const Rec q = r[k];
      const uint32_t fl = rec_flags(q);
      if ((fl & kPad) || lane * kTPL + k < start) return Map{0.0, 0.0};
      const int j = rec_g<W>(q) - G;
      if (j != 0 && j != 1) return Map{__builtin_inf(), __builtin_inf()};
      if (fl & kSide) return j == 0 ? Map{mp[k].x, mp[k].y} : Map{mp[k].z, mp[k].w};
      const double K = rec_k(q, j);
      return Map{K, K};
    };
    if constexpr (!W) {
      if (!any_side) {  // fp32 accumulators: the DPP scan in fp32, as in resolve_chain
        float Kk[kTPL], K = 0.0f;
#pragma unroll
        for (int k = 0; k < kTPL; ++k) {  // tile_map(k).e from the window's decoded records
          const int j = gk[k] - G;
          Kk[k] = ((flk[k] & kPad) || lane * kTPL + k < start) ? 0.0f
                                                                : (j == 0 ? K0f[k] : (j == 1 ? K1f[k] : __builtin_inff()));
          K += Kk[k];
        }
        const float Af = (float)A, I = wave_incl_f(K), o = Af + I;
        const unsigned long long ball = __ballot(!(o < 0x1p24f));
        if (ball == 0ull) return rebuild<W>((double)lane_f(o, 63), G);
        const int ls = __builtin_ctzll(ball);
        float Ab = ls > 0 ? Af + lane_f(I, ls - 1) : Af;  // lane ls's start, exact (wave-uniform)
        int kb = kTPL;
#pragma unroll
        for (int k = 0; k < kTPL; ++k) {
          if (kb == kTPL) {
            const float nxt = Ab + Kk[k];
            if (!(nxt < 0x1p24f)) kb = k;
            else Ab = nxt;
          }
        }
        const int tb = ls * kTPL + __builtin_amdgcn_readlane(kb, ls);
        acc = rebuild<W>((double)lane_f(Ab, ls), G);
        TN_STAT(11, clock64() - sc0);
        acc = resolve_tile<DT>(x, T, c, sp, tile_of<DT>(T, c, sp, w0 + tb), acc, lane);
        start = tb + 1;
        continue;
      }
    }
    double Al, out;
    if (!any_side) {
      double K = 0.0;
#pragma unroll
      for (int k = 0; k < kTPL; ++k) K += tile_map(k).e;
      Al = A + wave_excl_sum(K, lane);
      out = Al + K;
    } else {
      Map m{0.0, 0.0};
#pragma unroll
      for (int k = 0; k < kTPL; ++k) m = compose(m, tile_map(k));
      Al = apply(wave_excl(m, lane), A);
      out = apply(m, Al);
    }
    const unsigned long long ball = __ballot(!(out < Acc<W>::kTop));
    if (ball == 0ull) return rebuild<W>(__shfl(out, 63, 64), G);
    // the first tile not covered: each lane's first tile whose map leaves the binade from its Al
    int kb = kTPL;
    double Ab = Al;
#pragma unroll
    for (int k = 0; k < kTPL; ++k) {
      if (kb == kTPL) {
        const double nxt = apply(tile_map(k), Ab);
        if (!(nxt < Acc<W>::kTop)) kb = k;
        else Ab = nxt;
      }
    }
    const int ls = __builtin_ctzll(ball);
    const int tb = ls * kTPL + __shfl(kb, ls, 64);
    acc = rebuild<W>(__shfl(Ab, ls, 64), G);
    TN_STAT(11, clock64() - sc0);
    acc = resolve_tile<DT>(x, T, c, sp, tile_of<DT>(T, c, sp, w0 + tb), acc, lane);
    start = tb + 1;
  }
  return acc;
}

template <int DT>
__device__ typename Acc<Dt<DT>::kWide>::T resolve_chain(const void* x, const Tensor& T, int c, Split sp,
                                                        const double* S, const Rec* recs, const double4* maps,
                                                        const int* wing, const double4* winmaps, bool use_recs,
                                                        int lane) {
  constexpr bool W = Dt<DT>::kWide;
  using A_t = typename Acc<W>::T;
  const int64_t nt = chain_tiles<DT>(T, c, sp);
  A_t acc = (A_t)0;
  if (!use_recs) {
    for (int64_t t = 0; t < nt; ++t) acc = resolve_tile<DT>(x, T, c, sp, tile_of<DT>(T, c, sp, t), acc, lane);
    return acc;
  }
  // Windows 64 at a time (lane l: window wb + l), each as its summary map on acc's binade (phase C2); the
  // first window not covered is resolved tile by tile (resolve_window), then on from the window after it.
  const int64_t nw = (nt + kWinTiles - 1) / kWinTiles;
  for (int64_t wb = 0; wb < nw; wb += 64) {
    const int64_t w = wb + lane;
    const bool valid = w < nw;
    const int64_t wslot = tile_of<DT>(T, c, sp, (valid ? w : nw - 1) * kWinTiles).slot;  // clamped
    const int gw = wing[wslot];
    const double4 wm = winmaps[wslot];
    int wstart = 0;
    const int wlen = nw - wb < 64 ? (int)(nw - wb) : 64;
    while (wstart < wlen) {
      if (!__builtin_isfinite(acc)) {  // inf stays inf unless a NaN follows: the remaining tiles' sums say
        bool nan = false;
        for (int64_t u = (wb + wstart) * kWinTiles + lane; u < nt; u += 64)
          nan |= __builtin_isnan(S[tile_of<DT>(T, c, sp, u).slot]) || (rec_flags(recs[tile_of<DT>(T, c, sp, u).slot]) & kNaN);
        if (__ballot(nan)) acc = (A_t)__builtin_nan("");
        return acc;
      }
      const int G = grid_of(acc);
      const double A = a_of(acc);
      Map m{0.0, 0.0};
      if (valid && lane >= wstart) {
        const int j = gw - G;
        m = j == 0 ? Map{wm.x, wm.y} : (j == 1 ? Map{wm.z, wm.w} : Map{__builtin_inf(), __builtin_inf()});
      }
      const bool sums = __ballot(m.e != m.o) == 0ull;
      unsigned long long ball;
      int ls;
      if (!W && sums) {
        // fp32 accumulators: integer totals, exact in fp32 below 2^24 and at least 2^24 above (terms >= 0, RN
        // monotone — k_tn_short's argument), so the scan is k_tn_short's DPP one: no fp64, no shuffles
        const float Af = (float)A, I = wave_incl_f((float)m.e), o = Af + I;
        ball = __ballot(!(o < 0x1p24f));
        if (ball == 0ull) {
          acc = rebuild<W>((double)lane_f(o, 63), G);
          break;
        }
        ls = __builtin_ctzll(ball);
        acc = rebuild<W>((double)(ls > 0 ? Af + lane_f(I, ls - 1) : Af), G);
      } else {
        double Al, out;
        if (sums) {
          Al = A + wave_excl_sum(m.e, lane);
          out = Al + m.e;
        } else {
          Al = apply(wave_excl(m, lane), A);
          out = apply(m, Al);
        }
        ball = __ballot(!(out < Acc<W>::kTop));
        if (ball == 0ull) {
          acc = rebuild<W>(__shfl(out, 63, 64), G);
          break;
        }
        ls = __builtin_ctzll(ball);
        acc = rebuild<W>(__shfl(Al, ls, 64), G);
      }
      TN_STAT(0, 1);
#ifdef ADFL_TN_STATS
      const long long w0c = clock64();
#endif
      acc = resolve_window<DT>(x, T, c, sp, S, recs, maps, (wb + ls) * kWinTiles, nt, acc, lane);
#ifdef ADFL_TN_STATS
      TN_STAT(6, clock64() - w0c);
#endif
      wstart = ls + 1;
    }
  }
  return acc;
}

// Every tensor's first chunk, tfirst[tensor] (the short kernel's work list: one block per tensor, so its blocks
// spread over the XCDs, where one block per chunk put every working block of an equal layout with an even chunk
// count per tensor on the same XCDs).
__global__ __launch_bounds__(256) void k_tn_tfirst(const adfl_slq_chunk* __restrict__ chunks, int64_t nchunks,
                                                   int* __restrict__ tfirst) {
  const int64_t ci = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ci >= nchunks) return;
  const adfl_slq_chunk ch = chunks[ci];
  if (ch.first_chunk == ci) tfirst[ch.tensor] = (int)ci;
}

// One block per tensor (blockIdx.x = tensor, its first chunk from tfirst) of at most max_n elements (longer
// ones return). The 8 waves stream the tensor in 8192-element segments: every thread loads 16 consecutive-lane
// dwords per segment (buffer loads whose range ends at the chain steps' end, so the rest reads as +0, which no
// chain notices), two segments ahead in registers, and stages them chain-major into LDS; wave c then reads its
// lanes' 16-step runs of chain c (4 ds_read_b128 each) and advances the chain by short_segment. Then the lane
// sum left to right, the n % 8 tail and the sqrt, as k_norm_walk does.
__global__ __launch_bounds__(kShThreads) void k_tn_short(const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks,
                                                         const int* __restrict__ tfirst, int64_t max_n,
                                                         double* __restrict__ norms64, float* __restrict__ norms32) {
  __shared__ __attribute__((aligned(16))) float buf[2 * 8 * kShRow + 4];  // + the spare slot (off[] < 0 elements)
  __shared__ float s_acc[8];
#ifdef ADFL_TN_STATS
  unsigned long long shs[11] = {};
  __shared__ long long s_tl[8][48][2];
  int shn = 0;
#endif
  const int ci = tfirst[blockIdx.x];
  const adfl_slq_chunk ch = chunks[ci];
  const int64_t n = (int64_t)(ch.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + ch.nchunks - 1].len;
  if (n > max_n) return;
  const float* xt = x + ch.start;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (n < 8) {
    if (tid == 0) {
      const float b = tail32(xt, 0, n, 0.0f);
      const float r = n == 1 ? __builtin_fabsf(xt[0]) : (float)__builtin_sqrt((double)b);  // one element: |x|
      if (norms32) norms32[ch.tensor] = r;
      if (norms64) norms64[ch.tensor] = r;
    }
    return;
  }
  const int64_t nv = n - n % 8;
  const int nseg = (int)((nv + kShSeg - 1) / kShSeg);
  // 16-byte loads from the aligned block below the tensor's start: "aligned block" j is the 2048 vectors from
  // vector 2048 j there (elements 8192 j - delta .. 8192 j + 8191 - delta of the tensor; delta = its start's
  // offset in a vector, 0..3), plus vector 2048 (j + 1), whose first delta elements end segment j (every thread
  // loads it, so every wave counts the same loads; thread 0 stages it). Segment j = elements 8192 j ..
  // 8192 j + 8191 is thus staged from block j alone. Vectors holding an element of the tensor lie inside its
  // allocation, so the buffer range ends at the last such vector; elements past the chain steps' end are zeroed.
  const int delta = (int)(((uintptr_t)xt & 15) >> 2);
  const float* const xa = xt - delta;
  const int64_t vbytes = ((nv + delta) * 4 + 15) & ~(int64_t)15;
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef float f3v __attribute__((ext_vector_type(3)));
  struct Blk {
    f4v r[kShVec];
    f3v t;  // 3 dwords: a dead 4th component's register was reused at once, which waited for the load (WAW)
  };
  // part 0: every vector and the extra one; part 1 / 2: the first half / the rest
  const auto load_part = [&](Blk& k, int j, int part) {
    const int64_t base = (int64_t)j * (kShSeg * 4), left = vbytes - base;
    const int bytes = left <= 0 ? 0 : (int)min(left, (int64_t)kShSeg * 4 + 16);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xa) + (left <= 0 ? 0 : (int64_t)j * kShSeg), 0,
                                                      bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < kShVec; ++i)
      if (part == 0 || (part == 1) == (i < kShVec / 2))
        k.r[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (i * kShThreads + tid) * 16, 0, 0));
    if (part != 1) k.t = __builtin_bit_cast(f3v, __builtin_amdgcn_raw_buffer_load_b96(rs, kShSeg * 4, 0, 0));
  };
  const auto load = [&](Blk& k, int j) { load_part(k, j, 0); };
  // Thread tid's element p of vector i is e = kShSeg j + 2048 i + 4 tid + p - delta: chain e % 8, step e / 8 of
  // the segment (lane step / kSL, slot step % kSL); i adds 256 steps (256 / kSL lanes). Thread 0's first delta elements of
  // vector 0 belong to segment j - 1 (staged from its own extra vector): they go to a spare slot past the rows.
  constexpr int kBufF = 8 * kShRow;
  int off[4], off0[4];  // vector i > 0: off + 16 lanes per i; vector 0: off0 (the spare slot for e < 0)
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int e = 4 * tid + p - delta;  // e < 0 (thread 0): chain e & 7 at "lane -1, last slot", so that vector i > 0
    const int st = e >> 3;              // lands on step 256 i - 1
    off[p] = (e & 7) * kShRow + (st >= 0 ? st / kSL : -1) * kShLS + (st >= 0 ? st % kSL : kSL - 1);
    off0[p] = e < 0 ? 2 * kBufF + p : off[p];
  }
  const int nvi = (int)nv;
  const auto stage = [&](const Blk& k, int j) {
    SH_TL(1);
#ifdef ADFL_TN_STATS
    const long long c0 = clock64();
#endif
    float* const bj = buf + (j & 1) * kBufF;
    const int e0 = j * kShSeg - delta + 4 * tid;                    // this thread's element of vector 0
    const bool last = j * kShSeg - delta + kShSeg + 4 > nvi;         // the block holds the steps' end
    const auto put = [&](const f4v (&r)[kShVec]) {
#pragma unroll
      for (int p = 0; p < 4; ++p) (off0[p] < 2 * kBufF ? bj : buf)[off0[p]] = r[0][p];
#pragma unroll
      for (int i = 1; i < kShVec; ++i)
#pragma unroll
        for (int p = 0; p < 4; ++p) bj[off[p] + (256 / kSL) * kShLS * i] = r[i][p];
    };
    if (!last) {
      put(k.r);
    } else {  // the block holding the steps' end: zeros past it
      f4v z[kShVec];
#pragma unroll
      for (int i = 0; i < kShVec; ++i)
#pragma unroll
        for (int p = 0; p < 4; ++p) z[i][p] = e0 + 2048 * i + p < nvi ? k.r[i][p] : 0.0f;
      put(z);
    }
    if (tid == 0) {  // the extra vector's first delta elements: chains 8 - delta + p of the segment's last step
#pragma unroll
      for (int p = 0; p < 3; ++p)
        if (p < delta) {
          const float val = (j + 1) * kShSeg - delta + p < nvi ? k.t[p] : 0.0f;
          bj[(8 - delta + p) * kShRow + 63 * kShLS + kSL - 1] = val;
        }
    }
#ifdef ADFL_TN_STATS
    SH_STAT(9, clock64() - c0);
#endif
    SH_TL(2);
  };
  const auto sync = [&]() {
#ifdef ADFL_TN_STATS
    const long long c0 = clock64();
#endif
    __syncthreads();
#ifdef ADFL_TN_STATS
    SH_STAT(10, clock64() - c0);
#endif
    SH_TL(6);
  };
  const int rdo = wave * kShRow + lane * kShLS;
  float acc = 0.0f;
  const auto run = [&](int j) {
    SH_TL(3);
    const float4* const rd = reinterpret_cast<const float4*>(buf + (j & 1) * kBufF + rdo);
    float v[kSL];
#pragma unroll
    for (int q = 0; q < kSL / 4; ++q) {
      const float4 f = rd[q];
      v[4 * q] = f.x;
      v[4 * q + 1] = f.y;
      v[4 * q + 2] = f.z;
      v[4 * q + 3] = f.w;
    }
#ifdef ADFL_TN_STATS
    __asm__ volatile("" ::"v"(v[0]), "v"(v[15]));  // the LDS reads have landed
    SH_TL(4);
    const long long r0 = clock64();
#endif
    acc = short_segment(v, acc, lane SH_PASS);
#ifdef ADFL_TN_STATS
    SH_STAT(5, clock64() - r0);
    SH_TL(5);
#endif
  };
#ifdef ADFL_TN_STATS
  const long long k0 = clock64();
  SH_STAT(8, 1);
#endif
  // Two LDS buffers (segment j in buffer j % 2), two register sets: segment j is walked in one buffer, then
  // segment j + 1 staged into the other, while block j + 2 loads; one barrier per segment. Each set is staged in
  // the half after the one that loaded it, after the other set's loads were issued, so the wait before a stage
  // covers its own loads only (vmcnt(5)). (Staged at the loop head, or before the other set's loads, the
  // compiler's merged state at the loop header waited for both sets, and the loads' latency was exposed.)
  Blk ra, rb;
  SH_TL(0);
  load(ra, 0);
  // every wave's segment-0 loads queue before any segment-1 load (a bare s_barrier: no wait for the loads),
  // so the last wave's first data is not behind the other waves' second segment in the CU's load queue
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  load(rb, 1);
  stage(ra, 0);
  sync();
  // Each segment's loads in two halves: the first before the walk, the rest after the stage, so the CU's load
  // queue holds at most half a segment more while a wave issues (a whole segment before the walk stalled the
  // issue 0.5-1.4k cycles: queue full; all of it after the stage exposed the latency on long walks). Measured:
  // kernel 17.3 -> 16.6 us on C3 equal, C3 log-uniform call 50.2 -> 49.2 us (profiles/r06/norm/split_load_ab/).
  for (int j = 0;; j += 2) {  // block-uniform control flow throughout
    load_part(ra, j + 2, 1);
    run(j);
    stage(rb, j + 1);  // after the walk: its loads have had the walk's time to land (past the end: zeros)
    load_part(ra, j + 2, 2);
    sync();
    if (j + 1 >= nseg) break;
    load_part(rb, j + 3, 1);
    run(j + 1);
    stage(ra, j + 2);
    load_part(rb, j + 3, 2);
    sync();
    if (j + 2 >= nseg) break;
  }
#ifdef ADFL_TN_STATS
  SH_STAT(6, clock64() - k0);
  if (lane == 0)
    for (int i = 0; i < 11; ++i) atomicAdd(&g_sh_stats[i], shs[i]);
  if (blockIdx.x == 7 && lane == 0) {
    for (int k = 0; k < min(shn, 48); ++k) {
      g_sh_tl[wave][k][0] = s_tl[wave][k][0];
      g_sh_tl[wave][k][1] = s_tl[wave][k][1];
    }
    g_sh_tln[wave] = min(shn, 48);
  }
#endif
  if (lane == 0) s_acc[wave] = acc;
  __syncthreads();
  if (tid == 0) {  // lane sum left to right, the n % 8 tail, sqrt
    float b = s_acc[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) b = b + s_acc[j];
    b = tail32(xt, nv, n, b);
    const float r = (float)__builtin_sqrt((double)b);  // correctly rounded fp32 sqrt
    if (norms32) norms32[ch.tensor] = r;
    if (norms64) norms64[ch.tensor] = r;
  }
}

// ---- short fp16 tensors (up to kShortMax elements): one block per tensor, one wave per piece, one launch.
// torch's fp16 order is at::parallel_for's split (split_of): nt = 1 or 2 pieces here (n <= 2^16), each one fp32
// chain over its contiguous elements from 0, the piece sums added in order to 0. x^2 of an fp16 value is exact
// in fp32, so a piece is k_tn_short's chain with contiguous steps: wave c walks piece c in 1024-step segments
// (lane l: steps 16 l .. 16 l + 15) by short_segment. A piece's elements are contiguous, so each wave stages its
// own segment — 16-byte loads of the aligned block under it, converted to fp32 into the wave's own LDS rows —
// and needs no block barrier; the next three segments' loads are in flight while one is walked.
constexpr int kH16Waves = 2;                    // pieces per tensor at n <= kShortMax = 2^16 (GRAIN 32768)
constexpr int kH16Row = 64 * kShLS;             // floats per wave's staged segment (lane rows of 16 + 4)
static_assert(kShortMax <= 2 * kGrain, "k_tn_short_f16 holds two pieces per tensor");

__global__ __launch_bounds__(64 * kH16Waves) void k_tn_short_f16(const uint16_t* __restrict__ x,
                                                                  const adfl_slq_chunk* __restrict__ chunks,
                                                                  const int* __restrict__ tfirst, int64_t max_n, int threads,
                                                                  double* __restrict__ norms64, float* __restrict__ norms32) {
  __shared__ __attribute__((aligned(16))) float buf[kH16Waves][kH16Row];
  __shared__ float s_acc[kH16Waves];
  const int ci = tfirst[blockIdx.x];
  const adfl_slq_chunk ch = chunks[ci];
  const int64_t n = (int64_t)(ch.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + ch.nchunks - 1].len;
  if (n > max_n) return;
  const uint16_t* const xt = x + ch.start;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Split sp = split_of(n, threads);
  float acc = 0.0f;
  if (wave < (int)sp.nt) {
    const int64_t a = (int64_t)wave * sp.cs, L = (a + sp.cs < n ? a + sp.cs : n) - a;  // the piece's steps
    // one buffer resource over the tensor's 16-byte blocks (reads past them return 0)
    const int dt = (int)(((uintptr_t)xt & 15) >> 1);                // the tensor's start in its block, in halves
    const uint16_t* const xa = xt - dt;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(xa), 0, (int)(((n + dt) * 2 + 15) & ~15LL),
                                                      0x00020000);
    const int nseg = (int)((L + kSeg - 1) / kSeg);
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    struct Blk {
      u4 r0, r1, r2;  // vectors lane and lane + 64 of the segment's block, and vector 128 (lane 0's)
      int delta;
    };
    const auto load = [&](Blk& k, int j) {
      const int64_t e = dt + a + (int64_t)j * kSeg;                 // the segment's first element, from xa
      const int64_t vb = e >> 3;                                    // its 16-byte block
      k.delta = (int)(e & 7);
      const int o = (int)(vb * 16);
      k.r0 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + lane * 16, 0, 0));
      k.r1 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + (lane + 64) * 16, 0, 0));
      k.r2 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 128 * 16, 0, 0));
    };
    float* const row = buf[wave];
#ifdef ADFL_TN_STATS
    unsigned long long shs[11] = {};
#endif
    const auto stage_run = [&](const Blk& k, int j) {
      const int left = (int)(L - (int64_t)j * kSeg < kSeg ? L - (int64_t)j * kSeg : kSeg);  // steps in this segment
      const auto put = [&](const u4& r, int v) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int st = 8 * v + q - k.delta;
          if (st >= 0 && st < kSeg) {
            const uint32_t w = r[q >> 1];
            const float f = __half2float(__ushort_as_half((unsigned short)((q & 1) ? (w >> 16) : (w & 0xffffu))));
            row[(st >> 4) * kShLS + (st & 15)] = st < left ? f : 0.0f;
          }
        }
      };
      put(k.r0, lane);
      put(k.r1, lane + 64);
      if (lane == 0) put(k.r2, 128);
      const float4* const rd = reinterpret_cast<const float4*>(row + lane * kShLS);
      float v[kSL];
#pragma unroll
      for (int q = 0; q < kSL / 4; ++q) {
        const float4 f = rd[q];
        v[4 * q] = f.x;
        v[4 * q + 1] = f.y;
        v[4 * q + 2] = f.z;
        v[4 * q + 3] = f.w;
      }
      acc = short_segment<true>(v, acc, lane SH_PASS);
    };
#ifdef ADFL_TN_STATS
    const long long k0c = clock64();
#endif
    // wave-uniform: four register sets, the next three segments' loads in flight while one is walked (one
    // segment ahead left the HBM latency exposed: two waves per CU have nothing else to hide it behind)
    // (loads past the tensor read zeros from the buffer resource, so they are issued unconditionally: a guarded
    // load made the compiler wait for every load at the merge)
    Blk k0, k1, k2, k3;
    load(k0, 0);
    load(k1, 1);
    load(k2, 2);
    for (int j = 0;; j += 4) {
      load(k3, j + 3);
      stage_run(k0, j);
      if (j + 1 >= nseg) break;
      load(k0, j + 4);
      stage_run(k1, j + 1);
      if (j + 2 >= nseg) break;
      load(k1, j + 5);
      stage_run(k2, j + 2);
      if (j + 3 >= nseg) break;
      load(k2, j + 6);
      stage_run(k3, j + 3);
      if (j + 4 >= nseg) break;
    }
#ifdef ADFL_TN_STATS
    shs[6] += clock64() - k0c;
    shs[8] += 1;
    if (lane == 0)
      for (int i = 0; i < 11; ++i) atomicAdd(&g_sh_stats[i], shs[i]);
#endif
  }
  if (lane == 0) s_acc[wave] = acc;
  __syncthreads();
  if (tid == 0) {
    float tot = 0.0f;
    for (int c = 0; c < (int)sp.nt; ++c) tot = tot + s_acc[c];
    float r = __half2float(__float2half_rn((float)__builtin_sqrt((double)tot)));
    if (n == 1) r = __builtin_fabsf(__half2float(__ushort_as_half(xt[0])));  // a one-element tensor's norm is |x|
    if (norms32) norms32[ch.tensor] = r;
    if (norms64) norms64[ch.tensor] = r;
  }
}

__device__ __forceinline__ float rn_bf16(float f) {
  const uint32_t b = __float_as_uint(f);
  if (__builtin_isnan(f)) return __uint_as_float((b | 0x00400000u) & 0xffff0000u);
  return __uint_as_float((b + 0x7fffu + ((b >> 16) & 1u)) & 0xffff0000u);
}

// ---- short bf16 tensors (up to kShortMaxF32 elements): k_tn_short's layout for 2-byte elements. torch's bf16
// order is 8 fp32 chains over the leading n - n % 16 elements (element e into chain e % 8), the lane sum left to
// right, then the n % 16 tail with fma; x^2 of a bf16 value is exact in fp32 (tie rounds: short_sq_round). The
// 8 waves stream the tensor in 8192-element segments (16 KB): each thread loads 2 16-byte vectors of the aligned
// block (thread 0's third covers the start's offset), converts them to fp32 into the chains' LDS rows, and wave c
// walks chain c's 1024 steps by short_segment; two LDS buffers, one barrier per segment, the next segment's
// loads in flight while one is walked.
__global__ __launch_bounds__(kShThreads) void k_tn_short_bf16(const uint16_t* __restrict__ x,
                                                               const adfl_slq_chunk* __restrict__ chunks,
                                                               const int* __restrict__ tfirst, int64_t max_n,
                                                               double* __restrict__ norms64, float* __restrict__ norms32) {
  __shared__ __attribute__((aligned(16))) float buf[2][8 * kShRow];
  __shared__ float s_acc[8];
  const int ci = tfirst[blockIdx.x];
  const adfl_slq_chunk ch = chunks[ci];
  const int64_t n = (int64_t)(ch.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + ch.nchunks - 1].len;
  if (n > max_n) return;
  const uint16_t* const xt = x + ch.start;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const auto bf = [](uint32_t h) { return __uint_as_float(h << 16); };
  const int64_t nv = n - n % 16;
  float acc = 0.0f;
  if (nv > 0) {
    const int nseg = (int)((nv + kShSeg - 1) / kShSeg);
    const int dt = (int)(((uintptr_t)xt & 15) >> 1);  // the start's offset in its 16-byte block, in elements
    const uint16_t* const xa = xt - dt;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(xa), 0, (int)(((nv + dt) * 2 + 15) & ~15LL),
                                                      0x00020000);
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    struct Blk {
      u4 r0, r1, r2;  // vectors tid and tid + 512 of the segment's block, and vector 1024 (thread 0's)
    };
    const auto load = [&](Blk& k, int j) {
      const int o = j * (kShSeg * 2);
      k.r0 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + tid * 16, 0, 0));
      k.r1 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + (tid + kShThreads) * 16, 0, 0));
      k.r2 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 2 * kShThreads * 16, 0, 0));
    };
    const auto stage = [&](const Blk& k, int j) {
      float* const bj = buf[j & 1];
      const int64_t left = nv - (int64_t)j * kShSeg;  // chain steps' elements from this segment's start
      const auto put = [&](const u4& r, int v) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = 8 * v + q - dt;  // element of the segment: chain e % 8, step e / 8
          if (e >= 0 && e < kShSeg) {
            const uint32_t w = r[q >> 1];
            const float f = e < left ? bf((q & 1) ? (w >> 16) : (w & 0xffffu)) : 0.0f;
            const int st = e >> 3;
            bj[(e & 7) * kShRow + (st >> 4) * kShLS + (st & 15)] = f;
          }
        }
      };
      put(k.r0, tid);
      put(k.r1, tid + kShThreads);
      if (tid == 0) put(k.r2, 2 * kShThreads);
    };
    const int rdo = wave * kShRow + lane * kShLS;
#ifdef ADFL_TN_STATS
    unsigned long long shs[11] = {};
#endif
    const auto run = [&](int j) {
      const float4* const rd = reinterpret_cast<const float4*>(buf[j & 1] + rdo);
      float v[kSL];
#pragma unroll
      for (int q = 0; q < kSL / 4; ++q) {
        const float4 f = rd[q];
        v[4 * q] = f.x;
        v[4 * q + 1] = f.y;
        v[4 * q + 2] = f.z;
        v[4 * q + 3] = f.w;
      }
      acc = short_segment<true>(v, acc, lane SH_PASS);
    };
    Blk ra, rb;
    load(ra, 0);
    load(rb, 1);  // past the end: zeros from the buffer resource (unconditional, so the waits count exactly)
    stage(ra, 0);
    __syncthreads();
    for (int j = 0;; j += 2) {  // block-uniform control flow throughout
      load(ra, j + 2);
      run(j);
      stage(rb, j + 1);
      __syncthreads();
      if (j + 1 >= nseg) break;
      load(rb, j + 3);
      run(j + 1);
      stage(ra, j + 2);
      __syncthreads();
      if (j + 2 >= nseg) break;
    }
#ifdef ADFL_TN_STATS
    shs[8] += 1;
    if (lane == 0)
      for (int i = 0; i < 11; ++i) atomicAdd(&g_sh_stats[i], shs[i]);
#endif
  }
  if (lane == 0) s_acc[wave] = acc;
  __syncthreads();
  if (tid == 0) {  // lane sum left to right, the n % 16 tail with fma, sqrt, to bf16
    float b = s_acc[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) b = b + s_acc[j];
    for (int64_t i = nv; i < n; ++i) {
      const float e = bf(xt[i]);
      b = __builtin_fmaf(e, e, b);
    }
    float r = rn_bf16((float)__builtin_sqrt((double)b));
    if (n == 1) r = __builtin_fabsf(bf(xt[0]));  // a one-element tensor's norm is |x|
    if (norms32) norms32[ch.tensor] = r;
    if (norms64) norms64[ch.tensor] = r;
  }
}

#ifdef ADFL_TN_STATS
__global__ void k_sh_stats_print() {
  const unsigned long long* g = g_sh_stats;
  const double w = g[8] ? (double)g[8] : 1.0;
  printf("sh_stats waves %llu per wave: segments %.2f rounds %.2f exact-map rounds %.2f fma lanes %.2f g+1 finishes %.2f "
         "cycles in segments %.0f in stage %.0f in barriers %.0f total %.0f\n", g[8], g[0] / w, g[1] / w, g[2] / w,
         g[3] / w, g[4] / w, g[5] / w, g[9] / w, g[10] / w, g[6] / w);
  for (int i = 0; i < 11; ++i) g_sh_stats[i] = 0;
  const long long t0 = g_sh_tl[0][0][1];
  for (int w = 0; w < 8; ++w) {
    printf("sh_tl wave %d:", w);
    for (int k = 0; k < g_sh_tln[w]; ++k) printf(" %lld@%lld", g_sh_tl[w][k][0], g_sh_tl[w][k][1] - t0);
    printf("\n");
    g_sh_tln[w] = 0;
  }
}
#endif


// Phase D, one wave per chain: grid (tensors, 8) — by_chunk: (chunks, 8), only tensors' first chunks work
// (layouts of short tensors only, where phase A, which fills tfirst, did not run); blockIdx.y strides the
// chains (one chain per CU, so eight chains of one tensor do not share a SIMD). skip_short: fp32 tensors up
// to kShortMaxF32 are k_tn_short's (ADFL_TN_WALKER builds: the in-order walker's). Each chain's exact accumulator goes to
// chain_acc[tensor][chain] for k_tn_finish.
template <int DT>
__global__ __launch_bounds__(64) void k_tn_chains(const void* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                  const int* __restrict__ tfirst, int by_chunk, int skip_short,
                                                  int threads, const double* __restrict__ S, const Rec* __restrict__ recs,
                                                  const double4* __restrict__ maps, const int* __restrict__ wing,
                                                  const double4* __restrict__ winmaps, double* __restrict__ chain_acc) {
  using D = Dt<DT>;
  const int lane = threadIdx.x;
  int ci;
  if (by_chunk) {
    ci = blockIdx.x;
    if (chunks[ci].first_chunk != ci) return;
  } else {
    ci = tfirst[blockIdx.x];
  }
  const Tensor T = tensor_of(chunks, ci, nall);
  const bool long_ = T.n > short_max<DT>();
  if (skip_short && !long_) return;
  const Split sp = split_of(T.n, threads);
  const int nchains = D::kContig ? (int)sp.nt : D::NC;
#ifdef ADFL_TN_STATS
  const long long c0 = clock64();
#endif
  for (int c = blockIdx.y; c < nchains; c += gridDim.y) {
    const double a = (double)resolve_chain<DT>(x, T, c, sp, S, recs, maps, wing, winmaps, long_, lane);
    if (lane == 0) chain_acc[(int64_t)T.tensor * kMaxChains + c] = a;
  }
#ifdef ADFL_TN_STATS
  TN_STAT(3, clock64() - c0);
#endif
}

// The lane sum (strided) or the chain sums in order (fp16), the tail, sqrt, rounding to the dtype.
template <int DT>
__global__ __launch_bounds__(64) void k_tn_finish(const void* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, int64_t nall,
                                                  const int* __restrict__ tfirst, int by_chunk, int skip_short,
                                                  int threads, const double* __restrict__ chain_acc,
                                                  double* __restrict__ norms64, float* __restrict__ norms32) {
  using D = Dt<DT>;
  constexpr bool W = D::kWide;
  using A_t = typename Acc<W>::T;
  if (threadIdx.x != 0) return;
  int ci;
  if (by_chunk) {
    ci = blockIdx.x;
    if (chunks[ci].first_chunk != ci) return;
  } else {
    ci = tfirst[blockIdx.x];
  }
  const Tensor T = tensor_of(chunks, ci, nall);
  if (skip_short && T.n <= short_max<DT>()) return;
#ifdef ADFL_TN_STATS
  if (blockIdx.x == 0) {
    for (int w = 0; w < 8; ++w) {
      printf("tn_stats chain %d: windows %llu tiles %llu rounds %llu cycles %llu detail %llu segload %llu windesc %llu"
             " winscans %llu exactrounds %llu segcycles %llu recwait %llu scancycles %llu\n", w, g_tn_stats[w][0],
             g_tn_stats[w][1], g_tn_stats[w][2], g_tn_stats[w][3], g_tn_stats[w][4], g_tn_stats[w][5], g_tn_stats[w][6],
             g_tn_stats[w][7], g_tn_stats[w][8], g_tn_stats[w][9], g_tn_stats[w][10], g_tn_stats[w][11]);
      for (int i = 0; i < 12; ++i) g_tn_stats[w][i] = 0;
    }
  }
#endif
  const Split sp = split_of(T.n, threads);
  const double* ca = chain_acc + (int64_t)T.tensor * kMaxChains;
  double r;
  if constexpr (D::kContig) {
    float tot = 0.0f;
    for (int c = 0; c < (int)sp.nt; ++c) tot = tot + (float)ca[c];
    r = (double)__half2float(__float2half_rn((float)__builtin_sqrt((double)tot)));
  } else {
    const int64_t nv = T.n >= D::VB ? T.n - T.n % D::VB : 0;
    A_t b = (A_t)ca[0];  // (0 when there are no steps: fp32 below 8 elements, bf16 below 16)
    for (int c = 1; c < D::NC; ++c) b = b + (A_t)ca[c];
    int64_t d = nv;
    if (DT == ADFL_DTYPE_F32 && T.n - d >= 4) {  // torch's compiled tail: 4 rounded squares in order, then fma
      for (int k = 0; k < 4; ++k) {
        const float e = (float)D::ld(x, T.base + d + k);
        const float sq = e * e;
        b = b + sq;
      }
      d += 4;
    }
    for (int64_t i = d; i < T.n; ++i) {
      const A_t e = (A_t)D::ld(x, T.base + i);
      b = fma_t(e, e, b);
    }
    if constexpr (W) {
      r = __builtin_sqrt((double)b);
    } else {
      const float s = (float)__builtin_sqrt((double)b);  // correctly rounded fp32 sqrt
      r = DT == ADFL_DTYPE_BF16 ? (double)rn_bf16(s) : (double)s;
    }
  }
  if (T.n == 1) r = __builtin_fabs((double)D::ld(x, T.base));  // torch: a one-element tensor's norm is |x|
  if (norms64) norms64[T.tensor] = r;
  if (norms32) norms32[T.tensor] = (float)r;
}

struct Scratch {
  int* tfirst;
  double* S;
  Rec* recs;
  double4* maps;
  int* exact;  // [0] = count, then the chunk indices phase C lists for the exact path
  int* wing;   // phase C2: window summaries, at the slot of the window's first tile
  double4* winmaps;
  double* chain_acc;  // phase D: each chain's exact accumulator, [tensor][kMaxChains]
  double* wsum;       // phase B: each window's sum of S, at the slot of the window's first tile
};
inline int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }
inline int64_t scratch_bytes(int64_t nchunks, int64_t ntensors) {
  return align256(ntensors * 4) + align256(nchunks * kSlots * 8) + align256(nchunks * kSlots * (int64_t)sizeof(Rec)) +
         align256(nchunks * kSlots * 32) + align256((nchunks + 1) * 4) + align256(nchunks * kSlots * 4) +
         align256(nchunks * kSlots * 32) + align256(ntensors * kMaxChains * 8) + align256(nchunks * kSlots * 8);
}
inline Scratch carve(void* p, int64_t nchunks, int64_t ntensors) {
  char* b = (char*)p;
  Scratch s;
  s.tfirst = (int*)b;
  b += align256(ntensors * 4);
  s.S = (double*)b;
  b += align256(nchunks * kSlots * 8);
  s.recs = (Rec*)b;
  b += align256(nchunks * kSlots * (int64_t)sizeof(Rec));
  s.maps = (double4*)b;
  b += align256(nchunks * kSlots * 32);
  s.exact = (int*)b;
  b += align256((nchunks + 1) * 4);
  s.wing = (int*)b;
  b += align256(nchunks * kSlots * 4);
  s.winmaps = (double4*)b;
  b += align256(nchunks * kSlots * 32);
  s.chain_acc = (double*)b;
  b += align256(ntensors * kMaxChains * 8);
  s.wsum = (double*)b;
  return s;
}

template <int DT>
int launch(const void* x, const adfl_slq_chunk* chunks, int64_t nchunks, const int32_t* tfirst, int64_t ntensors,
           int32_t kinds, int threads, void* scratch, double* n64, float* n32, hipStream_t st) {
  const Scratch s = carve(scratch, nchunks, ntensors);
  const bool any_long = (kinds & ADFL_TORCH_NORM_LONG) != 0, any_short = (kinds & ADFL_TORCH_NORM_SHORT) != 0;
  const bool walk = DT == ADFL_DTYPE_F32;  // fp32 short tensors: k_tn_short (ADFL_TN_WALKER builds: the in-order walker)
  // fp16 short tensors: k_tn_short_f16; bf16 / fp64 ones go straight to phase D (with the long ones, or alone)
  const bool own_short = walk || DT == ADFL_DTYPE_F16 || DT == ADFL_DTYPE_BF16;
  if (DT == ADFL_DTYPE_BF16 && any_short) {
    if (!tfirst) {
      k_tn_tfirst<<<(unsigned)((nchunks + 255) / 256), 256, 0, st>>>(chunks, nchunks, s.tfirst);
      tfirst = s.tfirst;
    }
    k_tn_short_bf16<<<(unsigned)ntensors, kShThreads, 0, st>>>((const uint16_t*)x, chunks, tfirst, short_max<DT>(), n64, n32);
#ifdef ADFL_TN_STATS
    k_sh_stats_print<<<1, 1, 0, st>>>();
#endif
  }
  if (DT == ADFL_DTYPE_F16 && any_short) {
    if (!tfirst) {
      k_tn_tfirst<<<(unsigned)((nchunks + 255) / 256), 256, 0, st>>>(chunks, nchunks, s.tfirst);
      tfirst = s.tfirst;
    }
    k_tn_short_f16<<<(unsigned)ntensors, 64 * kH16Waves, 0, st>>>((const uint16_t*)x, chunks, tfirst, kShortMax, threads,
                                                                  n64, n32);
#ifdef ADFL_TN_STATS
    k_sh_stats_print<<<1, 1, 0, st>>>();
#endif
  }
  if (walk && any_short) {
#ifdef ADFL_TN_WALKER
    if (int e = adfl_tn::launch_walk((const float*)x, chunks, nchunks, n32, n64, st)) return e;
#else
    if (!tfirst) {  // no list from the caller: one launch builds it
      k_tn_tfirst<<<(unsigned)((nchunks + 255) / 256), 256, 0, st>>>(chunks, nchunks, s.tfirst);
      tfirst = s.tfirst;
    }
    k_tn_short<<<(unsigned)ntensors, kShThreads, 0, st>>>((const float*)x, chunks, tfirst, kShortMaxF32, n64, n32);
#ifdef ADFL_TN_STATS
    k_sh_stats_print<<<1, 1, 0, st>>>();
#endif
#endif
  }
  if (any_long) {
    if constexpr (!Dt<DT>::kWide)  // fp32 / bf16 / fp16: a 1/16 sample (S only predicts binades)
      k_tn_sums_sampled<DT><<<(unsigned)((nchunks + 4 * kSumsCPW - 1) / (4 * kSumsCPW)), 256, 0, st>>>(x, chunks, nchunks,
                                                                                                     threads, s.tfirst, s.S);
    else
      k_tn_sums<DT><<<(unsigned)nchunks, 256, 0, st>>>(x, chunks, nchunks, threads, s.tfirst, s.S);
    k_tn_winsums<DT><<<dim3((unsigned)ntensors, 8, 8), 256, 0, st>>>(chunks, nchunks, s.tfirst, threads, s.S, s.wsum);
    k_tn_grids<DT><<<dim3((unsigned)ntensors, 8, 8), 256, 0, st>>>(chunks, nchunks, s.tfirst, threads, s.S, s.wsum, s.recs);
    if (hipError_t e = hipMemsetAsync(s.exact, 0, 4, st)) return (int)e;
    if constexpr (DT == ADFL_DTYPE_F32) {
      k_tn_maps_f32<<<(unsigned)nchunks, 256, 0, st>>>((const float*)x, chunks, nchunks, s.recs, s.exact + 1);
      k_tn_maps_exact<DT><<<(unsigned)(nchunks < 1024 ? nchunks : 1024), 256, 0, st>>>(x, chunks, nchunks, threads, s.recs,
                                                                                     s.maps, s.exact + 1);
    } else if constexpr (Dt<DT>::kSq) {  // bf16 / fp16: every long tensor's chunk by exact maps, one pass
      k_tn_maps_exact<DT><<<(unsigned)(nchunks < 2048 ? nchunks : 2048), 256, 0, st>>>(x, chunks, nchunks, threads, s.recs,
                                                                                     s.maps, nullptr);
    } else {
      k_tn_maps<DT><<<(unsigned)nchunks, 256, 0, st>>>(x, chunks, nchunks, threads, s.recs, s.maps, s.exact + 1);
      k_tn_maps_exact<DT><<<(unsigned)(nchunks < 1024 ? nchunks : 1024), 256, 0, st>>>(x, chunks, nchunks, threads, s.recs,
                                                                                     s.maps, s.exact + 1);
    }
    k_tn_windows<DT><<<dim3((unsigned)ntensors, 8, 8), 256, 0, st>>>(chunks, nchunks, s.tfirst, threads, s.recs, s.maps, s.wing,
                                                                     s.winmaps);
    // one wave per chain: 8 strided chains, or fp16's pieces (up to min(threads, 512) of them)
    const unsigned cy = DT == ADFL_DTYPE_F16 ? (unsigned)(threads < 8 ? 8 : (threads > kMaxChains ? kMaxChains : threads)) : 8u;
    k_tn_chains<DT><<<dim3((unsigned)ntensors, cy), 64, 0, st>>>(x, chunks, nchunks, s.tfirst, 0, own_short, threads, s.S, s.recs,
                                                                 s.maps, s.wing, s.winmaps, s.chain_acc);
    k_tn_finish<DT><<<(unsigned)ntensors, 64, 0, st>>>(x, chunks, nchunks, s.tfirst, 0, own_short, threads, s.chain_acc, n64,
                                                       n32);
  } else if (!own_short) {
    k_tn_chains<DT><<<dim3((unsigned)nchunks, 8), 64, 0, st>>>(x, chunks, nchunks, s.tfirst, 1, 0, threads, s.S, s.recs,
                                                                s.maps, s.wing, s.winmaps, s.chain_acc);
    k_tn_finish<DT><<<(unsigned)nchunks, 64, 0, st>>>(x, chunks, nchunks, s.tfirst, 1, 0, threads, s.chain_acc, n64, n32);
  }
  return (int)hipGetLastError();
}

}  // namespace adfl_tnx


extern "C" {

int64_t adfl_torch_norm_scratch_bytes(int64_t nchunks, int64_t ntensors) {
  if (nchunks < 0 || ntensors < 0) return ADFL_E_ARG;
  return adfl_tnx::scratch_bytes(nchunks, ntensors);
}

int64_t adfl_torch_norm_short_max(void) { return adfl_tnx::kShortMax; }

int64_t adfl_torch_norm_short_max_dt(int32_t dtype) {
  if (dtype < ADFL_DTYPE_F32 || dtype > ADFL_DTYPE_F64) return ADFL_E_ARG;
  switch (dtype) {
    case ADFL_DTYPE_F32: return adfl_tnx::short_max<ADFL_DTYPE_F32>();
    case ADFL_DTYPE_BF16: return adfl_tnx::short_max<ADFL_DTYPE_BF16>();
    case ADFL_DTYPE_F16: return adfl_tnx::short_max<ADFL_DTYPE_F16>();
    default: return adfl_tnx::short_max<ADFL_DTYPE_F64>();
  }
}

int adfl_torch_norms_work(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks,
                          const int32_t* d_tfirst, int64_t ntensors, int32_t kinds, int32_t threads, void* d_scratch,
                          int64_t scratch_bytes, double* d_norms64, float* d_norms32, void* stream) {
  if (nchunks < 0 || ntensors < 0 || (nchunks > 0 && (!d_x || !d_chunks || !d_scratch)) || (!d_norms64 && !d_norms32))
    return ADFL_E_ARG;
  if (nchunks == 0) return ADFL_OK;
  // threads only shapes fp16's split (at most kMaxChains pieces per tensor); the other dtypes ignore it
  if (ntensors <= 0 || ntensors > nchunks || threads < 1 || (dtype == ADFL_DTYPE_F16 && threads > adfl_tnx::kMaxChains))
    return ADFL_E_ARG;
  if (scratch_bytes < adfl_tnx::scratch_bytes(nchunks, ntensors)) return ADFL_E_WORKSPACE;
  if (((uintptr_t)d_scratch & 255) != 0) return ADFL_E_ALIGN;
  if (kinds == 0) kinds = ADFL_TORCH_NORM_SHORT | ADFL_TORCH_NORM_LONG;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case ADFL_DTYPE_F32:
      return adfl_tnx::launch<ADFL_DTYPE_F32>(d_x, d_chunks, nchunks, d_tfirst, ntensors, kinds, threads, d_scratch, d_norms64, d_norms32, st);
    case ADFL_DTYPE_BF16:
      return adfl_tnx::launch<ADFL_DTYPE_BF16>(d_x, d_chunks, nchunks, d_tfirst, ntensors, kinds, threads, d_scratch, d_norms64, d_norms32, st);
    case ADFL_DTYPE_F16:
      return adfl_tnx::launch<ADFL_DTYPE_F16>(d_x, d_chunks, nchunks, d_tfirst, ntensors, kinds, threads, d_scratch, d_norms64, d_norms32, st);
    case ADFL_DTYPE_F64:
      return adfl_tnx::launch<ADFL_DTYPE_F64>(d_x, d_chunks, nchunks, d_tfirst, ntensors, kinds, threads, d_scratch, d_norms64, d_norms32, st);
    default:
      return ADFL_E_ARG;
  }
}

int adfl_torch_norms(int32_t dtype, const void* d_x, const adfl_slq_chunk* d_chunks, int64_t nchunks, int64_t ntensors,
                     int32_t kinds, int32_t threads, void* d_scratch, int64_t scratch_bytes, double* d_norms64,
                     float* d_norms32, void* stream) {
  return adfl_torch_norms_work(dtype, d_x, d_chunks, nchunks, nullptr, ntensors, kinds, threads, d_scratch,
                               scratch_bytes, d_norms64, d_norms32, stream);
}

}  // extern "C"
