// qerror_ref.hip — the reference's q-error metrics (Src/ADFL/model.py:256-323: parameter_relative_mse,
// parameter_cosine_similarity, exclude_bias=True, as Src/ADFL/Client/worker.py:186-189 calls them) with
// torch 2.10's CPU fp32 summation order, bit for bit. See include/adfl_qerror.h for what is computed and
// oracle/slq_oracle.c (oracle_torch_sum_f32) for the order, restated from ATen's cascade_sum:
//
//   A segment (one at::parallel_for range, or the whole tensor) of L >= 8 values is 32 streams: lane l of
//   ILP partial p holds value 32 g + 8 p + l for g < G = L / 32 (rounded down to whole 4-vector groups).
//   Each stream is a 4-level cascade with step 2^lp (lp = max(4, CeilLog2(G) / 4)): level 0 sums `step`
//   values from 0, level 1 `step` level-0 sums, level 2 `step` level-1 sums, level 3 all level-2 sums; the
//   incomplete tails are folded ((acc0 + acc1) + acc2) + acc3. Then the leftover vectors into partial 0, the
//   partials per lane ((p0 + p1) + p2) + p3, and 0 + the scalar tail + lanes 0..7 in order.
//
// Work split (every block independent, no atomics):
//   k_qe_units  one block per complete level-1 unit (32 step^2 consecutive values of a segment): 32 x step
//               level-0 sums in parallel, then the 32 level-1 sums — the bulk of the bytes, read once;
//   k_qe_segs   one wave per segment: its level-2 / level-3 sums over the unit results, the incomplete
//               unit at its end, the leftovers and the lane combine;
//   k_qe_sites  one thread per sum: a serial sum is its segment's; a two-pass one the cascade over the T
//               per-thread partials (zeros past the ranges used).
// Both outputs of a tensor (sum (x - d)^2 and sum x^2) ride the same pass; the cosine's product vector is
// one more site over the whole concatenation.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "adfl_qerror.h"
#include "adfl_slq.h"

namespace adfl_qe {

constexpr int64_t kGrain = 32768;  // at::internal::GRAIN_SIZE
constexpr int64_t kMagic = 0x71657231;
constexpr int kMaxLp = 6;          // step 64: segments up to 2^33 elements
constexpr int kMaxThreads = 4096;

// plan: int64 header, then sites, segments, units (all int64)
enum Hdr { H_MAGIC, H_NSITES, H_NSEGS, H_NUNITS, H_THREADS, H_NTENSORS, H_SITES, H_SEGS, H_UNITS, H_SCRATCH,
           H_BYTES, H_COUNT = 16 };
enum Site { S_BEGIN, S_LEN, S_MODE, S_SEG0, S_NSEG, S_OUT0, S_OUT1, S_TWOPASS, S_COUNT = 8 };
enum Seg { G_BEGIN, G_LEN, G_SITE, G_LP, G_UNIT0, G_NUNITS, G_MODE, G_COUNT = 8 };
enum Unit { U_SEG, U_M, U_COUNT = 2 };
enum Mode { kEX = 0, kCOS = 1 };

__host__ __device__ inline int level_power(int64_t count) {
  int c = 1;
  if (count > 2) {
    uint64_t v = (uint64_t)count - 1;
    c = 0;
    while (v) {
      ++c;
      v >>= 1;
    }
  }
  return c / 4 > 4 ? c / 4 : 4;
}

// the two values of element i: mode kEX (fp32 (x - d)^2, (x - 0)^2); mode kCOS ((x / n1) * (d / n2), 0)
struct Val {
  const float* x;
  const float* d;
  int mode;
  float n1, n2;
  __device__ __forceinline__ float operator()(int64_t i, int f) const {
    const float a = x[i];
    if (mode == kEX) {
      if (f == 0) {
        const float df = a - d[i];
        return df * df;
      }
      const float z = a - 0.0f;
      return z * z;
    }
    if (f != 0) return 0.0f;
    const float p = __fdiv_rn(a, n1), q = __fdiv_rn(d[i], n2);
    return p * q;
  }
};

// ---- serial restatement (one thread), for short segments and the two-pass combine
template <class Get>
__device__ float level_seq(const Get& get, int64_t count, int64_t stride, int64_t off) {
  const int lp = level_power(count);
  const int64_t step = (int64_t)1 << lp, mask = step - 1;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int64_t i = 0;
  while (i + step <= count) {
    for (int64_t j = 0; j < step; ++j, ++i) acc[0] = acc[0] + get(off + i * stride);
    for (int j = 1; j < 4; ++j) {
      acc[j] = acc[j] + acc[j - 1];
      acc[j - 1] = 0.0f;
      if ((i & (mask << (j * lp))) != 0) break;
    }
  }
  for (; i < count; ++i) acc[0] = acc[0] + get(off + i * stride);
  for (int j = 1; j < 4; ++j) acc[0] = acc[0] + acc[j];
  return acc[0];
}
template <class Get>
__device__ float row_seq(const Get& get, int64_t n, int64_t stride, int64_t off) {
  const int64_t g = n / 4;
  float p[4];
  for (int k = 0; k < 4; ++k) p[k] = level_seq(get, g, 4 * stride, off + k * stride);
  for (int64_t i = 4 * g; i < n; ++i) p[0] = p[0] + get(off + i * stride);
  for (int k = 1; k < 4; ++k) p[0] = p[0] + p[k];
  return p[0];
}
template <class Get>
__device__ float inner_seq(const Get& get, int64_t n) {
  if (n < 8) return row_seq(get, n, 1, 0);
  const int64_t v = n / 8;
  float acc = 0.0f;
  for (int64_t i = 8 * v; i < n; ++i) acc = acc + get(i);
  for (int l = 0; l < 8; ++l) acc = acc + row_seq(get, v, 8, l);
  return acc;
}

__device__ __forceinline__ float clamp_eps(float v) { return v != v ? v : (v < 1e-8f ? 1e-8f : v); }

// ---- k_qe_units: a complete level-1 unit of a segment, both values; out: 64 floats per unit (f * 32 + s)
__global__ __launch_bounds__(256) void k_qe_units(const float* __restrict__ x, const float* __restrict__ d,
                                                  const int64_t* __restrict__ plan, const float* __restrict__ norms,
                                                  float* __restrict__ unit_out) {
  __shared__ float s0[2][64][33];
  const int tid = threadIdx.x;
  const int64_t* U = plan + plan[H_UNITS] + (int64_t)blockIdx.x * U_COUNT;
  const int64_t* G = plan + plan[H_SEGS] + U[U_SEG] * G_COUNT;
  const int lp = (int)G[G_LP];
  const int step = 1 << lp;
  const Val val{x, d, (int)G[G_MODE], clamp_eps(norms[0]), clamp_eps(norms[1])};
  const int64_t base = G[G_BEGIN] + U[U_M] * 32 * (int64_t)step * step;
  for (int j = tid; j < 32 * step; j += 256) {
    const int s = j & 31, k = j >> 5;
    const int64_t e0 = base + (int64_t)k * step * 32 + s;
    float a0 = 0.0f, a1 = 0.0f;
    for (int i0 = 0; i0 < step; i0 += 16) {
      float v0[16], v1[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v0[i] = val(e0 + (int64_t)(i0 + i) * 32, 0);
        v1[i] = val(e0 + (int64_t)(i0 + i) * 32, 1);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        a0 = a0 + v0[i];
        a1 = a1 + v1[i];
      }
    }
    s0[0][k][s] = a0;
    s0[1][k][s] = a1;
  }
  __syncthreads();
  if (tid < 64) {
    const int f = tid >> 5, s = tid & 31;
    float b1 = 0.0f;
    for (int k = 0; k < step; ++k) b1 = b1 + s0[f][k][s];
    unit_out[(int64_t)blockIdx.x * 64 + tid] = b1;
  }
}

// ---- k_qe_segs: one wave per segment; seg_out: 2 floats per segment (0 + the segment's sum)
__global__ __launch_bounds__(64) void k_qe_segs(const float* __restrict__ x, const float* __restrict__ d,
                                                const int64_t* __restrict__ plan, const float* __restrict__ norms,
                                                const float* __restrict__ unit_out, float* __restrict__ seg_out) {
  __shared__ float sp[2][32];
  const int lane = threadIdx.x, f = lane >> 5, s = lane & 31, p = s >> 3, l = s & 7;
  const int64_t sg = blockIdx.x;
  const int64_t* G = plan + plan[H_SEGS] + sg * G_COUNT;
  const Val val{x, d, (int)G[G_MODE], clamp_eps(norms[0]), clamp_eps(norms[1])};
  const int64_t b = G[G_BEGIN], L = G[G_LEN];
  if (L < 8) {  // scalar row_sum (scalar_outer_sum with one row)
    if (lane < 2) {
      const auto get = [&](int64_t i) { return val(b + i, lane); };
      seg_out[sg * 2 + lane] = 0.0f + row_seq(get, L, 1, 0);
    }
    return;
  }
  const int64_t V = L / 8, Gn = V / 4;
  const int lp = (int)G[G_LP];
  const int64_t step = (int64_t)1 << lp;
  const int64_t nb0 = Gn >> lp, nb1 = nb0 >> lp, nb2 = nb1 >> lp;
  const float* B1 = unit_out + G[G_UNIT0] * 64 + lane;
  float acc3 = 0.0f;
  for (int64_t q = 0; q < nb2; ++q) {
    float b2 = 0.0f;
    for (int64_t j0 = 0; j0 < step; j0 += 16) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = B1[(q * step + j0 + i) * 64];
#pragma unroll
      for (int i = 0; i < 16; ++i) b2 = b2 + v[i];
    }
    acc3 = acc3 + b2;
  }
  float acc2 = 0.0f;
  for (int64_t q = nb2 * step; q < nb1; ++q) acc2 = acc2 + B1[q * 64];
  float acc1 = 0.0f;
  for (int64_t k = nb1 * step; k < nb0; ++k) {
    float b0 = 0.0f;
    for (int64_t i0 = 0; i0 < step; i0 += 16) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = val(b + ((k * step + i0 + i) * 32) + s, f);
#pragma unroll
      for (int i = 0; i < 16; ++i) b0 = b0 + v[i];
    }
    acc1 = acc1 + b0;
  }
  float acc0 = 0.0f;
  for (int64_t g = nb0 * step; g < Gn; ++g) acc0 = acc0 + val(b + g * 32 + s, f);
  float P = acc0 + acc1;
  P = P + acc2;
  P = P + acc3;
  if (p == 0)
    for (int64_t v = 4 * Gn; v < V; ++v) P = P + val(b + 8 * v + l, f);
  sp[f][s] = P;
  __syncthreads();
  if (s == 0) {
    float fin = 0.0f;
    for (int64_t o = 8 * V; o < L; ++o) fin = fin + val(b + o, f);
    for (int k = 0; k < 8; ++k) {
      float q = sp[f][k];
      q = q + sp[f][8 + k];
      q = q + sp[f][16 + k];
      q = q + sp[f][24 + k];
      fin = fin + q;
    }
    seg_out[sg * 2 + f] = 0.0f + fin;
  }
}

// ---- k_qe_sites: one thread per (site, value)
__global__ __launch_bounds__(64) void k_qe_sites(const int64_t* __restrict__ plan, const float* __restrict__ seg_out,
                                                 float* __restrict__ out) {
  const int64_t id = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t nsites = plan[H_NSITES];
  if (id >= 2 * nsites) return;
  const int64_t si = id >> 1;
  const int f = (int)(id & 1);
  const int64_t* S = plan + plan[H_SITES] + si * S_COUNT;
  const int64_t o = f ? S[S_OUT1] : S[S_OUT0];
  if (o < 0) return;
  const int64_t s0 = S[S_SEG0], ns = S[S_NSEG];
  float r;
  if (!S[S_TWOPASS]) {
    r = seg_out[s0 * 2 + f];
  } else {
    const auto get = [&](int64_t i) { return i < ns ? seg_out[(s0 + i) * 2 + f] : 0.0f; };
    r = 0.0f + inner_seq(get, plan[H_THREADS]);
  }
  out[o] = r;
}

// ---- host: the plan
int64_t build_plan(const int64_t* sizes, int32_t ntensors, int32_t threads, int64_t* out, int64_t cap) {
  if (!sizes || ntensors < 1 || threads < 1 || threads > kMaxThreads) return ADFL_E_ARG;
  int64_t total = 0;
  for (int32_t t = 0; t < ntensors; ++t) {
    if (sizes[t] < 1) return ADFL_E_ARG;
    total += sizes[t];
  }
  const int64_t nsites = ntensors + 1;
  // pass 1: count segments and units; pass 2: write
  int64_t nsegs = 0, nunits = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const int64_t off_sites = H_COUNT, off_segs = off_sites + nsites * S_COUNT, off_units = off_segs + nsegs * G_COUNT;
    const int64_t words = off_units + nunits * U_COUNT;
    const bool write = pass == 1 && out && cap >= words * 8;
    int64_t sg = 0, un = 0, begin = 0;
    for (int64_t si = 0; si < nsites; ++si) {
      const bool cos = si == ntensors;
      const int64_t b = cos ? 0 : begin, len = cos ? total : sizes[si];
      if (!cos) begin += len;
      int64_t nt = 1, cs = len;
      const bool two = len >= kGrain && threads > 1;
      if (two) {
        nt = (len + kGrain - 1) / kGrain;
        if (nt > threads) nt = threads;
        cs = (len + nt - 1) / nt;
      }
      const int64_t seg0 = sg;
      for (int64_t t = 0; t < nt; ++t) {
        const int64_t lo = t * cs;
        if (lo >= len) break;
        const int64_t L = cs < len - lo ? cs : len - lo;
        int lp = 0;
        int64_t nb1 = 0;
        if (L >= 8) {
          const int64_t Gn = L / 32;
          lp = level_power(Gn);
          if (lp > kMaxLp) return ADFL_E_ARG;
          nb1 = (Gn >> lp) >> lp;
        }
        if (write) {
          int64_t* g = out + off_segs + sg * G_COUNT;
          g[G_BEGIN] = b + lo;
          g[G_LEN] = L;
          g[G_SITE] = si;
          g[G_LP] = lp;
          g[G_UNIT0] = un;
          g[G_NUNITS] = nb1;
          g[G_MODE] = cos ? kCOS : kEX;
          g[7] = 0;
          for (int64_t m = 0; m < nb1; ++m) {
            out[off_units + (un + m) * U_COUNT + U_SEG] = sg;
            out[off_units + (un + m) * U_COUNT + U_M] = m;
          }
        }
        un += nb1;
        ++sg;
      }
      if (write) {
        int64_t* s = out + off_sites + si * S_COUNT;
        s[S_BEGIN] = b;
        s[S_LEN] = len;
        s[S_MODE] = cos ? kCOS : kEX;
        s[S_SEG0] = seg0;
        s[S_NSEG] = sg - seg0;
        s[S_OUT0] = cos ? 2 * (int64_t)ntensors : si;
        s[S_OUT1] = cos ? -1 : ntensors + si;
        s[S_TWOPASS] = two ? 1 : 0;
      }
    }
    nsegs = sg;
    nunits = un;
    if (pass == 1) {
      const int64_t bytes = words * 8;
      if (write) {
        std::memset(out, 0, H_COUNT * 8);
        out[H_MAGIC] = kMagic;
        out[H_NSITES] = nsites;
        out[H_NSEGS] = nsegs;
        out[H_NUNITS] = nunits;
        out[H_THREADS] = threads;
        out[H_NTENSORS] = ntensors;
        out[H_SITES] = off_sites;
        out[H_SEGS] = off_segs;
        out[H_UNITS] = off_units;
        out[H_SCRATCH] = ((nunits * 64 * 4 + 255) & ~(int64_t)255) + nsegs * 2 * 4;
        out[H_BYTES] = bytes;
      }
      return bytes;
    }
  }
  return ADFL_E_ARG;
}

}  // namespace adfl_qe

extern "C" {

int64_t adfl_qerror_ref_plan(const int64_t* sizes, int32_t ntensors, int32_t threads, void* h_plan, int64_t plan_bytes) {
  return adfl_qe::build_plan(sizes, ntensors, threads, (int64_t*)h_plan, plan_bytes);
}

int64_t adfl_qerror_ref_scratch_bytes(const void* h_plan) {
  const int64_t* p = (const int64_t*)h_plan;
  if (!p || p[adfl_qe::H_MAGIC] != adfl_qe::kMagic) return ADFL_E_ARG;
  return p[adfl_qe::H_SCRATCH];
}

int adfl_qerror_ref(const float* d_x, const float* d_d, const void* h_plan, const void* d_plan, const float* d_norms,
                    void* d_scratch, int64_t scratch_bytes, float* d_out, void* stream) {
  using namespace adfl_qe;
  if (!d_x || !d_d || !h_plan || !d_plan || !d_norms || !d_scratch || !d_out) return ADFL_E_ARG;
  const int64_t* h = (const int64_t*)h_plan;  // the counts the launches need: the host copy's header
  hipStream_t st = (hipStream_t)stream;
  if (h[H_MAGIC] != kMagic) return ADFL_E_ARG;
  if (scratch_bytes < h[H_SCRATCH]) return ADFL_E_WORKSPACE;
  if (((uintptr_t)d_scratch & 255) != 0) return ADFL_E_ALIGN;
  float* unit_out = (float*)d_scratch;
  float* seg_out = (float*)((char*)d_scratch + ((h[H_NUNITS] * 64 * 4 + 255) & ~(int64_t)255));
  const int64_t* plan = (const int64_t*)d_plan;
  if (h[H_NUNITS] > 0)
    hipLaunchKernelGGL(k_qe_units, dim3((unsigned)h[H_NUNITS]), dim3(256), 0, st, d_x, d_d, plan, d_norms, unit_out);
  hipLaunchKernelGGL(k_qe_segs, dim3((unsigned)h[H_NSEGS]), dim3(64), 0, st, d_x, d_d, plan, d_norms, unit_out, seg_out);
  hipLaunchKernelGGL(k_qe_sites, dim3((unsigned)((2 * h[H_NSITES] + 63) / 64)), dim3(64), 0, st, plan, seg_out, d_out);
  return (int)hipGetLastError();
}

}  // extern "C"
