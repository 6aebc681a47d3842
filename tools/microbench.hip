// microbench.hip — per-kernel timing of the product codec kernels on the 1 GiB C2 workload, one
// process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), plus the knobs being tuned.
// Not part of the product; it #includes the product source to reach its kernels.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench tools/microbench.hip
//   ./tools/microbench [log2_elems=28]
#include "../ad-federatedlearning_amd/csrc/slq_codec.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

namespace mb {
__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ in, float4* __restrict__ out, int64_t n4) {
  const int64_t s = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += s) out[i] = in[i];
}
template <bool NT>
__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ in, int64_t n4, uint32_t* sink) {
  const int64_t s = (int64_t)gridDim.x * 256;
  uint32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += s) m ^= abs_bits4(load4<NT>(in + i));
  if (m == 0x12345678u) sink[0] = m;
}
__global__ __launch_bounds__(256) void k_write_nt(float4* __restrict__ out, int64_t n4) {
  const int64_t s = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += s) store4_nt(out + i, make_float4(1.f, 2.f, 3.f, 4.f));
}
// the decode's store shape without its loads: wave tiles of 4 float4 NT stores per lane (1 KiB per
// wave-instruction), tile_grid blocks
__global__ __launch_bounds__(256) void k_write_nt_tiles(float4* __restrict__ out, int64_t ntiles) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < ntiles; t += wstride) {
    float4* o4 = out + t * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) store4_nt(o4 + j * 64 + lane, make_float4(1.f, 2.f, 3.f, (float)j));
  }
}
// quantize with the first tiles' loads issued before the partial reduction (hides its latency) and UT
// tiles in flight per wave iteration.
template <int UT, bool PREFETCH>
__global__ __launch_bounds__(kBlock) void k_quant_pf(const float* __restrict__ x, int64_t n, float qmax,
                                                    const uint32_t* __restrict__ partials, int8_t* __restrict__ q,
                                                    float* __restrict__ scale_out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][UT][kTile / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint4* q16 = reinterpret_cast<uint4*>(q);
  const int64_t ntiles = n / kTile;
  const int64_t wstride = (int64_t)gridDim.x * kWaves * UT;
  int64_t t0 = ((int64_t)blockIdx.x * kWaves + wave) * UT;
  float4 v[UT][4];
  auto issue = [&](int64_t tb) {
#pragma unroll
    for (int u = 0; u < UT; ++u)
      if (tb + u < ntiles) {
        const int64_t t = ntiles - 1 - (tb + u);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = load4<true>(x4 + t * 256 + j * 64 + lane);
      }
  };
  if (PREFETCH) issue(t0);
  const ScaleInv si = make_scale(reduce_partials(partials, (int)partials[kCountSlot]), qmax);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = si.scale;
  if (!PREFETCH) issue(t0);
  for (; t0 < ntiles; t0 += wstride) {
#pragma unroll
    for (int u = 0; u < UT; ++u)
      if (t0 + u < ntiles) {
#pragma unroll
        for (int j = 0; j < 4; ++j) lds[wave][u][j * 64 + lane] = quant4(v[u][j], si.inv);
      }
    __builtin_amdgcn_wave_barrier();
    uint4 o[UT];
#pragma unroll
    for (int u = 0; u < UT; ++u) o[u] = reinterpret_cast<const uint4*>(lds[wave][u])[lane];
    __builtin_amdgcn_wave_barrier();
    issue(t0 + wstride);  // next iteration's loads before this iteration's stores
#pragma unroll
    for (int u = 0; u < UT; ++u)
      if (t0 + u < ntiles) q16[(ntiles - 1 - (t0 + u)) * 64 + lane] = o[u];
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile + threadIdx.x; i < n; i += kBlock) q[i] = (int8_t)quant1(x[i], si.inv);
}

// dequantize with the next tile's payload load issued before the current tile's stores.
template <int UT>
__global__ __launch_bounds__(kBlock) void k_deq_pf(const int8_t* __restrict__ q, int64_t n, const float* __restrict__ scale_p,
                                                  float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves][UT][kTile / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* q16 = reinterpret_cast<const uint4*>(q);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ntiles = n / kTile;
  const int64_t wstride = (int64_t)gridDim.x * kWaves * UT;
  int64_t t0 = ((int64_t)blockIdx.x * kWaves + wave) * UT;
  uint4 p[UT];
  auto issue = [&](int64_t tb) {
#pragma unroll
    for (int u = 0; u < UT; ++u)
      if (tb + u < ntiles) p[u] = q16[(tb + u) * 64 + lane];
  };
  issue(t0);
  const float s = *scale_p;
  for (; t0 < ntiles; t0 += wstride) {
#pragma unroll
    for (int u = 0; u < UT; ++u) reinterpret_cast<uint4*>(lds[wave][u])[lane] = p[u];
    __builtin_amdgcn_wave_barrier();
    uint32_t w[UT][4];
#pragma unroll
    for (int u = 0; u < UT; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) w[u][j] = lds[wave][u][j * 64 + lane];
    __builtin_amdgcn_wave_barrier();
    issue(t0 + wstride);
#pragma unroll
    for (int u = 0; u < UT; ++u)
      if (t0 + u < ntiles) {
#pragma unroll
        for (int j = 0; j < 4; ++j) store4_nt(o4 + (t0 + u) * 256 + j * 64 + lane, dequant4(w[u][j], s));
      }
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile + threadIdx.x; i < n; i += kBlock) out[i] = s * (float)q[i];
}
}  // namespace mb

static float med(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const int64_t n = 1LL << lg;
  float *x, *out, *scale, *tmp;
  int8_t* q;
  uint32_t* ws;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&q, n * 8));  // room for 8 gathered payload rows
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&tmp, n * 4));
  CK(hipMalloc(&ws, 16384));
  CK(hipMalloc(&scale, 64));
  {
    std::vector<float> h(1 << 20);
    uint32_t st = 12345;
    for (auto& v : h) {
      st = st * 1664525u + 1013904223u;
      v = ((int)(st >> 8) - (1 << 23)) * 1e-9f;
    }
    for (int64_t o = 0; o < n; o += h.size()) CK(hipMemcpy(x + o, h.data(), std::min<int64_t>(h.size(), n - o) * 4, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t ev[4];
  for (auto& e : ev) CK(hipEventCreate(&e));
  const double gb = n * 1e-9;
  auto ms = [&](hipEvent_t a, hipEvent_t b) {
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    return t;
  };

  // ---- 1. variant matrix on the int8 round trip (absmax -> quantize -> dequantize)
  using L = std::function<void()>;
  struct V { std::string name; L fn; };
  const int tg = tile_grid(n / kTile);
  auto agrid = [&](int cap) { return clamp_grid((n >> 2) / (8 * kBlock), cap); };
  std::vector<V> A = {
      {"abs_U8_g1024", [&] { hipLaunchKernelGGL(k_absmax_flat<8>, dim3(agrid(1024)), dim3(kBlock), 0, st, x, n, (int64_t)0, ws); }},
  };
  std::vector<V> Q = {
      {"q_rev", [&] { hipLaunchKernelGGL((k_quantize_flat<true, false>), dim3(tg), dim3(kBlock), 0, st, x, n, 127.f, ws, q, scale); }},
      {"q_pf1", [&] { hipLaunchKernelGGL((mb::k_quant_pf<1, true>), dim3(tg), dim3(kBlock), 0, st, x, n, 127.f, ws, q, scale); }},
      {"q_pf2", [&] { hipLaunchKernelGGL((mb::k_quant_pf<2, true>), dim3(tg), dim3(kBlock), 0, st, x, n, 127.f, ws, q, scale); }},
      {"q_nopf2", [&] { hipLaunchKernelGGL((mb::k_quant_pf<2, false>), dim3(tg), dim3(kBlock), 0, st, x, n, 127.f, ws, q, scale); }},
      {"q_pf2_g1024", [&] { hipLaunchKernelGGL((mb::k_quant_pf<2, true>), dim3(1024), dim3(kBlock), 0, st, x, n, 127.f, ws, q, scale); }},
      {"q_pf4_g1024", [&] { hipLaunchKernelGGL((mb::k_quant_pf<4, true>), dim3(1024), dim3(kBlock), 0, st, x, n, 127.f, ws, q, scale); }},
  };
  std::vector<V> D = {
      {"d_fwd", [&] { hipLaunchKernelGGL((k_dequantize_flat<false, false>), dim3(tg), dim3(kBlock), 0, st, q, n, scale, out); }},
      {"d_ldnt", [&] { hipLaunchKernelGGL((k_dequantize_flat<false, true>), dim3(tg), dim3(kBlock), 0, st, q, n, scale, out); }},
      {"d_pf1", [&] { hipLaunchKernelGGL((mb::k_deq_pf<1>), dim3(tg), dim3(kBlock), 0, st, q, n, scale, out); }},
      {"d_pf2", [&] { hipLaunchKernelGGL((mb::k_deq_pf<2>), dim3(tg), dim3(kBlock), 0, st, q, n, scale, out); }},
      {"d_pf2_g1024", [&] { hipLaunchKernelGGL((mb::k_deq_pf<2>), dim3(1024), dim3(kBlock), 0, st, q, n, scale, out); }},
  };
  {  // correctness of every variant against the product kernels
    adfl_slq_encode(x, n, 8, q, scale, ws, 16384, st);
    adfl_slq_dequantize(q, n, scale, out, st);
    CK(hipStreamSynchronize(st));
    std::vector<int8_t> q_ref(n), q_h(n);
    std::vector<float> d_ref(n), d_h(n);
    CK(hipMemcpy(q_ref.data(), q, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d_ref.data(), out, n * 4, hipMemcpyDeviceToHost));
    for (auto& v : Q) {
      CK(hipMemset(q, 0, n));
      v.fn();
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(q_h.data(), q, n, hipMemcpyDeviceToHost));
      printf("check %-14s %s\n", v.name.c_str(), memcmp(q_h.data(), q_ref.data(), n) ? "MISMATCH" : "ok");
    }
    for (auto& v : D) {
      CK(hipMemset(out, 0, n * 4));
      v.fn();
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(d_h.data(), out, n * 4, hipMemcpyDeviceToHost));
      printf("check %-14s %s\n", v.name.c_str(), memcmp(d_h.data(), d_ref.data(), n * 4) ? "MISMATCH" : "ok");
    }
  }
  struct Row { std::string name; std::vector<float> a, q, d; };
  std::vector<Row> rows;
  for (auto& a : A) for (auto& qk : Q) for (auto& d : D) rows.push_back({a.name + " > " + qk.name + " > " + d.name, {}, {}, {}});
  const int ROUNDS = 5, STEPS = 6;
  for (int r = 0; r < ROUNDS; ++r) {
    size_t i = 0;
    for (auto& a : A) for (auto& qk : Q) for (auto& d : D) {
      for (int s = 0; s < STEPS; ++s) {
        (void)hipEventRecord(ev[0], st);
        a.fn();
        (void)hipEventRecord(ev[1], st);
        qk.fn();
        (void)hipEventRecord(ev[2], st);
        d.fn();
        (void)hipEventRecord(ev[3], st);
        CK(hipEventSynchronize(ev[3]));
        rows[i].a.push_back(ms(ev[0], ev[1]));
        rows[i].q.push_back(ms(ev[1], ev[2]));
        rows[i].d.push_back(ms(ev[2], ev[3]));
      }
      ++i;
    }
  }
  std::sort(rows.begin(), rows.end(), [&](const Row& u, const Row& v) {
    return med(u.a) + med(u.q) + med(u.d) < med(v.a) + med(v.q) + med(v.d);
  });
  printf("%-44s %8s %8s %8s | %8s %6s\n", "int8 round trip", "absmax", "quant", "deq", "sum ms", "frac");
  for (auto& R : rows) {
    const float t = med(R.a) + med(R.q) + med(R.d);
    printf("%-44s %8.4f %8.4f %8.4f | %8.4f %6.3f\n", R.name.c_str(), med(R.a), med(R.q), med(R.d), t,
           14.0 * gb / (t * 1e-3) / 8000.0);
  }

  // ---- 1b. cold decode: the Infinity Cache flushed (a 1 GiB read of another buffer) before each dequantize,
  // as when the payload arrives from another process
  {
    printf("%-20s %8s %8s\n", "cold decode", "ms", "frac");
    for (auto& d : D) {
      std::vector<float> t;
      for (int s = 0; s < 20; ++s) {
        hipLaunchKernelGGL(mb::k_read<false>, dim3(2048), dim3(256), 0, st, (const float4*)tmp, n >> 2, ws);
        (void)hipEventRecord(ev[0], st);
        d.fn();
        (void)hipEventRecord(ev[1], st);
        CK(hipEventSynchronize(ev[1]));
        t.push_back(ms(ev[0], ev[1]));
      }
      printf("%-20s %8.4f %6.3f\n", d.name.c_str(), med(t), 5.0 * gb / (med(t) * 1e-3) / 8000.0);
    }
  }

  // ---- 2. int4 round trip (13 B/elem algorithmic)
  {
    std::vector<float> a, qq, d;
    for (int s = 0; s < 30; ++s) {
      (void)hipEventRecord(ev[0], st);
      adfl_slq_absmax(x, n, ws, 16384, st);
      (void)hipEventRecord(ev[1], st);
      adfl_slq_quantize_int4(x, n, 4, ws, (uint8_t*)q, scale, st);
      (void)hipEventRecord(ev[2], st);
      adfl_slq_dequantize_int4((uint8_t*)q, n, scale, out, st);
      (void)hipEventRecord(ev[3], st);
      CK(hipEventSynchronize(ev[3]));
      a.push_back(ms(ev[0], ev[1]));
      qq.push_back(ms(ev[1], ev[2]));
      d.push_back(ms(ev[2], ev[3]));
    }
    const float t = med(a) + med(qq) + med(d);
    printf("%-20s %8.4f %8.4f %8.4f | %8.4f %6.3f\n", "int4 round trip", med(a), med(qq), med(d), t,
           13.0 * gb / (t * 1e-3) / 8000.0);
  }

  // ---- 3. dequantize-mean over K=8 gathered int8 rows (C4 epilogue shape)
  {
    const int K = 8;
    const int64_t m = n;
    for (int k = 1; k < K; ++k) CK(hipMemcpyAsync(q + k * m, q, m, hipMemcpyDeviceToDevice, st));
    std::vector<float> scales_h(K, 1e-3f);
    CK(hipMemcpy(scale, scales_h.data(), K * 4, hipMemcpyHostToDevice));
    std::vector<float> t;
    for (int s = 0; s < 20; ++s) {
      (void)hipEventRecord(ev[0], st);
      adfl_slq_dequantize_mean(q, m, K, m, scale, 1, out, st);
      (void)hipEventRecord(ev[1], st);
      CK(hipEventSynchronize(ev[1]));
      t.push_back(ms(ev[0], ev[1]));
    }
    const double bytes = (double)K * m + 4.0 * m;
    printf("%-20s %8.4f ms  %8.1f GB/s  (K=8 rows x %lld int8 -> fp32 mean)\n", "dequantize_mean", med(t),
           bytes / (med(t) * 1e-3) / 1e9, (long long)m);
  }

  // ---- 4. ceilings
  auto ceil = [&](const char* name, double bpe, std::function<void()> f) {
    std::vector<float> t;
    for (int s = 0; s < 30; ++s) {
      (void)hipEventRecord(ev[0], st);
      f();
      (void)hipEventRecord(ev[1], st);
      CK(hipEventSynchronize(ev[1]));
      t.push_back(ms(ev[0], ev[1]));
    }
    printf("%-20s %8.4f ms  %8.1f GB/s\n", name, med(t), bpe * gb / (med(t) * 1e-3));
  };
  ceil("copy_f32", 8, [&] { hipLaunchKernelGGL(mb::k_copy, dim3(2048), dim3(256), 0, st, (const float4*)x, (float4*)tmp, n >> 2); });
  ceil("read_f32", 4, [&] { hipLaunchKernelGGL(mb::k_read<false>, dim3(2048), dim3(256), 0, st, (const float4*)x, n >> 2, ws); });
  ceil("read_f32_nt", 4, [&] { hipLaunchKernelGGL(mb::k_read<true>, dim3(2048), dim3(256), 0, st, (const float4*)x, n >> 2, ws); });
  ceil("write_f32_nt", 4, [&] { hipLaunchKernelGGL(mb::k_write_nt, dim3(2048), dim3(256), 0, st, (float4*)tmp, n >> 2); });
  ceil("write_f32_nt_tiles", 4, [&] { hipLaunchKernelGGL(mb::k_write_nt_tiles, dim3(tg), dim3(256), 0, st, (float4*)tmp, n / kTile); });
  ceil("write_f32_nt_tiles_out", 4, [&] { hipLaunchKernelGGL(mb::k_write_nt_tiles, dim3(tg), dim3(256), 0, st, (float4*)out, n / kTile); });
  return 0;
}
