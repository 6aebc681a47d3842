// microbench_c5.hip — int4 quantize+pack variants on the C5 workload (2^30 fp32, 512 MiB packed payload,
// twice the 256 MiB Infinity Cache), interleaved rounds, medians; each variant's payload checked against
// the product kernel's. Not part of the product; it #includes the product source to reach its kernels.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_c5 tools/microbench_c5.hip
//   ./tools/microbench_c5 [log2_elems=30]
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
// k_quantize_int4_flat with the knobs: REVERSE tile order, ST_NT payload stores, PF = next tile's loads
// issued before the current tile is quantized (two register sets).
template <bool REVERSE, bool ST_NT, bool PF>
__global__ __launch_bounds__(kBlock) void k_q4(const float* __restrict__ x, int64_t n, float qmax,
                                               const uint32_t* __restrict__ partials, uint8_t* __restrict__ packed,
                                               float* __restrict__ scale_out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  uint4* p16 = reinterpret_cast<uint4*>(packed);
  const int64_t ntiles = n / kTile4;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  const int64_t first = (int64_t)blockIdx.x * kWaves + wave;
  auto tix = [&](int64_t t0) { return REVERSE ? ntiles - 1 - t0 : t0; };
  float4 v[8], w[8];
  if (first < ntiles) load_tile_int4(x4 + tix(first) * (kTile4 / 4), v, lane);
  const ScaleInv si = make_scale(reduce_partials(partials, (int)partials[kCountSlot]), qmax);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = si.scale;
  for (int64_t t0 = first; t0 < ntiles; t0 += wstride) {
    if (PF) {
      if (t0 + wstride < ntiles) load_tile_int4(x4 + tix(t0 + wstride) * (kTile4 / 4), w, lane);
    } else if (t0 != first) {
      load_tile_int4(x4 + tix(t0) * (kTile4 / 4), v, lane);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[wave][j * 64 + lane] = (uint16_t)quant4_int4(v[j], si.inv);
    __builtin_amdgcn_wave_barrier();
    const uint4 o = reinterpret_cast<const uint4*>(lds[wave])[lane];
    __builtin_amdgcn_wave_barrier();
    store16<ST_NT>(p16 + tix(t0) * 64 + lane, o);
    if (PF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = w[j];
    }
  }
}
}  // namespace mb

static float med(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int64_t n = 1LL << lg;
  float *x, *out, *scale;
  uint8_t *p, *pref;
  uint32_t* ws;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&p, n / 2));
  CK(hipMalloc(&pref, n / 2));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&ws, 16384));
  CK(hipMalloc(&scale, 64));
  {
    std::vector<float> h(1 << 20);
    uint32_t s = 12345;
    for (auto& v : h) {
      s = s * 1664525u + 1013904223u;
      v = ((int)(s >> 8) - (1 << 23)) * 1e-9f;
    }
    for (int64_t o = 0; o < n; o += h.size())
      CK(hipMemcpy(x + o, h.data(), std::min<int64_t>(h.size(), n - o) * 4, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t ev[4];
  for (auto& e : ev) CK(hipEventCreate(&e));
  auto ms = [&](hipEvent_t a, hipEvent_t b) {
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    return t;
  };
  const int tg = tile_grid(n / kTile4);
  using L = std::function<void(int)>;
  struct V {
    std::string name;
    L fn;
  };
  std::vector<V> Q = {
      {"prod (rev, alloc)", [&](int g) { hipLaunchKernelGGL(k_quantize_int4_flat, dim3(g), dim3(kBlock), 0, st, x, n, 7.f, ws, p, scale); }},
      {"rev, nt", [&](int g) { hipLaunchKernelGGL((mb::k_q4<true, true, false>), dim3(g), dim3(kBlock), 0, st, x, n, 7.f, ws, p, scale); }},
      {"fwd, alloc", [&](int g) { hipLaunchKernelGGL((mb::k_q4<false, false, false>), dim3(g), dim3(kBlock), 0, st, x, n, 7.f, ws, p, scale); }},
      {"fwd, nt", [&](int g) { hipLaunchKernelGGL((mb::k_q4<false, true, false>), dim3(g), dim3(kBlock), 0, st, x, n, 7.f, ws, p, scale); }},
      {"rev, alloc, pf", [&](int g) { hipLaunchKernelGGL((mb::k_q4<true, false, true>), dim3(g), dim3(kBlock), 0, st, x, n, 7.f, ws, p, scale); }},
      {"rev, nt, pf", [&](int g) { hipLaunchKernelGGL((mb::k_q4<true, true, true>), dim3(g), dim3(kBlock), 0, st, x, n, 7.f, ws, p, scale); }},
  };
  const int grids[] = {tg, 1024};
  // reference payload
  adfl_slq_absmax(x, n, ws, 16384, st);
  adfl_slq_quantize_int4(x, n, 4, ws, pref, scale, st);
  CK(hipStreamSynchronize(st));
  std::vector<uint8_t> href(n / 2), hp(n / 2);
  CK(hipMemcpy(href.data(), pref, n / 2, hipMemcpyDeviceToHost));
  printf("n = 2^%d, product grid %d; quantize+pack ms (median of 15 interleaved rounds), then decode after it\n", lg, tg);
  printf("%-22s %6s %-5s %9s %9s %9s %7s %s\n", "variant", "grid", "steps", "absmax", "quant4", "deq4", "frac13", "check");
  for (int g : grids) {
    for (auto& q : Q) {
      CK(hipMemset(p, 0, n / 2));
      adfl_slq_absmax(x, n, ws, 16384, st);
      q.fn(g);
      CK(hipStreamSynchronize(st));
      CK(hipGetLastError());
      CK(hipMemcpy(hp.data(), p, n / 2, hipMemcpyDeviceToHost));
      const bool ok = hp == href;
      for (int mode = 0; mode < 2; ++mode) {  // 0: host sync after every round; 1: rounds back to back
        std::vector<float> a, qq, d;
        const int R = 15;
        std::vector<hipEvent_t> E(4 * R);
        for (auto& e : E) CK(hipEventCreate(&e));
        for (int r = 0; r < R; ++r) {
          hipEvent_t* e = &E[4 * r];
          (void)hipEventRecord(e[0], st);
          adfl_slq_absmax(x, n, ws, 16384, st);
          (void)hipEventRecord(e[1], st);
          q.fn(g);
          (void)hipEventRecord(e[2], st);
          adfl_slq_dequantize_int4(p, n, scale, out, st);
          (void)hipEventRecord(e[3], st);
          if (mode == 0) CK(hipEventSynchronize(e[3]));
        }
        CK(hipStreamSynchronize(st));
        for (int r = 0; r < R; ++r) {
          hipEvent_t* e = &E[4 * r];
          a.push_back(ms(e[0], e[1]));
          qq.push_back(ms(e[1], e[2]));
          d.push_back(ms(e[2], e[3]));
        }
        for (auto& e : E) CK(hipEventDestroy(e));
        const float t = med(a) + med(qq) + med(d);
        printf("%-22s %6d %-5s %9.4f %9.4f %9.4f %7.3f %s\n", q.name.c_str(), g, mode ? "b2b" : "sync", med(a),
               med(qq), med(d), 13.0 * n / (t * 1e-3) / 8e12, ok ? "ok" : "MISMATCH");
      }
    }
  }
  return 0;
}
