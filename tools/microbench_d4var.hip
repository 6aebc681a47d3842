// microbench_d4var.hip — int4 unpack+dequantize variants against the int8 dequantize on one input (VERDICT
// r03 item 4: k_dequantize_int4_flat moved 0.93 of k_dequantize_flat's bytes per ms at 2^30). Interleaved
// rounds, each kernel after a 512 MiB read, medians; every variant's output checked against the product
// kernel's. Not part of the product; it #includes the product source.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_d4var tools/microbench_d4var.hip
//   ./tools/microbench_d4var [log2_elems=30] [rounds=11]
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
// 1024-element int4 tiles: one 8-byte packed load per lane (512 B per wave), a 512 B LDS transpose, and the
// int8 decode's store shape (4 coalesced NT float4 stores per lane).
__global__ __launch_bounds__(kBlock) void k_d4_half(const uint8_t* __restrict__ packed, int64_t n,
                                                    const float* __restrict__ scale_p, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile / 4];
  const float s = *scale_p;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint2* p8 = reinterpret_cast<const uint2*>(packed);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ntiles = n / kTile;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < ntiles; t += wstride) {
    reinterpret_cast<uint2*>(lds[wave])[lane] = p8[t * 64 + lane];
    __builtin_amdgcn_wave_barrier();
    uint32_t h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = lds[wave][j * 64 + lane];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j) store4_nt(o4 + t * (kTile / 4) + j * 64 + lane, dequant2_int4(h[j], s));
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile + threadIdx.x; i < n; i += kBlock) {
      float e0, e1;
      dequant_byte_int4(packed[i >> 1], s, e0, e1);
      out[i] = (i & 1) ? e1 : e0;
    }
}

// the product's 2048-element tile with its 8 stores issued as two groups of 4 around the second half's
// LDS reads (a shorter store burst per wave)
__global__ __launch_bounds__(kBlock) void k_d4_split(const uint8_t* __restrict__ packed, int64_t n,
                                                     const float* __restrict__ scale_p, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kWaves][kTile4 / 4];
  const float s = *scale_p;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint4* p16 = reinterpret_cast<const uint4*>(packed);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int64_t ntiles = n / kTile4;
  const int64_t wstride = (int64_t)gridDim.x * kWaves;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < ntiles; t += wstride) {
    reinterpret_cast<uint4*>(lds[wave])[lane] = p16[t * 64 + lane];
    __builtin_amdgcn_wave_barrier();
    uint32_t h[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = lds[wave][j * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) store4_nt(o4 + t * (kTile4 / 4) + j * 64 + lane, dequant2_int4(h[j], s));
#pragma unroll
    for (int j = 4; j < 8; ++j) h[j] = lds[wave][j * 64 + lane];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 4; j < 8; ++j) store4_nt(o4 + t * (kTile4 / 4) + j * 64 + lane, dequant2_int4(h[j], s));
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t i = ntiles * kTile4 + threadIdx.x; i < n; i += kBlock) {
      float e0, e1;
      dequant_byte_int4(packed[i >> 1], s, e0, e1);
      out[i] = (i & 1) ? e1 : e0;
    }
}
}  // namespace mb

__global__ void k_fill(float* x, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    x[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 2e-3f;
  }
}

__global__ void k_touch(const float4* __restrict__ a, int64_t n4, float* __restrict__ sink) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) *sink = s;
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const int rounds = argc > 2 ? atoi(argv[2]) : 11;
  const int64_t n = (int64_t)1 << lg;
  float *x, *out, *out_ref, *s8, *s4;
  int8_t* q8;
  uint8_t* p4;
  uint32_t *ws, *jpart;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&out_ref, n * 4));
  CK(hipMalloc(&q8, n));
  CK(hipMalloc(&p4, n / 2));
  CK(hipMalloc(&ws, kWorkspaceBytes));
  CK(hipMalloc(&jpart, kWorkspaceBytes));
  CK(hipMalloc(&s8, 16));
  CK(hipMalloc(&s4, 16));
  float* junk;
  const int64_t njunk = (int64_t)128 << 20;
  CK(hipMalloc(&junk, njunk * 4));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n, 12345u);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, junk, njunk, 777u);
  hipLaunchKernelGGL(k_absmax_flat<8>, dim3(absmax_grid(n)), dim3(kBlock), 0, 0, x, n, (int64_t)0, ws);
  hipLaunchKernelGGL((k_quantize_flat<true, false>), dim3(tile_grid(n / kTile)), dim3(kBlock), 0, 0, x, n, qmax_f(8),
                     ws, q8, s8);
  hipLaunchKernelGGL(k_quantize_int4_flat, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, 0, x, n, qmax_f(4), ws, p4,
                     s4);
  hipLaunchKernelGGL(k_dequantize_int4_flat, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, 0, p4, n, s4, out_ref);
  CK(hipDeviceSynchronize());
  struct V {
    std::string name;
    double bpe;
    bool int4;
    std::function<void()> launch;
  };
  const int g8 = tile_grid(n / kTile), g4 = tile_grid(n / kTile4);
  std::vector<V> vs = {
      {"int8 product", 5.0, false, [&] { hipLaunchKernelGGL((k_dequantize_flat<false, false>), dim3(g8), dim3(kBlock), 0, 0, q8, n, s8, out); }},
      {"int4 product", 4.5, true, [&] { hipLaunchKernelGGL(k_dequantize_int4_flat, dim3(g4), dim3(kBlock), 0, 0, p4, n, s4, out); }},
      {"int4 product grid1024", 4.5, true, [&] { hipLaunchKernelGGL(k_dequantize_int4_flat, dim3(1024), dim3(kBlock), 0, 0, p4, n, s4, out); }},
      {"int4 half tiles", 4.5, true, [&] { hipLaunchKernelGGL(mb::k_d4_half, dim3(g8), dim3(kBlock), 0, 0, p4, n, s4, out); }},
      {"int4 split stores", 4.5, true, [&] { hipLaunchKernelGGL(mb::k_d4_split, dim3(g4), dim3(kBlock), 0, 0, p4, n, s4, out); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> t(vs.size());
  std::vector<int> ok(vs.size(), 1);
  std::vector<float> a(n), b(n);
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      if (r == 0) CK(hipMemset(out, 0x7f, n * 4));
      hipLaunchKernelGGL(k_touch, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const float4*>(junk), njunk / 4,
                         reinterpret_cast<float*>(jpart));
      CK(hipEventRecord(e0, 0));
      vs[i].launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms);
      if (r == 0 && vs[i].int4) {
        CK(hipMemcpy(a.data(), out, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), out_ref, n * 4, hipMemcpyDeviceToHost));
        ok[i] = memcmp(a.data(), b.data(), n * 4) == 0;
      }
    }
  printf("n = 2^%d, %d interleaved rounds, each after a 512 MiB read; median ms (min); TB/s on the bytes moved\n", lg,
         rounds);
  const double base = 5.0 / med(t[0]);
  for (size_t i = 0; i < vs.size(); ++i) {
    const double m = med(t[i]);
    printf("%-24s %.4f (%.4f)  %.1f B/elem  %.3f TB/s  frac %.4f  per-byte vs int8 %.3f  %s\n", vs[i].name.c_str(), m,
           *std::min_element(t[i].begin(), t[i].end()), vs[i].bpe, vs[i].bpe * n / (m * 1e-3) / 1e12,
           vs[i].bpe * n / (m * 1e-3) / 8e12, (vs[i].bpe / m) / base, ok[i] ? "ok" : "MISMATCH");
  }
  return 0;
}
