// microbench_q8q4.hip — VERDICT r03 item 4: the product's int8 and int4 flat kernels on ONE 2^30-element
// fp32 input in one process, back to back, so the int4 quantize+pack / unpack+dequantize can be compared per
// byte with the int8 quantize / dequantize on the same box (and, under rocprofv3 --pmc, counter by counter).
// Not part of the product; it #includes the product source to launch exactly its kernels and grids.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_q8q4 tools/microbench_q8q4.hip
//   ./tools/microbench_q8q4 [log2_elems=30] [rounds=15]
#include "../ad-federatedlearning_amd/csrc/slq_codec.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

__global__ void k_fill(float* x, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    x[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 2e-3f;
  }
}

// a plain (allocating) 512 MiB read: the Infinity Cache then holds clean junk lines
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
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  const int64_t n = (int64_t)1 << lg;
  float *x, *out, *scale8, *scale4;
  int8_t* q8;
  uint8_t* p4;
  uint32_t* ws;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&q8, n));
  CK(hipMalloc(&p4, (n + 1) / 2));
  CK(hipMalloc(&ws, kWorkspaceBytes));
  CK(hipMalloc(&scale8, 16));
  CK(hipMalloc(&scale4, 16));
  float* junk;
  const int64_t njunk = (int64_t)128 << 20;  // 512 MiB read between kernels: nothing of the last one on-die
  CK(hipMalloc(&junk, njunk * 4));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n, 12345u);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, junk, njunk, 777u);
  uint32_t* jpart;
  CK(hipMalloc(&jpart, kWorkspaceBytes));
  hipLaunchKernelGGL(k_absmax_flat<8>, dim3(absmax_grid(n)), dim3(kBlock), 0, 0, x, n, (int64_t)0, ws);
  CK(hipDeviceSynchronize());

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto flush = [&]() {
    hipLaunchKernelGGL(k_touch, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const float4*>(junk), njunk / 4,
                       reinterpret_cast<float*>(jpart));
  };
  auto timed = [&](auto launch) {
    flush();
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return (double)ms;
  };
  const float q8max = qmax_f(8), q4max = qmax_f(4);
  auto q8k = [&]() {
    hipLaunchKernelGGL((k_quantize_flat<true, false>), dim3(tile_grid(n / kTile)), dim3(kBlock), 0, 0, x, n, q8max,
                       ws, q8, scale8);
  };
  auto q4k = [&]() {
    hipLaunchKernelGGL(k_quantize_int4_flat, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, 0, x, n, q4max, ws, p4,
                       scale4);
  };
  auto d8k = [&]() {
    hipLaunchKernelGGL((k_dequantize_flat<false, false>), dim3(tile_grid(n / kTile)), dim3(kBlock), 0, 0, q8, n,
                       scale8, out);
  };
  auto d4k = [&]() {
    hipLaunchKernelGGL(k_dequantize_int4_flat, dim3(tile_grid(n / kTile4)), dim3(kBlock), 0, 0, p4, n, scale4, out);
  };
  std::vector<double> tq8, tq4, td8, td4;
  for (int r = 0; r < rounds; ++r) {  // interleaved, every kernel behind a 512 MiB read
    tq8.push_back(timed(q8k));
    tq4.push_back(timed(q4k));
    td8.push_back(timed(d8k));
    td4.push_back(timed(d4k));
  }
  CK(hipDeviceSynchronize());
  const double N = (double)n;
  auto row = [&](const char* name, const std::vector<double>& t, double bytes_per_elem, int grid) {
    const double m = med(t);
    printf("%-22s grid %5d  median %.4f ms  min %.4f  max %.4f  %.1f B/elem  %.3f TB/s  frac %.4f\n", name, grid, m,
           *std::min_element(t.begin(), t.end()), *std::max_element(t.begin(), t.end()), bytes_per_elem,
           bytes_per_elem * N / (m * 1e-3) / 1e12, bytes_per_elem * N / (m * 1e-3) / 8e12);
  };
  printf("n = 2^%d, %d interleaved rounds, each kernel after a 512 MiB read (Infinity Cache holds none of it)\n", lg,
         rounds);
  row("k_quantize_flat", tq8, 5.0, tile_grid(n / kTile));
  row("k_quantize_int4_flat", tq4, 4.5, tile_grid(n / kTile4));
  row("k_dequantize_flat", td8, 5.0, tile_grid(n / kTile));
  row("k_dequantize_int4_flat", td4, 4.5, tile_grid(n / kTile4));
  printf("per-byte ratio int4/int8: quantize %.3f  dequantize %.3f (1.000 = same bytes per ms)\n",
         (4.5 / med(tq4)) / (5.0 / med(tq8)), (4.5 / med(td4)) / (5.0 / med(td8)));
  return 0;
}
