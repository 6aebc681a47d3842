// microbench_stoch.hip — ALU costs behind the stochastic quantize kernels, and an exhaustive-style check
// of the per-tensor-reciprocal division (Markstein: q = a*y, r = fma(-b, q, a), q' = fma(r, y, q) with
// y = RN(1/b)) against the correctly rounded __fdiv_rn.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/microbench_stoch tools/microbench_stoch.hip
//   tools/microbench_stoch            (prints one line per measurement)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                                        \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                      \
      return 2;                                                                                      \
    }                                                                                                \
  } while (0)

template <int R>
__device__ __forceinline__ uint4 philox(uint64_t ctr, uint64_t seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < R; ++r) {
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

// ALU throughput kernels: each thread does `iters` independent units and folds them into one word.
template <int R>
__global__ void k_philox_alu(uint32_t* out, int iters, uint64_t seed) {
  uint32_t acc = 0;
  const uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * iters;
  for (int i = 0; i < iters; ++i) {
    const uint4 w = philox<R>(base + i, seed);
    acc ^= w.x ^ w.y ^ w.z ^ w.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_div_alu(float* out, int iters, float b) {
  float acc = 0.f, a = 1.0f + threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
    acc += __fdiv_rn(a, b);
    a += 1.0f;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_mdiv_alu(float* out, int iters, float b, float y) {
  float acc = 0.f, a = 1.0f + threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    acc += __builtin_fmaf(r, y, q);
    a += 1.0f;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Division check: a, b from a hash (full fp32 significand range, exponents within +-20 of each other and
// away from over/underflow), plus b with all-ones / one-bit significands; counts q' != __fdiv_rn(a, b).
__device__ __forceinline__ uint32_t hash32(uint64_t i) {
  uint64_t h = i * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return (uint32_t)h;
}

__global__ void k_div_check(unsigned long long* bad, uint64_t n, uint64_t salt) {
  unsigned long long local = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h1 = hash32(i ^ salt), h2 = hash32(i * 3 + 1 + salt);
    const uint32_t mb = (i & 7) == 0 ? 0x7fffffu : (i & 7) == 1 ? (1u << (h2 % 23)) : (h2 & 0x7fffffu);
    const float b = __uint_as_float(((127u + (h2 >> 27)) << 23) | mb);                  // [1, 2^32)
    const float a = __uint_as_float(((107u + ((h1 >> 24) % 60u)) << 23) | (h1 & 0x7fffffu));  // [2^-20, 2^40)
    const float y = __fdiv_rn(1.0f, b);
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    const float m = __builtin_fmaf(r, y, q);
    local += (__float_as_uint(m) != __float_as_uint(__fdiv_rn(a, b)));
  }
  if (local) atomicAdd(bad, local);
}

int main() {
  uint32_t* d_u;
  float* d_f;
  unsigned long long* d_bad;
  const int blocks = 256 * 16, threads = 256, iters = 256;
  CK(hipMalloc(&d_u, (size_t)blocks * threads * 4));
  CK(hipMalloc(&d_f, (size_t)blocks * threads * 4));
  CK(hipMalloc(&d_bad, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double units = (double)blocks * threads * iters;
  auto timeit = [&](auto launch, const char* name, double per_unit_elems) -> int {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    const double per_s = units * per_unit_elems / (ms * 1e-3);
    // lane-cycles per element at 256 CUs x 4 SIMD x 16 lanes x 2.4 GHz = 39.3e12 lane-ops/s
    printf("%-22s %8.3f ms  %8.1f G elem/s  %6.2f lane-cycles/elem  (2^28 elems: %.3f ms)\n", name, ms,
           per_s / 1e9, 39.3e12 / per_s, (double)(1 << 28) / per_s * 1e3);
    return 0;
  };
  timeit([&] { hipLaunchKernelGGL(k_philox_alu<10>, dim3(blocks), dim3(threads), 0, 0, d_u, iters, 7ull); },
         "philox4x32-10", 4.0);
  timeit([&] { hipLaunchKernelGGL(k_philox_alu<7>, dim3(blocks), dim3(threads), 0, 0, d_u, iters, 7ull); },
         "philox4x32-7", 4.0);
  timeit([&] { hipLaunchKernelGGL(k_div_alu, dim3(blocks), dim3(threads), 0, 0, d_f, iters, 3.3f); }, "__fdiv_rn", 1.0);
  timeit([&] { hipLaunchKernelGGL(k_mdiv_alu, dim3(blocks), dim3(threads), 0, 0, d_f, iters, 3.3f, 1.f / 3.3f); },
         "reciprocal+fma div", 1.0);
  CK(hipMemset(d_bad, 0, 8));
  const uint64_t n = 1ull << 34;
  hipLaunchKernelGGL(k_div_check, dim3(8192), dim3(256), 0, 0, d_bad, n, 12345ull);
  CK(hipGetLastError());
  unsigned long long bad = 0;
  CK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
  printf("division check: %llu of %llu reciprocal+fma quotients differ from __fdiv_rn\n", bad, (unsigned long long)n);
  return 0;
}
