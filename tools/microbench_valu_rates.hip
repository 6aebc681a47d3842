// microbench_valu_rates.hip — VALU throughput of the instructions the stochastic codecs' Philox and
// element rules are made of, on gfx950: lane-operations per CU per clock for v_mad_u64_u32 (Philox's
// 32x32->64 products), v_mul_lo_u32 / v_mul_hi_u32, v_mul_u32_u24, v_xor_b32, v_add_f64 (the fp64 norm
// accumulation) and v_fma_f32 as the full-rate reference. 8 independent chains per lane, 2048 blocks of
// 256 threads; the clock is read from the kernel with s_memtime (wall clock / shader clock both printed).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench_valu_rates tools/microbench_valu_rates.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (hipError_t)(x);                                                         \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

constexpr int kChains = 8;
constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t seed, uint32_t* out) {
  uint32_t a[kChains];
  double d[kChains];
  float f[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    a[c] = seed + threadIdx.x * 7919u + c;
    d[c] = (double)a[c];
    f[c] = (float)a[c];
  }
  const uint32_t m = seed | 1u;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0) {  // v_mad_u64_u32: the 64-bit product's halves folded back into one word
        const uint64_t p = (uint64_t)a[c] * m;
        a[c] = (uint32_t)p + (uint32_t)(p >> 32);
      } else if (OP == 1) {
        a[c] = a[c] * m + 1u;  // v_mul_lo_u32 (+ add)
      } else if (OP == 2) {
        a[c] = __umulhi(a[c], m) ^ a[c];  // v_mul_hi_u32 (+ xor)
      } else if (OP == 3) {
        a[c] = __umul24(a[c] & 0xffffffu, m & 0xffffffu) + 1u;  // v_mul_u32_u24 (+ add)
      } else if (OP == 4) {
        a[c] = (a[c] ^ m) + 0x9e3779b9u;  // v_xor_b32 (+ add)
      } else if (OP == 5) {
        d[c] = d[c] + 1.25;  // v_add_f64
      } else {
        f[c] = __builtin_fmaf(f[c], 1.0000001f, 0.5f);  // v_fma_f32
      }
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r ^= a[c] ^ (uint32_t)d[c] ^ __float_as_uint(f[c]);
  if (r == 0x12345678u) out[0] = r;
}

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 64));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const char* names[] = {"v_mad_u64_u32 (+v_add)", "v_mul_lo_u32 (+v_add)", "v_mul_hi_u32 (+v_xor)",
                         "v_mul_u32_u24 (+v_add)", "v_xor_b32 (+v_add)", "v_add_f64", "v_fma_f32"};
  const int ops_per_step[] = {2, 2, 2, 2, 2, 1, 1};  // instructions per chain step (the op + its partner)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(2048), block(256);
  printf("CUs %d, clock %d MHz (device property), %d chains x %d steps per lane\n", cus, prop.clockRate / 1000, kChains,
         kIters);
  for (int op = 0; op < 7; ++op) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0));
      switch (op) {
        case 0: hipLaunchKernelGGL(k_rate<0>, grid, block, 0, 0, 3u, out); break;
        case 1: hipLaunchKernelGGL(k_rate<1>, grid, block, 0, 0, 3u, out); break;
        case 2: hipLaunchKernelGGL(k_rate<2>, grid, block, 0, 0, 3u, out); break;
        case 3: hipLaunchKernelGGL(k_rate<3>, grid, block, 0, 0, 3u, out); break;
        case 4: hipLaunchKernelGGL(k_rate<4>, grid, block, 0, 0, 3u, out); break;
        case 5: hipLaunchKernelGGL(k_rate<5>, grid, block, 0, 0, 3u, out); break;
        default: hipLaunchKernelGGL(k_rate<6>, grid, block, 0, 0, 3u, out); break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double steps = (double)grid.x * block.x * kChains * kIters;  // chain steps (lane level)
    const double steps_per_ns = steps / (best * 1e6);
    // lane-steps per CU per cycle at the property clock; a full-rate op alone would give 128 (4 SIMD-32)
    const double per_cu_clk = steps / (best * 1e-3) / cus / (prop.clockRate * 1e3);
    printf("  %-26s %8.3f ms  %8.1f G lane-steps/s  %6.1f lane-steps/CU/clk (%d instr per step)\n", names[op], best,
           steps_per_ns, per_cu_clk, ops_per_step[op]);
  }
  return 0;
}
