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

  // ---- 1. KEEP sweep on the int8 round trip (absmax -> quantize -> dequantize)
  std::vector<int64_t> keeps = {0, 64ll << 20, 128ll << 20, 192ll << 20, 256ll << 20, n * 4};
  struct Row { std::string name; std::vector<float> a, q, d; };
  std::vector<Row> rows;
  for (auto k : keeps) rows.push_back({"keep=" + std::to_string(k >> 20) + "MiB", {}, {}, {}});
  const int ROUNDS = 6, STEPS = 8;
  for (int r = 0; r < ROUNDS; ++r)
    for (size_t i = 0; i < keeps.size(); ++i)
      for (int s = 0; s < STEPS; ++s) {
        (void)hipEventRecord(ev[0], st);
        hipLaunchKernelGGL(k_absmax_flat, dim3(absmax_grid(n)), dim3(kBlock), 0, st, x, n, keeps[i] / 16, ws);
        (void)hipEventRecord(ev[1], st);
        adfl_slq_quantize(x, n, 8, ws, q, scale, st);
        (void)hipEventRecord(ev[2], st);
        adfl_slq_dequantize(q, n, scale, out, st);
        (void)hipEventRecord(ev[3], st);
        CK(hipEventSynchronize(ev[3]));
        rows[i].a.push_back(ms(ev[0], ev[1]));
        rows[i].q.push_back(ms(ev[1], ev[2]));
        rows[i].d.push_back(ms(ev[2], ev[3]));
      }
  printf("%-20s %8s %8s %8s | %8s %6s\n", "int8 round trip", "absmax", "quant", "deq", "sum ms", "frac");
  for (auto& R : rows) {
    const float t = med(R.a) + med(R.q) + med(R.d);
    printf("%-20s %8.4f %8.4f %8.4f | %8.4f %6.3f\n", R.name.c_str(), med(R.a), med(R.q), med(R.d), t,
           14.0 * gb / (t * 1e-3) / 8000.0);
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
  return 0;
}
