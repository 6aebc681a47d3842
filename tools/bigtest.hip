// bigtest.hip — the codec past 32-bit element counts (2^31 + 37 fp32 = 8 GiB), with no torch in the
// process: buffers from hipMalloc, data from a deterministic fill kernel, checks on sampled spans on
// the host. Run by tests/test_gpu_large.py as a subprocess.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/bigtest tools/bigtest.hip
#include "../ad-federatedlearning_amd/csrc/slq_codec.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 2;                                                                              \
    }                                                                                        \
  } while (0)

// value(i): a hash of i mapped to [-1, 1); element `peak` is 7.5 (the absmax)
__host__ __device__ inline float value_at(int64_t i, int64_t peak) {
  if (i == peak) return 7.5f;
  uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return (float)((int32_t)(h & 0xffffffu) - (1 << 23)) * (1.0f / (1 << 23));
}

__global__ void k_fill(float* x, int64_t n, int64_t peak) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = value_at(i, peak);
}

static int quant_ref(float x, float inv) {
  float y = x * inv;
  if (std::isnan(y)) return 127;
  y = std::fmin(std::fmax(y, -128.f), 127.f);
  return (int)std::nearbyint(y);
}

int main() {
  const int64_t n = (1ll << 31) + 37, peak = n - 3;
  float *x, *out, *scale;
  int8_t* q;
  uint8_t* p;
  void* ws;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&q, n));
  CK(hipMalloc(&p, (n + 1) / 2));
  CK(hipMalloc(&scale, 64));
  CK(hipMalloc(&ws, adfl_slq_workspace_bytes()));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n, peak);
  CK(hipGetLastError());
  int rc = adfl_slq_encode(x, n, 8, q, scale, ws, adfl_slq_workspace_bytes(), nullptr);
  if (!rc) rc = adfl_slq_dequantize(q, n, scale, out, nullptr);
  if (rc) {
    fprintf(stderr, "codec error %d %s\n", rc, adfl_slq_strerror(rc));
    return 2;
  }
  CK(hipDeviceSynchronize());
  printf("int8 round trip done\n");
  fflush(stdout);
  float s;
  CK(hipMemcpy(&s, scale, 4, hipMemcpyDeviceToHost));
  const float s_ref = 7.5f / 127.f, inv = 1.f / s_ref;
  int bad = (s != s_ref);
  // the last span straddles element 2^31 and ends at n (the buffer end)
  const int64_t spans[3][2] = {{0, 8192}, {1ll << 30, (1ll << 30) + 8192}, {n - 16384, n}};
  std::vector<int8_t> qh(16384);
  std::vector<float> oh(16384);
  for (auto& sp : spans) {
    const int64_t len = sp[1] - sp[0];
    CK(hipMemcpy(qh.data(), q + sp[0], len, hipMemcpyDeviceToHost));
    CK(hipMemcpy(oh.data(), out + sp[0], len * 4, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < len; ++k) {
      const int want = quant_ref(value_at(sp[0] + k, peak), inv);
      bad += (qh[k] != want) + (oh[k] != s_ref * (float)want);
    }
  }
  // int4 path over the same buffer
  rc = adfl_slq_encode_int4(x, n, 4, p, scale, ws, adfl_slq_workspace_bytes(), nullptr);
  if (!rc) rc = adfl_slq_dequantize_int4(p, n, scale, out, nullptr);
  if (rc) {
    fprintf(stderr, "codec error %d %s\n", rc, adfl_slq_strerror(rc));
    return 2;
  }
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(&s, scale, 4, hipMemcpyDeviceToHost));
  const float s4 = 7.5f / 7.f, inv4 = 1.f / s4;
  bad += (s != s4);
  for (auto& sp : spans) {
    const int64_t len = sp[1] - sp[0];
    CK(hipMemcpy(oh.data(), out + sp[0], len * 4, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < len; ++k) bad += (oh[k] != s4 * (float)quant_ref(value_at(sp[0] + k, peak), inv4));
  }
  printf("bigtest n=%lld mismatches=%d\n", (long long)n, bad);
  return bad ? 1 : 0;
}
