// microbench_stoch_bucket.hip — QSGD encode (norm partials -> finalize -> quantize) on the C3 bucket
// (11,689,512 fp32 in 256 tensors) and the C2 tensor (2^28 fp32): the product (norm pass keeps x's last
// 192 MiB in the Infinity Cache; one finalize launch) against an all-non-temporal norm pass, whole
// encodes and the norm pass alone. Interleaved variants inherit each other's cache state: the config
// bench (tools/bench_configs.py --mode stoch) is the arbiter (profiles/r01/stoch/keep_policy_ab.txt). Not part of the product; it #includes the
// product source to reach its kernels.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_stoch_bucket \
//         tools/microbench_stoch_bucket.hip ad-federatedlearning_amd/csrc/slq_codec.hip
#include "../ad-federatedlearning_amd/csrc/stoch_codec.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (hipError_t)(x);                                                         \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

namespace {
// Infinity-Cache flush by READING 512 MiB (clean junk lines; a write-based flush leaves dirty lines that
// drain during the next measurement)
__global__ void k_flush(const uint4* p, int64_t n) {
  uint32_t a = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a ^= p[i].x;
  if (a == 0x9e3779b9u) const_cast<uint4*>(p)[0].y = a;
}

// randn-like data (|x| ~ 1e-3) from a hash: the quantize pass takes its realistic branches
__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 4e-3f;
  }
}

// The product's norm pass with every load non-temporal (the product keeps the bucket's last 192 MiB
// in the Infinity Cache for the quantize pass), everything else as k_norm_partials.
__global__ __launch_bounds__(kBlock) void k_norm_nt(const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks,
                                                       void* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  const int head = chunk_head4(c.start, c.len);
  const float4* x4 = reinterpret_cast<const float4*>(xc + head);
  const int n4 = (c.len - head) >> 2;
  float4 v[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = threadIdx.x + j * kBlock;
    if (k < n4) v[j] = load4_nt(x4 + k);
  }
  NormAcc<ADFL_NORM_L2> acc;
  const int i = edge_elem(head, head + (n4 << 2), c.len);
  if (i >= 0) acc.add(xc[i]);
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if ((int)threadIdx.x + j * kBlock < n4) acc.add4(v[j]);
  acc.flush(partials, blockIdx.x);
}

int run(const char* label, const std::vector<int64_t>& sizes) {
  const int nt = (int)sizes.size();
  std::vector<int64_t> offs(nt);
  int64_t o = 0;
  for (int i = 0; i < nt; ++i) {
    offs[i] = o;
    o += (sizes[i] + 63) / 64 * 64;
  }
  const int64_t total = o;
  const int64_t nch = adfl_slq_build_chunks(offs.data(), sizes.data(), nt, nullptr, 0);
  std::vector<adfl_slq_chunk> ch(nch);
  adfl_slq_build_chunks(offs.data(), sizes.data(), nt, ch.data(), nch);
  float *x, *norms;
  uint8_t* lv;
  int8_t* sg;
  void* ws;
  adfl_slq_chunk* dch;
  uint4* junk;
  CK(hipMalloc(&x, total * 4));
  CK(hipMalloc(&lv, total));
  CK(hipMalloc(&sg, total));
  CK(hipMalloc(&norms, nt * 4));
  CK(hipMalloc(&ws, nch * kPartialBytes));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&junk, 512ll << 20));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, total);
  const Uniforms U{nullptr, 7, 0};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"product", "norm all-NT", "product norm only", "all-NT norm only"};
  const int nv = 4;
  std::vector<double> tot(nv, 0), totf(nv, 0);
  for (int rep = 0; rep < 42; ++rep)
    for (int v = 0; v < nv; ++v)
      for (int flush = 0; flush < 2; ++flush) {
        if (flush) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, (512ll << 20) / 16);
        CK(hipEventRecord(e0, 0));
        if (v == 0) {
          CK(adfl_qsgd_encode_batched(x, dch, nch, 8, nullptr, 7, 0, ws, nch * kPartialBytes, lv, sg, norms, nullptr));
        } else if (v == 1) {
          hipLaunchKernelGGL(k_norm_nt, dim3((unsigned)nch), dim3(kBlock), 0, 0, x, dch, ws);
          CK(launch_finalize<ADFL_NORM_L2>(dch, nch, ws, norms, nullptr, 0));
          CK(adfl_qsgd_quantize_batched(x, dch, nch, 8, norms, nullptr, 7, 0, lv, sg, nullptr));
        } else if (v == 2) {
          hipLaunchKernelGGL(k_norm_partials<ADFL_NORM_L2>, dim3((unsigned)nch), dim3(kBlock), 0, 0, x, dch,
                             nch - kKeepChunks, ws);
        } else {
          hipLaunchKernelGGL(k_norm_nt, dim3((unsigned)nch), dim3(kBlock), 0, 0, x, dch, ws);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep >= 2) (flush ? totf : tot)[v] += ms;
      }
  for (int v = 0; v < nv; ++v)
    printf("%-6s %-18s cached %.4f ms  flushed %.4f ms\n", label, names[v], tot[v] / 40, totf[v] / 40);
  CK(hipFree(x));
  CK(hipFree(lv));
  CK(hipFree(sg));
  CK(hipFree(norms));
  CK(hipFree(ws));
  CK(hipFree(dch));
  CK(hipFree(junk));
  return 0;
}
}  // namespace

int main() {
  std::vector<int64_t> c3(256);
  for (int i = 0; i < 256; ++i) c3[i] = 11689512 / 256 + (i < 11689512 % 256 ? 1 : 0);
  run("C3", c3);
  run("C2", {1ll << 28});
  return 0;
}
