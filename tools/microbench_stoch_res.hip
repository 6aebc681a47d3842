// microbench_stoch_res.hip — the stochastic encodes on the C3 bucket (11,689,512 fp32 in 256 tensors, every
// tensor resident) and the C2 tensor (2^28 fp32): the product encodes (one-launch resident and multi-launch;
// QSGD, RQSGD, CNAT), their passes, the SLQ resident encode as the data-movement reference, and the quantize
// kernels at Philox batch sizes PB = 1, 2, 4, 8 (philox4x32_batch). Not part of the product; it #includes
// the product source to reach its kernels.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_stoch_res \
//         tools/microbench_stoch_res.hip ad-federatedlearning_amd/csrc/slq_codec.hip
#include "../ad-federatedlearning_amd/csrc/stoch_codec.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
__global__ void k_flush(const uint4* p, int64_t n) {
  uint32_t a = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a ^= p[i].x;
  if (a == 0x9e3779b9u) const_cast<uint4*>(p)[0].y = a;
}

__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 4e-3f;
  }
}

int g_reps = 30;

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
  const int64_t nwork = adfl_slq_build_encode_work(ch.data(), nch, nullptr, 0);
  std::vector<int32_t> wk(nwork > 0 ? nwork : 1);
  adfl_slq_build_encode_work(ch.data(), nch, wk.data(), nwork);
  float *x, *norms, *scales;
  uint8_t* lv;
  int8_t *sg, *q;
  void* ws;
  adfl_slq_chunk* dch;
  int32_t* dwk;
  uint4* junk;
  CK(hipMalloc(&x, total * 4));
  CK(hipMalloc(&lv, total));
  CK(hipMalloc(&sg, total));
  CK(hipMalloc(&q, total));
  CK(hipMalloc(&norms, nt * 4));
  CK(hipMalloc(&scales, nt * 4));
  CK(hipMalloc(&ws, nch * kPartialBytes));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&dwk, wk.size() * sizeof(int32_t)));
  CK(hipMalloc(&junk, 512ll << 20));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  CK(hipMemcpy(dwk, wk.data(), wk.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, total);
  const Uniforms U{nullptr, 7, 0};
  const int64_t wsb = nch * kPartialBytes;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float* mins;
  CK(hipMalloc(&mins, nt * 4));
  const bool res = nwork > 0;
  const char* names[] = {"qsgd multi-launch", "qsgd resident", "rqsgd multi-launch", "rqsgd resident",
                         "cnat multi-launch", "cnat resident", "qsgd norm pass (2 launches)",
                         "slq resident/two-pass encode", "qsgd quantize PB1", "qsgd quantize PB2", "qsgd quantize PB4",
                         "qsgd quantize PB8", "cnat quantize PB1", "cnat quantize PB2", "cnat quantize PB4",
                         "cnat quantize PB8", "qsgd resident late signs", "qsgd resident early signs", "cnat resident PB1",
                         "cnat resident PB2"};
  const int nv = sizeof(names) / sizeof(names[0]);
  const int reps = g_reps;
  const dim3 gq((unsigned)nch), bq(kBlock), gr((unsigned)(res ? nwork : 1)), br(kResBlock);
  std::vector<std::vector<float>> t(nv * 2);
  for (int rep = 0; rep < reps + 2; ++rep)
    for (int v = 0; v < nv; ++v)
      for (int flush = 0; flush < 2; ++flush) {
        if (!res && (v == 1 || v == 3 || v == 5 || v >= 16)) continue;
        if (flush) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, (512ll << 20) / 16);
        CK(hipEventRecord(e0, 0));
        switch (v) {
          case 0: CK(adfl_qsgd_encode_batched_work(x, dch, nch, dwk, 0, 8, nullptr, 7, 0, ws, wsb, lv, sg, norms, 0)); break;
          case 1: CK(adfl_qsgd_encode_batched_work(x, dch, nch, dwk, nwork, 8, nullptr, 7, 0, ws, wsb, lv, sg, norms, 0)); break;
          case 2: CK(adfl_rqsgd_encode_batched_work(x, dch, nch, dwk, 0, 8, nullptr, 7, 0, ws, wsb, lv, sg, norms, mins, 0)); break;
          case 3: CK(adfl_rqsgd_encode_batched_work(x, dch, nch, dwk, nwork, 8, nullptr, 7, 0, ws, wsb, lv, sg, norms, mins, 0)); break;
          case 4: CK(adfl_cnat_encode_batched_work(x, dch, nch, dwk, 0, 8, nullptr, 7, 0, ws, wsb, sg, q, norms, 0)); break;
          case 5: CK(adfl_cnat_encode_batched_work(x, dch, nch, dwk, nwork, 8, nullptr, 7, 0, ws, wsb, sg, q, norms, 0)); break;
          case 6: CK(adfl_stoch_norms_batched(x, dch, nch, ADFL_NORM_L2, ws, wsb, norms, nullptr, 0)); break;
          case 7: CK(adfl_slq_encode_batched_work(x, dch, nch, dwk, res ? nwork : 0, 8, q, scales, (uint32_t*)ws, 0)); break;
          case 8: hipLaunchKernelGGL(k_qsgd_quantize<1>, gq, bq, 0, 0, x, dch, 255.0f, norms, U, lv, sg); break;
          case 9: hipLaunchKernelGGL(k_qsgd_quantize<2>, gq, bq, 0, 0, x, dch, 255.0f, norms, U, lv, sg); break;
          case 10: hipLaunchKernelGGL(k_qsgd_quantize<4>, gq, bq, 0, 0, x, dch, 255.0f, norms, U, lv, sg); break;
          case 11: hipLaunchKernelGGL(k_qsgd_quantize<8>, gq, bq, 0, 0, x, dch, 255.0f, norms, U, lv, sg); break;
          case 12: hipLaunchKernelGGL(k_cnat_quantize<1>, gq, bq, 0, 0, x, dch, -128, 127, U, sg, q, (double*)ws); break;
          case 13: hipLaunchKernelGGL(k_cnat_quantize<2>, gq, bq, 0, 0, x, dch, -128, 127, U, sg, q, (double*)ws); break;
          case 14: hipLaunchKernelGGL(k_cnat_quantize<4>, gq, bq, 0, 0, x, dch, -128, 127, U, sg, q, (double*)ws); break;
          case 15: hipLaunchKernelGGL(k_cnat_quantize<8>, gq, bq, 0, 0, x, dch, -128, 127, U, sg, q, (double*)ws); break;
          case 16: hipLaunchKernelGGL((k_qsgd_encode_resident<ADFL_NORM_L2, 2, false>), gr, br, 0, 0, x, dch, dwk, 255.0f, U, lv, sg, norms, mins); break;
          case 17: hipLaunchKernelGGL((k_qsgd_encode_resident<ADFL_NORM_L2, 2, true>), gr, br, 0, 0, x, dch, dwk, 255.0f, U, lv, sg, norms, mins); break;
          case 18: hipLaunchKernelGGL(k_cnat_encode_resident<1>, gr, br, 0, 0, x, dch, dwk, -128, 127, U, sg, q, norms); break;
          default: hipLaunchKernelGGL(k_cnat_encode_resident<2>, gr, br, 0, 0, x, dch, dwk, -128, 127, U, sg, q, norms); break;
        }
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep >= 2) t[v * 2 + flush].push_back(ms);
      }
  printf("%s: %lld elements, %d tensors, %lld chunks, %lld resident blocks\n", label, (long long)total, nt,
         (long long)nch, (long long)nwork);
  for (int v = 0; v < nv; ++v) {
    if (t[v * 2].empty()) continue;
    double med[2];
    for (int f = 0; f < 2; ++f) {
      auto& a = t[v * 2 + f];
      std::sort(a.begin(), a.end());
      med[f] = a[a.size() / 2] * 1e3;
    }
    printf("  %-30s warm %7.2f us   flushed %7.2f us   (6 B/elem moved: %.3f of 8 TB/s)\n", names[v], med[0], med[1],
           6.0 * total / (med[1] * 1e-6) / 8e12);
  }
  CK(hipFree(x));
  CK(hipFree(lv));
  CK(hipFree(sg));
  CK(hipFree(q));
  CK(hipFree(norms));
  CK(hipFree(scales));
  CK(hipFree(ws));
  CK(hipFree(dch));
  CK(hipFree(dwk));
  CK(hipFree(junk));
  CK(hipFree(mins));
  return 0;
}
}  // namespace

// The quantize kernels on the C3 bucket with chunk tables of smaller chunks (8192 / 4096 / 2048 elements):
// more, shorter blocks, so the load and compute phases of different blocks can overlap.
int run_chunk_sizes() {
  const int nt = 256;
  std::vector<int64_t> sizes(nt), offs(nt);
  int64_t o = 0;
  for (int i = 0; i < nt; ++i) {
    sizes[i] = 11689512 / 256 + (i < 11689512 % 256 ? 1 : 0);
    offs[i] = o;
    o += (sizes[i] + 63) / 64 * 64;
  }
  const int64_t total = o;
  float *x, *norms;
  uint8_t* lv;
  int8_t *sg, *q;
  void* ws;
  uint4* junk;
  CK(hipMalloc(&x, total * 4));
  CK(hipMalloc(&lv, total));
  CK(hipMalloc(&sg, total));
  CK(hipMalloc(&q, total));
  CK(hipMalloc(&norms, nt * 4));
  CK(hipMalloc(&ws, 8192 * kPartialBytes));
  CK(hipMalloc(&junk, 512ll << 20));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, total);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, norms, nt);
  const Uniforms U{nullptr, 7, 0};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("C3 quantize kernels by chunk size (flushed, median of %d)\n", g_reps);
  for (int cs : {8192, 4096, 2048}) {
    std::vector<adfl_slq_chunk> ch;
    for (int t = 0; t < nt; ++t) {
      const int first = (int)ch.size(), nc = (int)((sizes[t] + cs - 1) / cs);
      for (int k = 0; k < nc; ++k)
        ch.push_back({offs[t] + (int64_t)k * cs, (int32_t)std::min<int64_t>(cs, sizes[t] - (int64_t)k * cs), t, first, nc});
    }
    adfl_slq_chunk* dch;
    CK(hipMalloc(&dch, ch.size() * sizeof(adfl_slq_chunk)));
    CK(hipMemcpy(dch, ch.data(), ch.size() * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
    for (int v = 0; v < 2; ++v) {
      std::vector<float> ts;
      for (int rep = 0; rep < g_reps + 2; ++rep) {
        hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, (512ll << 20) / 16);
        CK(hipEventRecord(e0, 0));
        if (v == 0)
          hipLaunchKernelGGL(k_cnat_quantize<4>, dim3((unsigned)ch.size()), dim3(kBlock), 0, 0, x, dch, -128, 127, U, sg, q,
                             (double*)ws);
        else
          hipLaunchKernelGGL(k_qsgd_quantize<4>, dim3((unsigned)ch.size()), dim3(kBlock), 0, 0, x, dch, 255.0f, norms, U,
                             lv, sg);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep >= 2) ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      printf("  %-14s chunk %5d  blocks %5zu  %7.2f us\n", v == 0 ? "cnat quantize" : "qsgd quantize", cs, ch.size(),
             ts[ts.size() / 2] * 1e3);
    }
    CK(hipFree(dch));
  }
  CK(hipFree(x));
  CK(hipFree(lv));
  CK(hipFree(sg));
  CK(hipFree(q));
  CK(hipFree(norms));
  CK(hipFree(ws));
  CK(hipFree(junk));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1) g_reps = atoi(argv[1]);  // e.g. 2 under rocprofv3 --pmc
  if (argc > 2 && strcmp(argv[2], "chunks") == 0) return run_chunk_sizes();
  std::vector<int64_t> c3(256);
  for (int i = 0; i < 256; ++i) c3[i] = 11689512 / 256 + (i < 11689512 % 256 ? 1 : 0);
  run("C3", c3);
  run("C2", {1ll << 28});
  return 0;
}
