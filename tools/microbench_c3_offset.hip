// microbench_c3_offset.hip — verdict r04 item 6's experiment: can the C3 one-launch encode's store tail be
// overlapped with other tensors' loads by putting half of the blocks half a load phase behind the others?
// Every tensor of the equal layout is one 1024-thread block on its own CU, and all 256 blocks load, reduce and
// store in lockstep (profiles/r03/c3_resident/timeline.txt), so the ~3 us of stores at the end overlap
// nothing. Here a copy of k_encode_resident waits `delay` wall-clock ticks (10 ns) before its loads in half
// of the blocks (odd blocks, or the second half of the work list), so those blocks load while the first half
// stores. Outputs are compared with the product kernel's bit for bit; encode-only spans, Infinity Cache
// read-flushed, medians of 55. Not part of the product; it #includes the product source.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_c3_offset \
//     tools/microbench_c3_offset.hip
#include "../ad-federatedlearning_amd/csrc/slq_codec.hip"

#include <algorithm>
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
__global__ void k_flush(const uint4* __restrict__ junk, int64_t n16, uint32_t* __restrict__ sink) {
  uint32_t a = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    a ^= junk[i].x;
  if (a == 0x12345678u) *sink = a;
}

// k_encode_resident<false> with a start delay for the blocks `mode` selects (1: odd blocks, 2: second half).
__global__ __launch_bounds__(kSegBlock) void k_encode_resident_delay(const float* __restrict__ x,
                                                                     const adfl_slq_chunk* __restrict__ chunks,
                                                                     const int32_t* __restrict__ work, float qmax,
                                                                     int8_t* __restrict__ q, float* __restrict__ scales,
                                                                     int mode, uint64_t delay) {
  const bool late = mode == 1 ? (blockIdx.x & 1) != 0 : (mode == 2 ? blockIdx.x >= gridDim.x / 2 : false);
  if (late && delay) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < delay) __builtin_amdgcn_s_sleep(2);
  }
  __shared__ __attribute__((aligned(16))) uint32_t lds[kSegWaves][kTile / 4];
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk c = chunks[ci];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int len = (c.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + c.nchunks - 1].len;
  const float* xt = x + c.start;
  const int head = chunk_head(c.start, len, 16);
  const int ntiles = (len - head) / kTile;
  const float4* x4 = reinterpret_cast<const float4*>(xt + head);
  float4 v[kSegTilesPerWave][4];
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles) {
      load_tile(x4 + t * (kTile / 4), v[k], lane);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[k][j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float hv = (int)threadIdx.x < head ? xt[threadIdx.x] : 0.0f;
  const int ti = head + ntiles * kTile + (int)threadIdx.x;
  const float tv = ti < len ? __builtin_nontemporal_load(xt + ti) : 0.0f;
  uint32_t m = max(abs_bits(hv), abs_bits(tv));
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) m = max(m, abs_bits4(v[k][j]));
  const ScaleInv si = make_scale(block_max_seg(m), qmax);
  if (threadIdx.x == 0) scales[c.tensor] = si.scale;
  int8_t* qt = q + c.start;
  uint4* q16 = reinterpret_cast<uint4*>(qt + head);
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles) quantize_tile_regs<false>(v[k], q16 + t * (kTile / 16), si.inv, lds[wave], lane);
  }
  if ((int)threadIdx.x < head) qt[threadIdx.x] = (int8_t)quant1(hv, si.inv);
  if (ti < len) qt[ti] = (int8_t)quant1(tv, si.inv);
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
}  // namespace

int main() {
  const int64_t n = 11689512;
  std::vector<int64_t> sizes, offs;
  int64_t o = 0;
  for (int i = 0; i < 256; ++i) {
    const int64_t s = n / 256 + (i < n % 256 ? 1 : 0);
    sizes.push_back(s);
    offs.push_back(o);
    o += s;  // compact, as the channel stages it
  }
  const int64_t total = o;
  const int64_t nch = adfl_slq_build_chunks(offs.data(), sizes.data(), 256, nullptr, 0);
  std::vector<adfl_slq_chunk> ch(nch);
  adfl_slq_build_chunks(offs.data(), sizes.data(), 256, ch.data(), nch);
  const int64_t nwork = adfl_slq_build_encode_work(ch.data(), nch, nullptr, 0);
  std::vector<int32_t> work(nwork);
  adfl_slq_build_encode_work(ch.data(), nch, work.data(), nwork);
  float *x, *sc, *sc2;
  int8_t *q, *q2;
  uint32_t *part, *sink;
  int32_t* dwork;
  adfl_slq_chunk* dch;
  uint4* junk;
  const int64_t junk_bytes = 512ll << 20;
  CK(hipMalloc(&x, total * 4));
  CK(hipMalloc(&q, total));
  CK(hipMalloc(&q2, total));
  CK(hipMalloc(&sc, 1024));
  CK(hipMalloc(&sc2, 1024));
  CK(hipMalloc(&part, nch * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&dwork, nwork * 4));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&junk, junk_bytes));
  CK(hipMemset(junk, 0, junk_bytes));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  CK(hipMemcpy(dwork, work.data(), nwork * 4, hipMemcpyHostToDevice));
  std::vector<float> hx(total);
  uint32_t r = 12345;
  for (int64_t i = 0; i < total; ++i) {
    r = r * 1664525u + 1013904223u;
    hx[i] = ((int32_t)r) * 1e-12f;
  }
  CK(hipMemcpy(x, hx.data(), total * 4, hipMemcpyHostToDevice));
  const float qmax = 127.0f;
  auto product = [&]() { CK(adfl_slq_encode_batched_work(x, dch, nch, dwork, nwork, 8, q, sc, part, nullptr)); };
  auto variant = [&](int mode, uint64_t delay) {
    hipLaunchKernelGGL(k_encode_resident_delay, dim3((unsigned)nwork), dim3(kSegBlock), 0, 0, x, dch, dwork, qmax, q2,
                       sc2, mode, delay);
    CK(hipGetLastError());
  };
  product();
  variant(1, 200);
  CK(hipDeviceSynchronize());
  std::vector<int8_t> a(total), b(total);
  std::vector<float> sa(256), sb(256);
  CK(hipMemcpy(a.data(), q, total, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), q2, total, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sa.data(), sc, 1024, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sb.data(), sc2, 1024, hipMemcpyDeviceToHost));
  printf("C3 equal, compact: %lld tensors, one block each; variant == product: %s\n", (long long)nwork,
         (a == b && sa == sb) ? "yes" : "NO");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    int mode;
    uint64_t delay;
  };
  const V vs[] = {{"product k_encode_resident", -1, 0}, {"copy, no delay", 0, 0},
                  {"odd blocks +1 us", 1, 100},        {"odd blocks +2 us", 1, 200},
                  {"odd blocks +3 us", 1, 300},        {"odd blocks +4 us", 1, 400},
                  {"second half +2 us", 2, 200},       {"second half +4 us", 2, 400}};
  const int nv = sizeof(vs) / sizeof(vs[0]);
  std::vector<std::vector<double>> t(nv);
  for (int rep = 0; rep < 60; ++rep)
    for (int v = 0; v < nv; ++v) {
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
      CK(hipEventRecord(e0, 0));
      if (vs[v].mode < 0) product();
      else variant(vs[v].mode, vs[v].delay);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 5) t[v].push_back(ms);
    }
  const double moved = 5.0 * n;  // x read once, payload written once
  for (int v = 0; v < nv; ++v) {
    const double us = median(t[v]) * 1e3;
    printf("  %-28s %7.2f us  (%.3f of 8 TB/s on 5 B/element)\n", vs[v].name, us, moved / (us * 1e-6) / 8e12);
  }
  return 0;
}
