// microbench_stoch_timeline.hip — where the C3 one-launch CNAT encode (k_cnat_encode_resident: one 1024-thread
// block per tensor, 4 groups of 256 threads, each group quantizing 2 chunks) spends its time. An
// instrumented copy of the product kernel (same arithmetic, output compared bit for bit) stamps
// wall_clock64() (100 MHz) in wave 0 of every block at entry, after chunk round 0's quantize, after chunk
// round 1's quantize, and after the block's norm barrier. Also times the product kernel and variants:
//   norng   the product kernel with the uniforms taken as a constant (no Philox): the RNG's share
// Not part of the product; it #includes the product source.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_stoch_timeline \
//         tools/microbench_stoch_timeline.hip ad-federatedlearning_amd/csrc/slq_codec.hip
#include "../ad-federatedlearning_amd/csrc/stoch_codec.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

struct Stamp {
  uint64_t t[5];  // entry, round 0 quantized, round 1 quantized, norm barrier passed, every store acked
  uint64_t pad[3];
};

// MODE 0: instrumented copy; 1: no RNG (constant uniforms; output differs, timing only)
template <int PB, int MODE>
__global__ __launch_bounds__(kResBlock) void k_cnat_res_tl(const float* __restrict__ x,
                                                           const adfl_slq_chunk* __restrict__ chunks,
                                                           const int32_t* __restrict__ work, int min_e, int max_e,
                                                           Uniforms U, int8_t* __restrict__ exps,
                                                           int8_t* __restrict__ signs, float* __restrict__ norms,
                                                           Stamp* __restrict__ st) {
  __shared__ double red_s[kResPerGroup][kResWaves];
  uint64_t ts[5];
  ts[0] = wall_clock64();
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk ct = chunks[ci];
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x / kBlock);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = threadIdx.x % kBlock, lane = threadIdx.x & 63;
  const auto fast = [=](float xv, float uv, bool& bad) { return cnat_exp_fast(xv, uv, min_e, max_e, bad); };
  const auto exact = [=](float xv, float uv) { return cnat_exp_exact(xv, uv, min_e, max_e); };
  float4 v[kResPerGroup][kPer];
  int n4s[kResPerGroup];
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    n4s[r] = 0;
    if (kc < ct.nchunks) {
      const adfl_slq_chunk c = chunks[ci + kc];
      const int head = chunk_head4(c.start, c.len);
      n4s[r] = (c.len - head) >> 2;
      load_chunk_regs(reinterpret_cast<const float4*>(x + c.start + head), n4s[r], tg, v[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    NormAcc<ADFL_NORM_L2> acc;
    if (kc < ct.nchunks) {
      const adfl_slq_chunk c = chunks[ci + kc];
      const float* xc = x + c.start;
      int8_t* ex = exps + c.start;
      int8_t* sg = signs + c.start;
      const int head = chunk_head4(c.start, c.len);
      if (MODE == 1) {
        const float4 uc = make_float4(0.3f, 0.6f, 0.1f, 0.9f);
        uint32_t* l4 = reinterpret_cast<uint32_t*>(ex + head);
        uint32_t* s4 = reinterpret_cast<uint32_t*>(sg + head);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const int k = tg + j * kBlock;
          if (k < n4s[r]) {
            bool bad = false;
            l4[k] = pack4(fast(v[r][j].x, uc.x, bad), fast(v[r][j].y, uc.y, bad), fast(v[r][j].z, uc.z, bad),
                          fast(v[r][j].w, uc.w, bad));
            s4[k] = pack4(sign_byte(v[r][j].x), sign_byte(v[r][j].y), sign_byte(v[r][j].z), sign_byte(v[r][j].w));
            acc.add4(v[r][j]);
          }
        }
      } else {
        quantize_regs<PB>(v[r], tg, n4s[r], c.start + head, U, reinterpret_cast<uint32_t*>(ex + head),
                          reinterpret_cast<uint32_t*>(sg + head), fast, exact, false, &acc);
      }
      const int i = edge_elem_t(tg, head, head + (n4s[r] << 2), c.len);
      if (i >= 0) {
        const float e = xc[i];
        ex[i] = (int8_t)exact(e, U.one(c.start + i));
        sg[i] = (int8_t)sign_byte(e);
        acc.add(e);
      }
    }
    double a = acc.s;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (lane == 0) red_s[r][wave] = a;
    ts[1 + r] = wall_clock64();
  }
  __syncthreads();
  const float norm = resident_l2(red_s, ct.nchunks);
  if (threadIdx.x == 0) norms[ct.tensor] = norm;
  ts[3] = wall_clock64();
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    Stamp s;
    for (int k = 0; k < 4; ++k) s.t[k] = ts[k];
    s.t[4] = wall_clock64();
    st[blockIdx.x] = s;
  }
}

// Variant: round 0's Philox words made into LDS while x streams in (as k_qsgd_encode_resident does), round 1
// quantized with PB1 Philox blocks per batch. Same stream, same output as the product.
template <bool PRE, int PB0, int PB1>
__global__ __launch_bounds__(kResBlock) void k_cnat_res_v2(const float* __restrict__ x,
                                                           const adfl_slq_chunk* __restrict__ chunks,
                                                           const int32_t* __restrict__ work, int min_e, int max_e,
                                                           Uniforms U, int8_t* __restrict__ exps,
                                                           int8_t* __restrict__ signs, float* __restrict__ norms,
                                                           Stamp* __restrict__ st) {
  uint64_t ts[5] = {(uint64_t)wall_clock64(), 0, 0, 0, 0};
  __shared__ double red_s[kResPerGroup][kResWaves];
  __shared__ uint4 pre[PRE ? kPer : 1][kResBlock];
  const int64_t ci = work[blockIdx.x];
  const adfl_slq_chunk ct = chunks[ci];
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x / kBlock);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = threadIdx.x % kBlock, lane = threadIdx.x & 63;
  const auto fast = [=](float xv, float uv, bool& bad) { return cnat_exp_fast(xv, uv, min_e, max_e, bad); };
  const auto exact = [=](float xv, float uv) { return cnat_exp_exact(xv, uv, min_e, max_e); };
  float4 v[kResPerGroup][kPer];
  int n4s[kResPerGroup];
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    n4s[r] = 0;
    if (kc < ct.nchunks) {
      const adfl_slq_chunk c = chunks[ci + kc];
      const int head = chunk_head4(c.start, c.len);
      n4s[r] = (c.len - head) >> 2;
      load_chunk_regs(reinterpret_cast<const float4*>(x + c.start + head), n4s[r], tg, v[r]);
    }
  }
  if (PRE && !U.inj && grp < ct.nchunks) {
    const adfl_slq_chunk c = chunks[ci + grp];
    const int64_t q0 = (c.start + chunk_head4(c.start, c.len)) >> 2;
#pragma unroll
    for (int jb = 0; jb < kPer; jb += PB0) {
      if (jb * kBlock >= n4s[0]) break;
      uint64_t ctr[PB0];
      uint4 w[PB0];
#pragma unroll
      for (int i = 0; i < PB0; ++i) ctr[i] = U.counter + (uint64_t)(q0 + tg + (jb + i) * kBlock);
      philox4x32_batch(ctr, U.seed, w);
#pragma unroll
      for (int i = 0; i < PB0; ++i) pre[PRE ? jb + i : 0][threadIdx.x] = w[i];
    }
  }
  ts[4] = wall_clock64();  // Philox precompute done (before any use of x)
#pragma unroll
  for (int r = 0; r < kResPerGroup; ++r) {
    const int kc = grp + r * kResGroups;
    NormAcc<ADFL_NORM_L2> acc;
    if (kc < ct.nchunks) {
      const adfl_slq_chunk c = chunks[ci + kc];
      const float* xc = x + c.start;
      int8_t* ex = exps + c.start;
      int8_t* sg = signs + c.start;
      const int head = chunk_head4(c.start, c.len);
      if (r == 0)
        quantize_regs<PB0>(v[r], tg, n4s[r], c.start + head, U, reinterpret_cast<uint32_t*>(ex + head),
                           reinterpret_cast<uint32_t*>(sg + head), fast, exact, false, &acc,
                           PRE ? &pre[0][threadIdx.x] : nullptr, kResBlock);
      else
        quantize_regs<PB1>(v[r], tg, n4s[r], c.start + head, U, reinterpret_cast<uint32_t*>(ex + head),
                           reinterpret_cast<uint32_t*>(sg + head), fast, exact, false, &acc);
      const int i = edge_elem_t(tg, head, head + (n4s[r] << 2), c.len);
      if (i >= 0) {
        const float e = xc[i];
        ex[i] = (int8_t)exact(e, U.one(c.start + i));
        sg[i] = (int8_t)sign_byte(e);
        acc.add(e);
      }
    }
    double a = acc.s;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (lane == 0) red_s[r][wave] = a;
    ts[1 + r] = wall_clock64();
  }
  __syncthreads();
  const float norm = resident_l2(red_s, ct.nchunks);
  if (threadIdx.x == 0) norms[ct.tensor] = norm;
  ts[3] = wall_clock64();
  if (st && threadIdx.x == 0) {
    Stamp s;
    for (int k = 0; k < 5; ++k) s.t[k] = ts[k];
    st[blockIdx.x] = s;
  }
}

double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

Stamp* g_st = nullptr;

void run(int reps) {
  // C3 equal layout: 256 x 45,662 (11,689,512 fp32), 64-element aligned
  const int T = 256;
  std::vector<int64_t> sizes, offs;
  int64_t o = 0;
  for (int i = 0; i < T; ++i) {
    const int64_t s = 11689512 / T + (i < 11689512 % T ? 1 : 0);
    sizes.push_back(s);
    offs.push_back(o);
    o += (s + 63) / 64 * 64;
  }
  const int64_t total = o;
  const int64_t nch = adfl_slq_build_chunks(offs.data(), sizes.data(), T, nullptr, 0);
  std::vector<adfl_slq_chunk> ch(nch);
  adfl_slq_build_chunks(offs.data(), sizes.data(), T, ch.data(), nch);
  const int64_t nwork = adfl_slq_build_encode_work(ch.data(), nch, nullptr, 0);
  std::vector<int32_t> work(nwork);
  adfl_slq_build_encode_work(ch.data(), nch, work.data(), nwork);
  float *x, *nr, *nr2;
  int8_t *e1, *s1, *e2, *s2;
  int32_t* dwork;
  adfl_slq_chunk* dch;
  uint4* junk;
  uint32_t* sink;
  Stamp* dst;
  const int64_t junk_bytes = 512ll << 20;
  CK(hipMalloc(&x, total * 4));
  CK(hipMalloc(&e1, total));
  CK(hipMalloc(&s1, total));
  CK(hipMalloc(&e2, total));
  CK(hipMalloc(&s2, total));
  CK(hipMalloc(&nr, T * 4));
  CK(hipMalloc(&nr2, T * 4));
  CK(hipMalloc(&dwork, nwork * 4));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&junk, junk_bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&dst, nwork * sizeof(Stamp)));
  CK(hipMemset(junk, 0, junk_bytes));
  CK(hipMemcpy(dwork, work.data(), nwork * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  std::vector<float> hx(total, 0.0f);
  uint32_t r = 777;
  for (int64_t i = 0; i < total; ++i) {
    r = r * 1664525u + 1013904223u;
    hx[i] = ((int32_t)r) * 1e-12f;
  }
  CK(hipMemcpy(x, hx.data(), total * 4, hipMemcpyHostToDevice));
  Uniforms U{nullptr, 99, 0};
  const int min_e = -127, max_e = 0;  // bits 8 (quant.py:516-520)
  auto product = [&]() {
    hipLaunchKernelGGL(k_cnat_encode_resident<kPbResident>, dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch,
                       dwork, min_e, max_e, U, e1, s1, nr);
  };
  auto tl = [&]() {
    hipLaunchKernelGGL((k_cnat_res_tl<kPbResident, 0>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork,
                       min_e, max_e, U, e2, s2, nr2, dst);
  };
  auto norng = [&]() {
    hipLaunchKernelGGL((k_cnat_res_tl<kPbResident, 1>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork,
                       min_e, max_e, U, e2, s2, nr2, dst);
  };
  auto same = [&]() {
    CK(hipDeviceSynchronize());
    std::vector<int8_t> a(total), b(total), c(total), d(total);
    std::vector<float> na(T), nb(T);
    CK(hipMemcpy(a.data(), e1, total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), e2, total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), s1, total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d.data(), s2, total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(na.data(), nr, T * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(nb.data(), nr2, T * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int t = 0; t < T && ok; ++t)
      ok = std::equal(a.begin() + offs[t], a.begin() + offs[t] + sizes[t], b.begin() + offs[t]) &&
           std::equal(c.begin() + offs[t], c.begin() + offs[t] + sizes[t], d.begin() + offs[t]) && na[t] == nb[t];
    CK(hipMemset(e2, 0x55, total));
    return ok;
  };
  std::vector<std::pair<const char*, std::function<void()>>> vars = {
      {"pre + PB0 2 / PB1 2", [&]() { hipLaunchKernelGGL((k_cnat_res_v2<true, 2, 2>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork, min_e, max_e, U, e2, s2, nr2, g_st); }},
      {"pre + PB0 4 / PB1 4", [&]() { hipLaunchKernelGGL((k_cnat_res_v2<true, 4, 4>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork, min_e, max_e, U, e2, s2, nr2, g_st); }},
      {"pre + PB0 8 / PB1 4", [&]() { hipLaunchKernelGGL((k_cnat_res_v2<true, 8, 4>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork, min_e, max_e, U, e2, s2, nr2, g_st); }},
      {"pre + PB0 4 / PB1 8", [&]() { hipLaunchKernelGGL((k_cnat_res_v2<true, 4, 8>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork, min_e, max_e, U, e2, s2, nr2, g_st); }},
      {"no pre, PB 4 / 4", [&]() { hipLaunchKernelGGL((k_cnat_res_v2<false, 4, 4>), dim3((unsigned)nwork), dim3(kResBlock), 0, 0, x, dch, dwork, min_e, max_e, U, e2, s2, nr2, g_st); }},
  };
  product();
  tl();
  const bool ok_tl = same();
  for (auto& vv : vars) {
    vv.second();
    printf("  variant %-22s parity vs product: %s\n", vv.first, same() ? "yes" : "NO");
  }
  std::vector<std::vector<double>> tv(vars.size());
  for (int rep = 0; rep < reps; ++rep)
    for (size_t k = 0; k < vars.size(); ++k) {
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
      hipEvent_t a0, a1;
      CK(hipEventCreate(&a0));
      CK(hipEventCreate(&a1));
      CK(hipEventRecord(a0, 0));
      vars[k].second();
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      float ms;
      CK(hipEventElapsedTime(&ms, a0, a1));
      if (rep >= 5) tv[k].push_back(ms * 1e3);
      CK(hipEventDestroy(a0));
      CK(hipEventDestroy(a1));
    }
  {
    int wall_khz = 0;
    CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    for (size_t k = 0; k < vars.size(); ++k) {
      CK(hipMemset(dst, 0, nwork * sizeof(Stamp)));
      g_st = dst;
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
      vars[k].second();
      CK(hipDeviceSynchronize());
      g_st = nullptr;
      std::vector<Stamp> hs(nwork);
      CK(hipMemcpy(hs.data(), dst, nwork * sizeof(Stamp), hipMemcpyDeviceToHost));
      uint64_t tmin = ~0ull;
      for (auto& q : hs) tmin = std::min(tmin, q.t[0]);
      const double us = 1e3 / wall_khz;
      std::vector<double> p[5];
      for (auto& q : hs)
        for (int j = 0; j < 5; ++j) p[j].push_back((double)(q.t[j] - tmin) * us);
      printf("  variant %-22s p50 us: philox pre done %6.2f, round 0 %6.2f, round 1 %6.2f, norm %6.2f\n",
             vars[k].first, pct(p[4], 0.5), pct(p[1], 0.5), pct(p[2], 0.5), pct(p[3], 0.5));
    }
  }
  for (size_t k = 0; k < vars.size(); ++k) {
    const double m = pct(tv[k], 0.5);
    printf("  variant %-22s flushed median %7.2f us (6 B/elem: %.3f of 8 TB/s)\n", vars[k].first, m,
           6.0 * 11689512 / (m * 1e-6) / 8e12);
  }
  printf("C3 CNAT resident (bits 8): %lld tensors; parity vs product: instrumented %s\n", (long long)nwork,
         ok_tl ? "yes" : "NO");
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  const char* names[] = {"product", "instrumented", "no RNG (timing only)"};
  std::vector<std::vector<double>> t(3);
  std::vector<std::vector<double>> ph(5);
  int wall_khz = 0;
  CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  for (int rep = 0; rep < reps; ++rep)
    for (int v = 0; v < 3; ++v) {
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
      CK(hipEventRecord(ev0, 0));
      if (v == 0) product();
      if (v == 1) tl();
      if (v == 2) norng();
      CK(hipEventRecord(ev1, 0));
      CK(hipEventSynchronize(ev1));
      float ms;
      CK(hipEventElapsedTime(&ms, ev0, ev1));
      if (rep >= 5) t[v].push_back(ms * 1e3);
      if ((v == 1 || v == 2) && rep == reps - 1) {
        std::vector<Stamp> hs(nwork);
        CK(hipMemcpy(hs.data(), dst, nwork * sizeof(Stamp), hipMemcpyDeviceToHost));
        uint64_t tmin = ~0ull;
        for (auto& s : hs) tmin = std::min(tmin, s.t[0]);
        const double us = 1e3 / wall_khz;
        const char* pn[] = {"entry", "round 0 done", "round 1 done", "norm barrier", "stores acked"};
        printf("  timeline (%s, last rep), us from the first entry:\n", names[v]);
        for (int k = 0; k < 5; ++k) {
          std::vector<double> p;
          for (auto& s : hs) p.push_back((double)(s.t[k] - tmin) * us);
          printf("    %-14s min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f\n", pn[k], pct(p, 0.0),
                 pct(p, 0.1), pct(p, 0.5), pct(p, 0.9), pct(p, 1.0));
        }
      }
    }
  for (int v = 0; v < 3; ++v) {
    const double m = pct(t[v], 0.5);
    printf("  %-24s flushed median %7.2f us (6 B/elem: %.3f of 8 TB/s)\n", names[v], m,
           6.0 * 11689512 / (m * 1e-6) / 8e12);
  }
}
}  // namespace

int main(int argc, char** argv) {
  run(argc > 1 ? atoi(argv[1]) : 40);
  return 0;
}
