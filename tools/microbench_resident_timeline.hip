// microbench_resident_timeline.hip — where the C3 one-launch encode (k_encode_resident: one 1024-thread block
// per tensor, the whole tensor in VGPRs) spends its time, and whether a schedule that overlaps one tensor's
// stores with the next tensor's loads shortens it. Not part of the product; it #includes the product source.
//
//   timeline   an instrumented copy of k_encode_resident stamps wall_clock64() (100 MHz) per block at
//              entry, after the tensor's loads have landed (its max loop consumed every register), after
//              the block max (all waves loaded), and after its stores completed (a release fence, then a
//              block barrier). Printed as min / median / max over blocks relative to the first entry.
//   pair<P>    k_encode_resident_multi<P>: a block takes P tensors of the work list in turn; tile k of
//              tensor p+1 is loaded into the registers of tile k of tensor p right after that tile is
//              quantized, so tensor p's stores overlap tensor p+1's loads (grid = ntensors / P).
// Every variant's payload and scales are compared with the product's bit for bit. C3 layouts as
// tools/microbench_c3.hip (equal 256 x 45,662; 11,689,512 fp32), Infinity Cache read-flushed per launch.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_resident_timeline tools/microbench_resident_timeline.hip
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

struct Stamp {
  uint64_t t[4];  // entry, wave 0's loads landed, block max done, wave 0's stores issued
  uint32_t hw;
  uint32_t pad;   // ticks from entry to every wave's stores acknowledged (L2)
};

__device__ __forceinline__ uint32_t hw_id() {
  // HW_ID register: wave / SIMD / CU / SH / SE fields (the CU and SE bits identify the block's CU)
  return __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
}

// k_encode_resident with time stamps (same arithmetic, same output)
__global__ __launch_bounds__(kSegBlock) void k_encode_resident_tl(const float* __restrict__ x,
                                                                  const adfl_slq_chunk* __restrict__ chunks,
                                                                  const int32_t* __restrict__ work, float qmax,
                                                                  int8_t* __restrict__ q, float* __restrict__ scales,
                                                                  Stamp* __restrict__ st) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kSegWaves][kTile / 4];
  const uint64_t t0 = wall_clock64();
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
  const uint64_t t1 = wall_clock64();
  const ScaleInv si = make_scale(block_max_seg(m), qmax);
  const uint64_t t2 = wall_clock64();
  if (threadIdx.x == 0) scales[c.tensor] = si.scale;
  int8_t* qt = q + c.start;
  uint4* q16 = reinterpret_cast<uint4*>(qt + head);
#pragma unroll
  for (int k = 0; k < kSegTilesPerWave; ++k) {
    const int t = wave + k * kSegWaves;
    if (t < ntiles) quantize_tile_regs(v[k], q16 + t * (kTile / 16), si.inv, lds[wave], lane);
  }
  if ((int)threadIdx.x < head) qt[threadIdx.x] = (int8_t)quant1(hv, si.inv);
  if (ti < len) qt[ti] = (int8_t)quant1(tv, si.inv);
  const uint64_t t3 = wall_clock64();
  __builtin_amdgcn_s_waitcnt(0);  // this wave's stores acknowledged (vmcnt counts stores on gfx9)
  __syncthreads();
  if (threadIdx.x == 0) {
    Stamp s;
    s.t[0] = t0;
    s.t[1] = t1;
    s.t[2] = t2;
    s.t[3] = t3;
    s.hw = hw_id();
    s.pad = (uint32_t)(wall_clock64() - t0);
    st[blockIdx.x] = s;
  }
}

__device__ __forceinline__ uint32_t block_max_seg_buf(uint32_t v, uint32_t* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t m = red[0];
#pragma unroll
  for (int w = 1; w < kSegWaves; ++w) m = max(m, red[w]);
  return m;
}

struct ResTensor {
  int64_t start;
  int len, head, ntiles, tensor;
};

__device__ __forceinline__ ResTensor res_tensor(const adfl_slq_chunk* __restrict__ chunks, int64_t ci) {
  const adfl_slq_chunk c = chunks[ci];
  ResTensor r;
  r.start = c.start;
  r.len = (c.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ci + c.nchunks - 1].len;
  r.head = chunk_head(c.start, r.len, 16);
  r.ntiles = (r.len - r.head) / kTile;
  r.tensor = c.tensor;
  return r;
}

template <int P, bool ST_NT = false>
__global__ __launch_bounds__(kSegBlock) void k_encode_resident_multi(const float* __restrict__ x,
                                                                     const adfl_slq_chunk* __restrict__ chunks,
                                                                     const int32_t* __restrict__ work, int nwork,
                                                                     float qmax, int8_t* __restrict__ q,
                                                                     float* __restrict__ scales) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kSegWaves][kTile / 4];
  __shared__ uint32_t red[2][kSegWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w0 = blockIdx.x * P;
  ResTensor cur = res_tensor(chunks, work[w0]);
  float4 v[kSegTilesPerWave][4];
  {
    const float4* x4 = reinterpret_cast<const float4*>(x + cur.start + cur.head);
#pragma unroll
    for (int k = 0; k < kSegTilesPerWave; ++k) {
      const int t = wave + k * kSegWaves;
      if (t < cur.ntiles) {
        load_tile(x4 + t * (kTile / 4), v[k], lane);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if (w0 + p >= nwork) break;  // block-uniform
    const float* xt = x + cur.start;
    const float hv = (int)threadIdx.x < cur.head ? xt[threadIdx.x] : 0.0f;
    const int ti = cur.head + cur.ntiles * kTile + (int)threadIdx.x;
    const float tv = ti < cur.len ? __builtin_nontemporal_load(xt + ti) : 0.0f;
    uint32_t m = max(abs_bits(hv), abs_bits(tv));
#pragma unroll
    for (int k = 0; k < kSegTilesPerWave; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) m = max(m, abs_bits4(v[k][j]));
    const ScaleInv si = make_scale(block_max_seg_buf(m, red[p & 1]), qmax);
    if (threadIdx.x == 0) scales[cur.tensor] = si.scale;
    const bool more = p + 1 < P && w0 + p + 1 < nwork;
    ResTensor nxt = cur;
    if (more) nxt = res_tensor(chunks, work[w0 + p + 1]);
    const float4* xn4 = reinterpret_cast<const float4*>(x + nxt.start + nxt.head);
    int8_t* qt = q + cur.start;
    uint4* q16 = reinterpret_cast<uint4*>(qt + cur.head);
#pragma unroll
    for (int k = 0; k < kSegTilesPerWave; ++k) {
      const int t = wave + k * kSegWaves;
      if (t < cur.ntiles) quantize_tile_regs<ST_NT>(v[k], q16 + t * (kTile / 16), si.inv, lds[wave], lane);
      if (more) {
        if (t < nxt.ntiles) {
          load_tile(xn4 + t * (kTile / 4), v[k], lane);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[k][j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    if ((int)threadIdx.x < cur.head) qt[threadIdx.x] = (int8_t)quant1(hv, si.inv);
    if (ti < cur.len) qt[ti] = (int8_t)quant1(tv, si.inv);
    cur = nxt;
  }
}

struct Layout {
  const char* name;
  std::vector<int64_t> sizes, offs;
  int64_t total = 0;
};

Layout equal_layout() {
  Layout L{"equal"};
  const int64_t n = 11689512;
  int64_t o = 0;
  for (int i = 0; i < 256; ++i) {
    const int64_t s = n / 256 + (i < n % 256 ? 1 : 0);
    L.sizes.push_back(s);
    L.offs.push_back(o);
    o += (s + 63) / 64 * 64;
  }
  L.total = o;
  return L;
}

double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

void run(const Layout& L, int reps) {
  const int T = (int)L.sizes.size();
  const int64_t nch = adfl_slq_build_chunks(L.offs.data(), L.sizes.data(), T, nullptr, 0);
  std::vector<adfl_slq_chunk> ch(nch);
  adfl_slq_build_chunks(L.offs.data(), L.sizes.data(), T, ch.data(), nch);
  const int64_t nwork = adfl_slq_build_encode_work(ch.data(), nch, nullptr, 0);
  if (nwork == 0) {
    printf("%s: a tensor exceeds one block; no resident encode\n", L.name);
    return;
  }
  std::vector<int32_t> work(nwork);
  adfl_slq_build_encode_work(ch.data(), nch, work.data(), nwork);
  int64_t n = 0;
  for (auto s : L.sizes) n += s;
  int32_t* dwork;
  float *x, *sc, *sc2;
  int8_t *q, *q2;
  uint32_t* sink;
  adfl_slq_chunk* dch;
  uint4* junk;
  Stamp* dst;
  const int64_t junk_bytes = 512ll << 20;
  CK(hipMalloc(&dwork, nwork * 4));
  CK(hipMalloc(&x, L.total * 4));
  CK(hipMalloc(&q, L.total));
  CK(hipMalloc(&q2, L.total));
  CK(hipMalloc(&sc, T * 4));
  CK(hipMalloc(&sc2, T * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&junk, junk_bytes));
  CK(hipMalloc(&dst, nwork * sizeof(Stamp)));
  CK(hipMemset(junk, 0, junk_bytes));
  CK(hipMemcpy(dwork, work.data(), nwork * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  std::vector<float> hx(L.total, 0.0f);
  uint32_t r = 12345;
  for (int t = 0; t < T; ++t)
    for (int64_t i = 0; i < L.sizes[t]; ++i) {
      r = r * 1664525u + 1013904223u;
      hx[L.offs[t] + i] = ((int32_t)r) * 1e-12f * (float)(1 + t % 7);
    }
  CK(hipMemcpy(x, hx.data(), L.total * 4, hipMemcpyHostToDevice));
  const float qmax = 127.0f;

  auto product = [&]() {
    hipLaunchKernelGGL(k_encode_resident<false>, dim3((unsigned)nwork), dim3(kSegBlock), 0, 0, x, dch, dwork, qmax, q, sc);
  };
  auto timeline = [&]() {
    hipLaunchKernelGGL(k_encode_resident_tl, dim3((unsigned)nwork), dim3(kSegBlock), 0, 0, x, dch, dwork, qmax, q2,
                       sc2, dst);
  };
  auto multi = [&](int P) {
    const unsigned g = (unsigned)((nwork + std::abs(P) - 1) / std::abs(P));
    if (P == 1) hipLaunchKernelGGL(k_encode_resident_multi<1>, dim3(g), dim3(kSegBlock), 0, 0, x, dch, dwork, (int)nwork, qmax, q2, sc2);
    if (P == 2) hipLaunchKernelGGL(k_encode_resident_multi<2>, dim3(g), dim3(kSegBlock), 0, 0, x, dch, dwork, (int)nwork, qmax, q2, sc2);
    if (P == 4) hipLaunchKernelGGL(k_encode_resident_multi<4>, dim3(g), dim3(kSegBlock), 0, 0, x, dch, dwork, (int)nwork, qmax, q2, sc2);
    if (P == -1) hipLaunchKernelGGL((k_encode_resident_multi<1, true>), dim3(g), dim3(kSegBlock), 0, 0, x, dch, dwork, (int)nwork, qmax, q2, sc2);
  };
  auto same = [&]() {
    std::vector<int8_t> a(L.total), b(L.total);
    std::vector<float> sa(T), sb(T);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a.data(), q, L.total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), q2, L.total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sa.data(), sc, T * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sb.data(), sc2, T * 4, hipMemcpyDeviceToHost));
    bool ok = std::equal(sa.begin(), sa.end(), sb.begin());
    for (int t = 0; t < T && ok; ++t)
      ok = std::equal(a.begin() + L.offs[t], a.begin() + L.offs[t] + L.sizes[t], b.begin() + L.offs[t]);
    CK(hipMemset(q2, 0x55, L.total));
    CK(hipMemset(sc2, 0, T * 4));
    return ok;
  };
  product();
  timeline();
  const bool ok_tl = same();
  multi(1);
  const bool ok1 = same();
  multi(2);
  const bool ok2 = same();
  multi(4);
  const bool ok4 = same();
  multi(-1);
  const bool oknt = same();
  printf("%s: %lld elements in %d tensors (%lld work entries); parity vs product: timeline %s, multi<1> %s, "
         "multi<2> %s, multi<4> %s, nt-stores %s\n", L.name, (long long)n, T, (long long)nwork, ok_tl ? "yes" : "NO",
         ok1 ? "yes" : "NO", ok2 ? "yes" : "NO", ok4 ? "yes" : "NO", oknt ? "yes" : "NO");

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"product k_encode_resident", "timeline (instrumented)", "multi<1>", "multi<2>", "multi<4>",
                         "multi<1> nt stores"};
  const int nv = 6;
  std::vector<std::vector<double>> t(nv);
  int wall_khz = 0;
  CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  std::vector<std::vector<double>> ph(4);
  std::vector<double> span, acked;
  std::vector<uint32_t> hws;
  for (int rep = 0; rep < reps; ++rep)
    for (int v = 0; v < nv; ++v) {
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
      CK(hipEventRecord(e0, 0));
      switch (v) {
        case 0: product(); break;
        case 1: timeline(); break;
        case 2: multi(1); break;
        case 3: multi(2); break;
        case 4: multi(4); break;
        case 5: multi(-1); break;
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 5) t[v].push_back(ms * 1e3);
      if (v == 1 && rep == reps - 1) {
        std::vector<Stamp> hs(nwork);
        CK(hipMemcpy(hs.data(), dst, nwork * sizeof(Stamp), hipMemcpyDeviceToHost));
        uint64_t tmin = ~0ull, tmax = 0;
        for (auto& s : hs) {
          tmin = std::min(tmin, s.t[0]);
          tmax = std::max(tmax, s.t[3]);
        }
        const double us = 1e3 / wall_khz;
        for (auto& s : hs) {
          for (int k = 0; k < 4; ++k) ph[k].push_back((double)(s.t[k] - tmin) * us);
          acked.push_back((double)(s.t[0] - tmin + s.pad) * us);
          hws.push_back(s.hw);
        }
        span.push_back((double)(tmax - tmin) * us);
      }
    }
  for (int v = 0; v < nv; ++v) {
    const double m = pct(t[v], 0.5);
    printf("  %-28s flushed median %7.2f us  (5 B/elem counted: %.3f of 8 TB/s; 9 B/elem: %.3f)\n", names[v], m,
           5.0 * n / (m * 1e-6) / 8e12, 9.0 * n / (m * 1e-6) / 8e12);
  }
  const char* pn[] = {"entry", "w0 loads landed", "block max done", "w0 stores issued"};
  printf("  timeline of the instrumented encode (last rep; wall clock %d kHz), us from the first block's entry:\n",
         wall_khz);
  for (int k = 0; k < 4; ++k)
    printf("    %-16s min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f\n", pn[k], pct(ph[k], 0.0),
           pct(ph[k], 0.1), pct(ph[k], 0.5), pct(ph[k], 0.9), pct(ph[k], 1.0));
  printf("    %-16s min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f\n", "stores acked", pct(acked, 0.0),
         pct(acked, 0.1), pct(acked, 0.5), pct(acked, 0.9), pct(acked, 1.0));
  std::vector<double> d01, d12, d23;
  for (size_t i = 0; i < ph[0].size(); ++i) {
    d01.push_back(ph[1][i] - ph[0][i]);
    d12.push_back(ph[2][i] - ph[1][i]);
    d23.push_back(ph[3][i] - ph[2][i]);
  }
  printf("    per block: load %5.2f us (p50), barrier+max %5.2f us, quantize+store %5.2f us; span entry..last store "
         "%.2f us\n", pct(d01, 0.5), pct(d12, 0.5), pct(d23, 0.5), span.empty() ? 0.0 : span.back());
  std::sort(hws.begin(), hws.end());
  printf("    distinct HW_ID values %zu of %zu blocks\n", (size_t)(std::unique(hws.begin(), hws.end()) - hws.begin()),
         (size_t)nwork);
  CK(hipFree(dwork));
  CK(hipFree(x));
  CK(hipFree(q));
  CK(hipFree(q2));
  CK(hipFree(sc));
  CK(hipFree(sc2));
  CK(hipFree(sink));
  CK(hipFree(dch));
  CK(hipFree(junk));
  CK(hipFree(dst));
}
}  // namespace

int main(int argc, char** argv) {
  run(equal_layout(), argc > 1 ? atoi(argv[1]) : 40);
  return 0;
}
