// microbench_c3.hip — the C3 bucketed round trip (11,689,512 fp32 in 256 tensors), timed as ONE span of
// events around encode + decode (no event between the launches), Infinity Cache warm and read-flushed:
//   two-pass  adfl_slq_encode_batched (absmax partials, then quantize re-reading x) + decode
//   work      adfl_slq_encode_batched_work: one launch, a whole tensor per 1024-thread block (x read once)
//             when every tensor has <= 65,536 elements, else the two-pass encode + decode
// for the equal layout (256 x 45,662) and the log-uniform layout (64 .. 2.4 M elements; tensors above
// 65,536 elements take the partials + quantize passes). Outputs are compared bit for bit. Also the
// encode and the decode alone. Not part of the product; it #includes the product source.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_c3 tools/microbench_c3.hip
#include "../ad-federatedlearning_amd/csrc/slq_codec.hip"

#include <algorithm>
#include <cmath>
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
  if (a == 0x12345678u) *sink = a;  // keeps the reads; never true for the zero-filled junk
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

// seeded log-uniform sizes in [64, 2.4 M], rescaled to sum to ResNet-18's count (as tests/golden/recipes.py)
Layout loguniform_layout() {
  Layout L{"loguniform"};
  uint64_t s = 0x9E3779B97F4A7C15ull;
  std::vector<double> raw(256);
  double sum = 0;
  for (auto& r : raw) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;
    r = std::exp(std::log(64.0) + u * (std::log(2.4e6) - std::log(64.0)));
    sum += r;
  }
  int64_t o = 0, acc = 0;
  for (int i = 0; i < 256; ++i) {
    int64_t sz = std::max<int64_t>(64, (int64_t)(raw[i] / sum * 11689512.0));
    if (i == 255) sz = std::max<int64_t>(64, 11689512 - acc);
    acc += sz;
    L.sizes.push_back(sz);
    L.offs.push_back(o);
    o += (sz + 63) / 64 * 64;
  }
  L.total = o;
  return L;
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

void run(const Layout& L) {
  const int64_t nch = adfl_slq_build_chunks(L.offs.data(), L.sizes.data(), 256, nullptr, 0);
  std::vector<adfl_slq_chunk> ch(nch);
  adfl_slq_build_chunks(L.offs.data(), L.sizes.data(), 256, ch.data(), nch);
  int32_t maxc = 0;
  int64_t n = 0, nbig = 0;
  for (auto& c : ch) maxc = std::max(maxc, c.nchunks);
  for (auto sz : L.sizes) {
    n += sz;
    if (sz > kSegMaxElems) nbig += sz;
  }
  const int64_t nwork = adfl_slq_build_encode_work(ch.data(), nch, nullptr, 0);
  std::vector<int32_t> work(nwork + 1);
  if (nwork) adfl_slq_build_encode_work(ch.data(), nch, work.data(), nwork);
  int32_t* dwork;
  CK(hipMalloc(&dwork, (nwork + 1) * 4));
  CK(hipMemcpy(dwork, work.data(), (nwork + 1) * 4, hipMemcpyHostToDevice));
  float *x, *out, *sc, *sc2;
  int8_t *q, *q2;
  uint32_t *part, *sink;
  adfl_slq_chunk* dch;
  uint4* junk;
  const int64_t junk_bytes = 512ll << 20;
  CK(hipMalloc(&x, L.total * 4));
  CK(hipMalloc(&out, L.total * 4));
  CK(hipMalloc(&q, L.total));
  CK(hipMalloc(&q2, L.total));
  CK(hipMalloc(&sc, 256 * 4));
  CK(hipMalloc(&sc2, 256 * 4));
  CK(hipMalloc(&part, nch * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&junk, junk_bytes));
  CK(hipMemset(junk, 0, junk_bytes));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  std::vector<float> hx(L.total, 0.0f);
  uint32_t r = 12345;
  for (int t = 0; t < 256; ++t)
    for (int64_t i = 0; i < L.sizes[t]; ++i) {
      r = r * 1664525u + 1013904223u;
      hx[L.offs[t] + i] = ((int32_t)r) * 1e-12f * (float)(1 + t % 7);
    }
  CK(hipMemcpy(x, hx.data(), L.total * 4, hipMemcpyHostToDevice));

  auto enc_prev = [&]() { CK(adfl_slq_encode_batched(x, dch, nch, 8, q, sc, part, nullptr)); };
  auto enc_res = [&]() { CK(adfl_slq_encode_batched_work(x, dch, nch, dwork, nwork, 8, q2, sc2, part, nullptr)); };
  auto dec = [&](const int8_t* qq, const float* ss) {
    CK(adfl_slq_dequantize_batched(qq, dch, nch, ss, out, nullptr));
  };
  // parity: the resident encode against the two-pass one
  enc_prev();
  enc_res();
  CK(hipDeviceSynchronize());
  std::vector<int8_t> a(L.total), b(L.total);
  std::vector<float> sa(256), sb(256);
  CK(hipMemcpy(a.data(), q, L.total, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), q2, L.total, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sa.data(), sc, 1024, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sb.data(), sc2, 1024, hipMemcpyDeviceToHost));
  bool same = std::equal(sa.begin(), sa.end(), sb.begin());
  for (int t = 0; t < 256 && same; ++t)
    same = std::equal(a.begin() + L.offs[t], a.begin() + L.offs[t] + L.sizes[t], b.begin() + L.offs[t]);
  printf("%s: %lld elements, %lld chunks, max %d chunks/tensor, %.1f%% of elements in tensors > %lld; "
         "one-launch work list: %lld tensors; work-entry payload+scales == two-pass: %s\n",
         L.name, (long long)n, (long long)nch, maxc, 100.0 * nbig / n, (long long)kSegMaxElems, (long long)nwork,
         same ? "yes" : "NO");

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"round trip two-pass", "round trip work entry", "encode two-pass", "encode work entry",
                         "decode"};
  const int nv = 5;
  std::vector<std::vector<double>> t(2 * nv);
  for (int rep = 0; rep < 60; ++rep)
    for (int v = 0; v < nv; ++v)
      for (int flush = 0; flush < 2; ++flush) {
        if (flush) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
        if (v == 4) enc_res();  // decode alone: after a fresh encode (the payload as the encode left it)
        CK(hipEventRecord(e0, 0));
        switch (v) {
          case 0: enc_prev(); dec(q, sc); break;
          case 1: enc_res(); dec(q2, sc2); break;
          case 2: enc_prev(); break;
          case 3: enc_res(); break;
          case 4: dec(q2, sc2); break;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep >= 5) t[2 * v + flush].push_back(ms);
      }
  for (int v = 0; v < nv; ++v) {
    const double w = median(t[2 * v]) * 1e3, f = median(t[2 * v + 1]) * 1e3;
    const double alg = v < 2 ? 14.0 * n : (v < 4 ? 9.0 * n : 5.0 * n);
    printf("  %-22s warm %7.2f us (%.3f of 8 TB/s)   flushed %7.2f us (%.3f)\n", names[v], w, alg / (w * 1e-6) / 8e12,
           f, alg / (f * 1e-6) / 8e12);
  }
  CK(hipFree(x));
  CK(hipFree(out));
  CK(hipFree(q));
  CK(hipFree(q2));
  CK(hipFree(sc));
  CK(hipFree(sc2));
  CK(hipFree(part));
  CK(hipFree(sink));
  CK(hipFree(dch));
  CK(hipFree(junk));
  CK(hipFree(dwork));
}
}  // namespace

int main() {
  run(equal_layout());
  run(loguniform_layout());
  return 0;
}
