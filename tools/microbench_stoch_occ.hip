// microbench_stoch_occ.hip — occupancy A/B of the C2 stochastic quantize kernels. The product's
// k_cnat_quantize<4> / k_qsgd_quantize<4> take 76-77 VGPRs (6 waves per SIMD); the same bodies compiled under
// amdgpu_waves_per_eu(7 / 8) (<= 72 / 64 VGPRs) and with 2 Philox blocks per batch instead of 4, timed on a
// 2^28-element tensor with the Infinity Cache flushed, outputs checked byte for byte against the product.
// Not part of the product; it #includes the product source.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/microbench_stoch_occ \
//         tools/microbench_stoch_occ.hip ad-federatedlearning_amd/csrc/slq_codec.hip
#include "../ad-federatedlearning_amd/csrc/stoch_codec.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
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

__global__ void k_fill(float* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = ((float)(h & 0xffffff) / 16777216.0f - 0.5f) * 4e-3f;
  }
}

// k_cnat_quantize's body under an occupancy attribute
template <int PB, int WPE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void k_cnat_occ(
    const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, int min_e, int max_e, Uniforms U,
    int8_t* __restrict__ exps, int8_t* __restrict__ signs, double* __restrict__ partials) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const float* xc = x + c.start;
  int8_t* ex = exps + c.start;
  int8_t* sg = signs + c.start;
  const int head = chunk_head4(c.start, c.len);
  const int n4 = (c.len - head) >> 2;
  const auto fast = [=](float xv, float uv, bool& bad) { return cnat_exp_fast(xv, uv, min_e, max_e, bad); };
  const auto exact = [=](float xv, float uv) { return cnat_exp_exact(xv, uv, min_e, max_e); };
  NormAcc<ADFL_NORM_L2> acc;
  quantize_chunk_vec<PB>(reinterpret_cast<const float4*>(xc + head), n4, c.start + head, U,
                         reinterpret_cast<uint32_t*>(ex + head), reinterpret_cast<uint32_t*>(sg + head), fast, exact,
                         false, &acc);
  const int i = edge_elem(head, head + (n4 << 2), c.len);
  if (i >= 0) {
    const float v = xc[i];
    ex[i] = (int8_t)exact(v, U.one(c.start + i));
    sg[i] = (int8_t)sign_byte(v);
    acc.add(v);
  }
  acc.flush(partials, blockIdx.x);
}

// k_qsgd_quantize's body under an occupancy attribute
template <int PB, int WPE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void k_qsgd_occ(
    const float* __restrict__ x, const adfl_slq_chunk* __restrict__ chunks, float s, const float* __restrict__ norms,
    Uniforms U, uint8_t* __restrict__ levels, int8_t* __restrict__ signs) {
  const adfl_slq_chunk c = chunks[gridDim.x - 1 - blockIdx.x];
  const float norm = norms[c.tensor];
  uint8_t* lv = levels + c.start;
  int8_t* sg = signs + c.start;
  if (norm == 0.0f) {
    fill_zero_norm(lv, sg, c.len);
    return;
  }
  const Div d = make_div(norm);
  const float* xc = x + c.start;
  const int head = chunk_head4(c.start, c.len);
  const int n4 = (c.len - head) >> 2;
  const auto fast = [&](float xv, float uv, bool& bad) { return qsgd_level_fast(xv, s, d, uv, bad); };
  const auto exact = [&](float xv, float uv) { return qsgd_level_exact(xv, s, norm, uv); };
  quantize_chunk_vec<PB>(reinterpret_cast<const float4*>(xc + head), n4, c.start + head, U,
                         reinterpret_cast<uint32_t*>(lv + head), reinterpret_cast<uint32_t*>(sg + head), fast, exact,
                         !d.fast, (NormAcc<ADFL_NORM_L2>*)nullptr);
  const int i = edge_elem(head, head + (n4 << 2), c.len);
  if (i >= 0) {
    lv[i] = (uint8_t)exact(xc[i], U.one(c.start + i));
    sg[i] = (int8_t)sign_byte(xc[i]);
  }
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

void run(int reps) {
  const int64_t n = 1ll << 28;
  int64_t off = 0;
  const int64_t nch = adfl_slq_build_chunks(&off, &n, 1, nullptr, 0);
  std::vector<adfl_slq_chunk> ch(nch);
  adfl_slq_build_chunks(&off, &n, 1, ch.data(), nch);
  float *x, *norm;
  int8_t *e1, *s1, *e2, *s2;
  double *p1, *p2;
  adfl_slq_chunk* dch;
  uint4* junk;
  uint32_t* sink;
  const int64_t junk_bytes = 512ll << 20;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&norm, 4));
  CK(hipMalloc(&e1, n));
  CK(hipMalloc(&s1, n));
  CK(hipMalloc(&e2, n));
  CK(hipMalloc(&s2, n));
  CK(hipMalloc(&p1, nch * 8));
  CK(hipMalloc(&p2, nch * 8));
  CK(hipMalloc(&dch, nch * sizeof(adfl_slq_chunk)));
  CK(hipMalloc(&junk, junk_bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(junk, 0, junk_bytes));
  CK(hipMemcpy(dch, ch.data(), nch * sizeof(adfl_slq_chunk), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n);
  const float nv = 3.0f;
  CK(hipMemcpy(norm, &nv, 4, hipMemcpyHostToDevice));
  const Uniforms U{nullptr, 1234, 0};
  const int min_e = -128, max_e = 127;
  const float s = 255.0f;
  const dim3 grid((unsigned)nch), block(kBlock);
  auto* l1 = reinterpret_cast<uint8_t*>(e1);
  auto* l2 = reinterpret_cast<uint8_t*>(e2);
  struct Var {
    std::string name;
    bool cnat;
    std::function<void(int8_t*, int8_t*, double*)> f;
  };
  std::vector<Var> vars = {
      {"cnat product <4> (76 VGPR)", true,
       [&](int8_t* e, int8_t* g, double* p) {
         hipLaunchKernelGGL(k_cnat_quantize<kPbQuantize>, grid, block, 0, 0, x, dch, min_e, max_e, U, e, g, p);
       }},
      {"cnat <4> waves_per_eu 7", true,
       [&](int8_t* e, int8_t* g, double* p) {
         hipLaunchKernelGGL((k_cnat_occ<4, 7>), grid, block, 0, 0, x, dch, min_e, max_e, U, e, g, p);
       }},
      {"cnat <4> waves_per_eu 8", true,
       [&](int8_t* e, int8_t* g, double* p) {
         hipLaunchKernelGGL((k_cnat_occ<4, 8>), grid, block, 0, 0, x, dch, min_e, max_e, U, e, g, p);
       }},
      {"cnat <2> waves_per_eu 8", true,
       [&](int8_t* e, int8_t* g, double* p) {
         hipLaunchKernelGGL((k_cnat_occ<2, 8>), grid, block, 0, 0, x, dch, min_e, max_e, U, e, g, p);
       }},
      {"qsgd product <4> (77 VGPR)", false,
       [&](int8_t* e, int8_t* g, double*) {
         hipLaunchKernelGGL(k_qsgd_quantize<kPbQuantize>, grid, block, 0, 0, x, dch, s, norm, U,
                            reinterpret_cast<uint8_t*>(e), g);
       }},
      {"qsgd <4> waves_per_eu 7", false,
       [&](int8_t* e, int8_t* g, double*) {
         hipLaunchKernelGGL((k_qsgd_occ<4, 7>), grid, block, 0, 0, x, dch, s, norm, U, reinterpret_cast<uint8_t*>(e), g);
       }},
      {"qsgd <4> waves_per_eu 8", false,
       [&](int8_t* e, int8_t* g, double*) {
         hipLaunchKernelGGL((k_qsgd_occ<4, 8>), grid, block, 0, 0, x, dch, s, norm, U, reinterpret_cast<uint8_t*>(e), g);
       }},
      {"qsgd <2> waves_per_eu 8", false,
       [&](int8_t* e, int8_t* g, double*) {
         hipLaunchKernelGGL((k_qsgd_occ<2, 8>), grid, block, 0, 0, x, dch, s, norm, U, reinterpret_cast<uint8_t*>(e), g);
       }},
  };
  (void)l1;
  (void)l2;
  // parity: every variant against its product kernel
  std::vector<int8_t> ha(n), hb(n), sa(n), sb(n);
  std::vector<double> pa(nch), pb(nch);
  for (size_t k = 0; k < vars.size(); ++k) {
    const size_t ref = vars[k].cnat ? 0 : 4;
    CK(hipMemset(e1, 0x55, n));
    CK(hipMemset(s1, 0x55, n));
    CK(hipMemset(p1, 0, nch * 8));
    vars[ref].f(e1, s1, p1);
    CK(hipMemset(e2, 0x33, n));
    CK(hipMemset(s2, 0x33, n));
    CK(hipMemset(p2, 0, nch * 8));
    vars[k].f(e2, s2, p2);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ha.data(), e1, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), e2, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sa.data(), s1, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sb.data(), s2, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(pa.data(), p1, nch * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(pb.data(), p2, nch * 8, hipMemcpyDeviceToHost));
    const bool ok = ha == hb && sa == sb && (!vars[k].cnat || std::memcmp(pa.data(), pb.data(), nch * 8) == 0);
    printf("  %-28s output == product: %s\n", vars[k].name.c_str(), ok ? "yes" : "NO");
  }
  hipEvent_t a0, a1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  std::vector<std::vector<double>> t(vars.size());
  for (int rep = 0; rep < reps; ++rep)
    for (size_t k = 0; k < vars.size(); ++k) {
      hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk_bytes / 16, sink);
      CK(hipEventRecord(a0, 0));
      vars[k].f(e1, s1, p1);
      CK(hipEventRecord(a1, 0));
      CK(hipEventSynchronize(a1));
      float ms;
      CK(hipEventElapsedTime(&ms, a0, a1));
      if (rep >= 3) t[k].push_back(ms * 1e3);
    }
  for (size_t k = 0; k < vars.size(); ++k) {
    const double m = median(t[k]);
    printf("  %-28s C2 quantize %8.1f us  (6 B/elem: %.3f of 8 TB/s)\n", vars[k].name.c_str(), m,
           6.0 * n / (m * 1e-6) / 8e12);
  }
}
}  // namespace

int main(int argc, char** argv) {
  run(argc > 1 ? atoi(argv[1]) : 15);
  return 0;
}
