// torch_sum_order.h — the fp32 summation order of torch 2.10's CPU `torch.sum(torch.stack(rows), dim=0)`,
// restated for the mean kernels so that their output is bit-identical to the reference's aggregates:
//   simple_aggregate       Src/ADFL/model.py:229-231   torch.sum(torch.stack(contributions), dim=0) / K
//   peer mean              Examples/ray_ad.py:188, Src/ADFL/Client/async_peer.py:172-174   stack(...).mean(0)
//                          (CPU mean = the same sum, then a true division by K)
//
// What torch computes (aten/src/ATen/native/cpu/SumKernel.cpp, cascade_sum; the AVX2 kernel on any x86-64
// host with AVX2 — ATen registers no AVX-512 variant of sum_stub, so Vectorized<float> is 8 wide). A stack of
// K tensors of n elements is a contiguous [K, n] array reduced over K (the outer dim). For element j of a
// tensor (0 <= j < n), with d_s the value of row s (0 <= s < K, in list order):
//  * SEQ  — j in a full group of 32 columns (4 vectors x 8; for 2 <= n < 8, groups of 4 scalar columns),
//           i.e. j < (n >= 8 ? n & ~31 : n & ~3): multi_row_sum over the K rows. Rows are added in order
//           into level 0, starting from +0; after every 16th row level 0 is added into level 1 and reset to
//           +0; after every 256th row level 1 likewise into level 2, after every 4096th level 2 into 3 (the
//           cascade's level_step is 2^max(4, ceil_log2(K)/4) = 16 for K < 2^20). At the end
//           ((level0 + level1) + level2) + level3.
//  * ILP4 — every other column of an n >= 2 tensor (its last n % 32 elements, or n % 4 for n < 8), and a
//           one-element tensor when K < 8: row_sum with ilp_factor 4 — partial p (0..3) sums rows 4g+p over
//           g < K/4 with the same cascade over g; the K % 4 leftover rows are then added to partial 0 in
//           order; the result is ((p0 + p1) + p2) + p3.
//  * INNER — a one-element tensor (n == 1) with K >= 8: the K values are one contiguous row
//           (vectorized_inner_sum): V = K/8 vectors of 8, lane l's partial is the ILP4 sum of d_{8v+l} over
//           v < V; then acc = +0, the K % 8 leftover values added in order, then the 8 lane partials in
//           lane order.
// Pinned bit for bit against torch itself and against the reference's simple_aggregate executed in place
// (oracle/slq_oracle.c oracle_torch_sum_col; tests/golden/aggregate.npz, tests/test_sum_order_golden.py).
// Every thread of a mean kernel calls these with its own element; K is the same for the whole launch.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace adfl_sum {

enum Mode : int { kSeq = 0, kIlp4 = 1, kInner = 2 };

// Largest K whose cascade step is 16 (ceil_log2(K) / 4 <= 4); the C ABI refuses more rows.
constexpr int kMaxRows = 1 << 19;

// The order element j (0-based, within its tensor of n elements) is summed in.
__device__ __forceinline__ int mode_of(int64_t j, int64_t n, int k) {
  if (n == 1) return k >= 8 ? kInner : kIlp4;
  const int64_t seq_end = n >= 8 ? (n & ~(int64_t)31) : (n & ~(int64_t)3);
  return j < seq_end ? kSeq : kIlp4;
}

// First tensor-relative index that is not SEQ.
__device__ __forceinline__ int64_t seq_end(int64_t n) {
  if (n == 1) return 0;
  return n >= 8 ? (n & ~(int64_t)31) : (n & ~(int64_t)3);
}

// multi_row_sum over count values get(off + stride * i), i < count (one column, nrows = 1).
template <class Get>
__device__ __forceinline__ float cascade(const Get& get, int count, int stride, int off) {
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
  for (int i = 0; i < count;) {
    a0 = a0 + get(off + stride * i);
    ++i;
    if ((i & 15) == 0) {  // a full block of 16 rows completed: fold the levels
      a1 = a1 + a0;
      a0 = 0.0f;
      if ((i & 0xF0) == 0) {
        a2 = a2 + a1;
        a1 = 0.0f;
        if ((i & 0xF00) == 0) {
          a3 = a3 + a2;
          a2 = 0.0f;
        }
      }
    }
  }
  a0 = a0 + a1;
  a0 = a0 + a2;
  return a0 + a3;
}

// row_sum (ilp_factor 4) over count values get(off + stride * i).
template <class Get>
__device__ __forceinline__ float ilp4(const Get& get, int count, int stride, int off) {
  const int g = count >> 2;
  float p0 = cascade(get, g, 4 * stride, off);
  const float p1 = cascade(get, g, 4 * stride, off + stride);
  const float p2 = cascade(get, g, 4 * stride, off + 2 * stride);
  const float p3 = cascade(get, g, 4 * stride, off + 3 * stride);
  for (int i = 4 * g; i < count; ++i) p0 = p0 + get(off + stride * i);
  p0 = p0 + p1;
  p0 = p0 + p2;
  return p0 + p3;
}

// The torch-order sum of the k row values get(0) .. get(k-1) of one element in `mode`.
template <class Get>
__device__ __forceinline__ float sum_elem(const Get& get, int k, int mode) {
  if (mode == kSeq) return cascade(get, k, 1, 0);
  if (mode == kIlp4) return ilp4(get, k, 1, 0);
  const int v = k >> 3;  // kInner
  float acc = 0.0f;
  for (int i = 8 * v; i < k; ++i) acc = acc + get(i);
  for (int l = 0; l < 8; ++l) acc = acc + ilp4(get, v, 8, l);
  return acc;
}

// SEQ order over register tiles of NV float4 per lane (the mean kernels' vector paths): level 0 takes the
// rows; step() after each row folds the levels as multi_row_sum does. DEEP (K >= 256) carries levels 2-3;
// otherwise they stay +0 and the final additions of +0 are exact no-ops (no level is ever -0: each starts
// at +0 and only receives round-to-nearest sums, which are -0 only when both addends are).
__device__ __forceinline__ float4 add4s(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int NV, bool DEEP>
struct SeqTile {
  float4 l0[NV], l1[NV], l2[DEEP ? NV : 1], l3[DEEP ? NV : 1];
  int rows;

  __device__ __forceinline__ void init() {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < NV; ++j) l0[j] = l1[j] = z;
    if (DEEP) {
#pragma unroll
      for (int j = 0; j < NV; ++j) l2[j] = l3[j] = z;
    }
    rows = 0;
  }
  __device__ __forceinline__ void add(int j, float4 v) { l0[j] = add4s(l0[j], v); }
  // after a row has been added to every l0[j]
  __device__ __forceinline__ void step() {
    ++rows;
    if ((rows & 15) != 0) return;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      l1[j] = add4s(l1[j], l0[j]);
      l0[j] = z;
    }
    if (!DEEP || (rows & 0xF0) != 0) return;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      l2[j] = add4s(l2[j], l1[j]);
      l1[j] = z;
    }
    if ((rows & 0xF00) != 0) return;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      l3[j] = add4s(l3[j], l2[j]);
      l2[j] = z;
    }
  }
  __device__ __forceinline__ float4 result(int j) const {
    float4 r = add4s(l0[j], l1[j]);
    if (DEEP) r = add4s(add4s(r, l2[j]), l3[j]);
    return r;
  }
};

}  // namespace adfl_sum
