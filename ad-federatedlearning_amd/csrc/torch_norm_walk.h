// torch_norm_walk.h — torch 2.10's fp32 L2 norm (the reference's QSGD / CNAT norm, quant.py:226,512) bit for
// bit, run in order: k_norm_walk, one block per tensor. Included by stoch_codec.hip (device code).
//
// The order. torch's CPU vector_norm(ord=2) over fp32 elements keeps 8 accumulators,
// acc[j] = fmaf(x[8i+j], x[8i+j], acc[j]) for i in order, then sums them left to right and runs the n % 8
// tail (tail_sum: a group of 4 rounded squares, then fmaf); a one-element tensor's norm is |x|
// (oracle/slq_oracle.c oracle_torch_l2_norm, pinned to torch itself). Each chain is a sequence of
// dependent roundings: run in order it costs one dependent FMA latency per step. This walker serves the
// short tensors (<= kWalkMax elements) of adfl_torch_norms (csrc/torch_norm.hip takes the long ones in
// parallel phases) and ADFL_NORM_L2_TORCH of adfl_stoch_norms_batched.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "adfl_slq.h"

namespace adfl_tn {

// The n % 8 tail after the lane sum, as torch's compiled scalar loop `b += x * x` runs it: a first group of 4
// (when there are 4 or more) with each square rounded and added in order (an in-order vectorised reduction),
// the rest with fma (oracle_torch_l2_norm). Also the whole sum below 8 elements, from b = 0.
__device__ __forceinline__ float tail_sum(const float* x, int64_t d, int64_t n, float b) {
  if (n - d >= 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float sq = x[d + k] * x[d + k];
      b = b + sq;
    }
    d += 4;
  }
  for (int64_t i = d; i < n; ++i) b = __builtin_fmaf(x[i], x[i], b);
  return b;
}

constexpr int64_t kWalkMax = 1 << 16;                     // tensors up to this size are walked (k_norm_walk)

// One block per tensor of at most kWalkMax elements (the phased kernels take the longer ones) runs the
// 8 chains in order — the reference's loop itself. Its four waves stream the tensor in 2048-element blocks
// into LDS buffers, chain-major (buf[c][step]), so lane c < 8 of wave 0 reads its chain back 4 steps
// per ds_read_b128, eight reads ahead of the dependent FMAs (about 6.6 cycles per step,
// MI355X_MICROARCH.md), while the next two blocks are in flight. A one-wave version with a 32-row
// register ring (2 KiB in flight) took 56 us on C3; with cross-lane shuffles instead of the LDS
// transpose 95 us, and with its loads under branches (an s_waitcnt vmcnt(0) after each) 312 us.
constexpr int kWalkThreads = 256;
#ifndef ADFL_TN_WALK_REGS
#define ADFL_TN_WALK_REGS 8
#endif
constexpr int kWalkRegs = ADFL_TN_WALK_REGS;
constexpr int kWalkBlock = kWalkThreads * kWalkRegs;  // 2048 elements: 256 steps of each chain
constexpr int kWalkBlockStride = kWalkBlock / 8 + 4;   // floats per chain row (+4: banks, 16-byte reads)

__global__ __launch_bounds__(kWalkThreads) void k_norm_walk(const float* __restrict__ x,
                                                           const adfl_slq_chunk* __restrict__ chunks,
                                                           int64_t max_n, float* __restrict__ norms,
                                                           double* __restrict__ norms64 = nullptr) {
  __shared__ __attribute__((aligned(16))) float buf[3][8 * kWalkBlockStride];
  const adfl_slq_chunk ch = chunks[blockIdx.x];
  if ((int64_t)blockIdx.x != ch.first_chunk) return;
  const int64_t n = (int64_t)(ch.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[blockIdx.x + ch.nchunks - 1].len;
  if (n > max_n) return;
  const float* xt = x + ch.start;
  const int tid = threadIdx.x, c = tid & 7, s0 = tid >> 3;
  if (n < 8) {
    if (tid == 0) {
      const float b = tail_sum(xt, 0, n, 0.0f);
      const float r = n == 1 ? __builtin_fabsf(xt[0]) : (float)__builtin_sqrt((double)b);  // one element: |x|
      if (norms) norms[ch.tensor] = r;
      if (norms64) norms64[ch.tensor] = r;
    }
    return;
  }
  const int64_t nv = n - n % 8, nblocks = (nv + kWalkBlock - 1) / kWalkBlock;
  // Buffer loads through a per-block descriptor whose range ends at nv: elements past it (and whole blocks
  // past the end) read as zeros, which leave the accumulators unchanged (fmaf(0, 0, a) == a), so loads and
  // stages carry no masks or branches. While block b is summed, block b + 1 is already in LDS (so the walk's
  // reads run on into it without a stall), block b + 2 is staged from registers loaded one block earlier
  // and block b + 3 loads (three LDS buffers, two register sets used alternately).
  const auto load = [&](float (&r)[kWalkRegs], int64_t blk) {
    const int64_t base = blk * kWalkBlock, left = nv - base;
    const int bytes = left <= 0 ? 0 : (int)(min(left, (int64_t)kWalkBlock) * 4);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xt + (left <= 0 ? 0 : base)), 0, bytes,
                                                      0x00020000);
#pragma unroll
    for (int i = 0; i < kWalkRegs; ++i)
      r[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (i * kWalkThreads + tid) * 4, 0, 0));
  };
  const auto stage = [&](const float (&r)[kWalkRegs], float* dst) {
#pragma unroll
    for (int i = 0; i < kWalkRegs; ++i) dst[c * kWalkBlockStride + (kWalkThreads / 8) * i + s0] = r[i];
  };
  // The walk: lanes 0-7 of wave 0 each run one chain through a ring of 16 float4 reads (64 steps) ahead of
  // the FMAs; a read is issued as each group of 4 FMAs retires its slot, and the ring's reads run from the
  // end of the block on into the head of the next one. sched_barrier keeps that order: left alone, the
  // scheduler batched the 16 reads and left the LDS latency exposed once per 64 steps (36 us on C3).
  constexpr int kGroups = kWalkBlock / 32, kRing = 16;
  static_assert(kGroups % kRing == 0, "the ring must restart at the same slot every block");
  float acc = 0.0f;
  float4 ring[kRing];
  const auto walk = [&](const float* cur, const float* nxt) {
    if (tid < 8) {
      const float4* l4 = reinterpret_cast<const float4*>(cur + c * kWalkBlockStride);
      const float4* n4 = reinterpret_cast<const float4*>(nxt + c * kWalkBlockStride);
#pragma unroll
      for (int j = 0; j < kGroups; ++j) {
        const float4 v = ring[j % kRing];
        acc = __builtin_fmaf(v.x, v.x, acc);
        acc = __builtin_fmaf(v.y, v.y, acc);
        acc = __builtin_fmaf(v.z, v.z, acc);
        acc = __builtin_fmaf(v.w, v.w, acc);
        ring[j % kRing] = j + kRing < kGroups ? l4[j + kRing] : n4[j + kRing - kGroups];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  float ra[kWalkRegs], rb[kWalkRegs];
  load(ra, 0);
  load(rb, 1);
  stage(ra, buf[0]);
  stage(rb, buf[1]);
  load(ra, 2);
  __syncthreads();
  if (tid < 8) {
    const float4* l4 = reinterpret_cast<const float4*>(buf[0] + c * kWalkBlockStride);
#pragma unroll
    for (int j = 0; j < kRing; ++j) ring[j] = l4[j];
  }
  for (int64_t blk = 0; blk < nblocks; blk += 2) {  // block-uniform control flow throughout
    load(rb, blk + 3);
    walk(buf[blk % 3], buf[(blk + 1) % 3]);
    stage(ra, buf[(blk + 2) % 3]);
    __syncthreads();
    if (blk + 1 >= nblocks) break;
    load(ra, blk + 4);
    walk(buf[(blk + 1) % 3], buf[(blk + 2) % 3]);
    stage(rb, buf[(blk + 3) % 3]);
    __syncthreads();
  }
  if (tid < 64) {  // wave 0: lane sum left to right, the n % 8 tail, sqrt
    float b = __shfl(acc, 0, 64);
#pragma unroll
    for (int j = 1; j < 8; ++j) b = b + __shfl(acc, j, 64);
    if (tid == 0) {
      b = tail_sum(xt, nv, n, b);
      const float r = (float)__builtin_sqrt((double)b);  // correctly rounded fp32 sqrt
      if (norms) norms[ch.tensor] = r;
      if (norms64) norms64[ch.tensor] = r;
    }
  }
}

}  // namespace adfl_tn
