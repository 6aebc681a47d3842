// torch_norm_lb.h — torch's fp32 L2 norm (the reference's QSGD / CNAT norm, quant.py:226,512) bit for bit,
// tile-parallel at streaming rate. Included by stoch_codec.hip (device code + launch helper).
//
// The order. torch 2.10's CPU vector_norm(ord=2) over fp32 elements keeps 8 accumulators,
// acc[j] = fmaf(x[8i+j], x[8i+j], acc[j]) for i in order, then sums them left to right and runs the n % 8
// tail (tail_sum: a group of 4 rounded squares, then fmaf; oracle/slq_oracle.c oracle_torch_l2_norm,
// pinned to torch itself). Each chain is a
// sequence of dependent roundings: run in order (k_norm_walk) it costs one dependent FMA latency per step.
//
// Why it parallelises. A step is RN32(acc + p) with p = x*x exact (48 bits: exact in fp64). While acc stays
// in one binade, acc = A * u with u = 2^(g-23) the binade's ulp and A an integer below 2^24 (g = -126 also
// covers the subnormals, same u). If A + p/u < 2^24 the step rounds on the grid u, so it is
// A <- A + R(p/u): an integer increment that depends on acc only through the tie-to-even rule (R(v) = v
// rounded to nearest; an exact tie v = f + 1/2 goes to whichever of f, f + 1 makes A + k even). So, for a
// run of steps with no tie, given the grid, the run adds the integer sum of its R(p/u) — order-free — and
// it is exact as long as the start A plus that sum stays below 2^24 (every partial sum is then below it
// too, the increments being >= 0 and R(v) >= v - 1/2). tools/torch_norm_proto.c checks this model against
// the sequential chain on random, tie-heavy, subnormal, overflow and NaN / inf data.
//
// Short tensors (<= kWalkMax elements): k_norm_walk, one block per tensor running the chains in order, the
// rows written to LDS chain-major so each chain reads 4 steps per ds_read_b128 ahead of its FMA chain.
//
// Long tensors: k_norm_torch. The 8 chains run over tiles of kTile = 16384 elements (2048 steps of each
// chain; two chunks — one ticket per chunk, the tile's first chunk's block does the work), taken in ticket
// order; lane l of wave w reads elements w * 64 * kRegs + 64 * i + l (i < kRegs): always chain l & 7,
// 256 B contiguous per wave-instruction, no alignment requirement. Each tile publishes, in its record,
// three kinds of values (decoupled look-back):
//   1  fp64 sums of x^2 per chain (aggS);
//   2  the fp64 inclusive prefix, and for each chain the integer totals of its steps under one or two
//      candidate grids — the binade(s) the fp32 accumulator can be in at the tile's start, predicted from
//      the fp64 prefix (the fp32 chain runs at most a few % below the exact sum: 7.2% at 2^28 elements
//      of randn, so the candidates span [S(1 - 1/8), S(1 + 2^-16)]); a tile with a tie, a step at or
//      above 2^24 ulps, or a non-finite value has no valid total;
//   3  the chain's exact fp32 accumulator after the tile.
// A tile's exclusive state = the nearest predecessor with 3 published plus the totals of the tiles in
// between for that accumulator's grid, when all of them hold one and the sum stays below 2^24. If not (a
// crossing into the next binade, a tie, a miss of the predictor) the tile waits for the first tile from the
// base's side that breaks it to publish 3, and looks again. Its own inclusive state is its exclusive state
// plus its total under the same rule; otherwise lanes 0..7 run the tile's steps with fmaf from LDS — the
// reference arithmetic itself. Tile size and round size were measured (profiles/r04/torch_norm/: C2
// 4.5 ms at 4096-element tiles, 2.4 at 8192, 2.1 at 16384 with 512 threads, 3.2 at 32768).
//
// Hand-off between blocks: every published value is an 8-byte granule {tag, 32-bit value} written and read
// with relaxed agent-scope atomics (global sc1 stores / loads: write-through, L1 bypassed), so the data is
// its own flag — no release / acquire fence anywhere (cdna_hip_programming.md Guideline 16, R2: an agent
// fence costs 1.7-7 us per episode; the first version of this kernel, with acquire polls and
// __threadfence publishes, ran C2's norm in 60 ms). A record is 5 rows of 8 granules (one per chain):
// aggS, inclS (fp32 prefix sums: the predictor), two candidate totals, and the exact accumulator.
//
// Scratch: a header (ticket, done, epoch) and one 320-byte record per tile, zeroed once when allocated.
// Granules carry tag = epoch + 1 of their launch; the last block to finish resets ticket and done and
// bumps the epoch, so the scratch is ready for the next launch without a memset (graph replays too: the
// epoch lives in the scratch). One scratch per stream. Every wait is bounded (kSpinCap): a broken
// invariant ends in NaN norms and hdr->error, not a hang.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "adfl_slq.h"

namespace adfl_tn {

#ifndef ADFL_TN_THREADS
#define ADFL_TN_THREADS 512
#endif
constexpr int kThreads = ADFL_TN_THREADS;
constexpr int kWaves = kThreads / 64;
#ifndef ADFL_TN_REGS
#define ADFL_TN_REGS 32
#endif
constexpr int kRegs = ADFL_TN_REGS;                             // dwords per lane
constexpr int kTile = kThreads * kRegs;                         // 16384 elements: 2048 steps per chain
// a tile is part of a chunk (kTilesPerChunk tiles per chunk, one ticket each) or whole chunks (kChunksPerTile;
// one ticket per chunk, the tile's first chunk does the work, the others exit)
constexpr int kTilesPerChunk = kTile <= ADFL_SLQ_CHUNK_ELEMS ? ADFL_SLQ_CHUNK_ELEMS / kTile : 1;
constexpr int kChunksPerTile = kTile >= ADFL_SLQ_CHUNK_ELEMS ? kTile / ADFL_SLQ_CHUNK_ELEMS : 1;
constexpr int kWin = 8;                                         // predecessors per look-back round (x 8 chains)
#ifndef ADFL_TN_BATCH
#define ADFL_TN_BATCH 1
#endif
constexpr int kBatch = ADFL_TN_BATCH;                           // windows per look-back round (one round trip)
constexpr int kMaxD = 64;                                       // predecessors whose candidates are kept
static_assert(kMaxD % (kWin * kBatch) == 0 || kWin * kBatch > kMaxD, "rounds tile the kept window");
constexpr double kMagic = 6755399441055744.0;                   // 1.5 * 2^52: fma(d, ds, kMagic) - kMagic = rint
constexpr double kTop = 16777216.0;                             // 2^24
constexpr int kNoGrid = -1024;
constexpr uint32_t kCodeNaN = 254, kCodeBad = 255;              // candidate codes: 0..253 = grid + 126
constexpr long long kSpinCap = 1ll << 20;                       // polls (about 1 us each): a second
constexpr unsigned long long kChain0 = 0x0101010101010101ull;  // ballot bits of the chain-0 lanes

static_assert(kTilesPerChunk * kTile == ADFL_SLQ_CHUNK_ELEMS * kChunksPerTile, "tiles and chunks nest");

typedef __attribute__((address_space(1))) unsigned long long gu64;

struct Header {
  unsigned long long ticket, done, epoch, error;
  unsigned long long stats[4];  // look-back retries, sequential tiles, far misses, failed compositions (tools)
};

struct Rec {                      // granules {tag << 32 | value}, one per chain
  unsigned long long aggS[8];     // fp32 sum of x^2 over the tile's steps of the chain
  unsigned long long inclS[8];    // fp32 inclusive prefix of aggS (the predictor)
  unsigned long long cand[2][8];  // code << 24 | total: the tile's steps in ulps of a candidate grid
  unsigned long long incl[8];     // the chain's exact fp32 accumulator after the tile
};
static_assert(sizeof(Rec) == 320, "record layout");

__device__ __forceinline__ void put(unsigned long long* p, uint32_t tag, uint32_t v) {
  __hip_atomic_store((gu64*)p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long get(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool has(unsigned long long g, uint32_t tag) { return (uint32_t)(g >> 32) == tag; }
__device__ __forceinline__ float fval(unsigned long long g) { return __uint_as_float((uint32_t)g); }

__device__ __forceinline__ double pow2(int k) { return __longlong_as_double((long long)(k + 1023) << 52); }

// binade of a finite fp32 accumulator >= 0, as its grid exponent g (ulp 2^(g-23))
__device__ __forceinline__ int grid_of(float a) {
  const uint32_t ef = __float_as_uint(a) >> 23;
  return ef <= 1u ? -126 : (int)ef - 127;
}

// the grid an fp32 accumulator near the value a >= 0 would be on
__device__ __forceinline__ int grid_of_d(double a) {
  if (!(a < 0x1p127)) return 127;
  if (a < 0x1p-125) return -126;
  return (int)((__double_as_longlong(a) >> 52) & 0x7ff) - 1023;
}

// total of a candidate granule for grid g, or false
__device__ __forceinline__ bool pick(unsigned long long c0, unsigned long long c1, int g, double& total) {
  if (g == kNoGrid) return false;
  const uint32_t want = (uint32_t)(g + 126);
  const uint32_t v0 = (uint32_t)c0, v1 = (uint32_t)c1;
  const uint32_t v = (v0 >> 24) == want ? v0 : v1;
  if ((v >> 24) != want) return false;
  total = (double)(v & 0xffffffu);
  return true;
}

__device__ __forceinline__ bool spin(long long& n, int* err) {  // false once the cap ran out
  if (++n > kSpinCap) {
    *err = 1;
    return false;
  }
  __builtin_amdgcn_s_sleep(2);
  return true;
}

// per-chain OR of a lane predicate over the 8 lanes of each chain (result valid in every lane)
__device__ __forceinline__ bool chain_any(bool p, int c) { return ((__ballot(p) >> c) & kChain0) != 0ull; }

// for each chain, the first predecessor slot q whose lane has p (kWin if none)
__device__ __forceinline__ int chain_first(bool p, int c) {
  const unsigned long long m = (__ballot(p) >> c) & kChain0;
  return m ? (__builtin_ctzll(m) >> 3) : kWin;
}

__device__ __forceinline__ double chain_sum(double v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// integer total (in ulps of grid g) and tie flag of a lane's elements
__device__ __forceinline__ double lane_total(const float (&e)[kRegs], int g, bool& tie) {
  const double sc = pow2(23 - g);
  double T = 0.0;
  bool t = false;
#pragma unroll
  for (int i = 0; i < kRegs; ++i) {
    const double d = (double)e[i];
    const double ds = d * sc;
    const double kd = __fma_rn(d, ds, kMagic) - kMagic;  // rint(d * d * sc): exact below 2^51
    const double r = __fma_rn(d, ds, -kd);                // v - rint(v), exact when v < 2^24
    t |= __builtin_fabs(r) == 0.5;
    T += kd;
  }
  tie = t;
  return T;
}

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
constexpr int kStageStride = kTile / 8 + 4;               // a slow tile staged chain-major (+4: banks, 16 B)

// One block per tensor of at most kWalkMax elements (the look-back kernel takes the longer ones) runs the
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

__global__ __launch_bounds__(kThreads) void k_norm_torch(const float* __restrict__ x,
                                                         const adfl_slq_chunk* __restrict__ chunks, int64_t ntiles,
                                                         Header* hdr, Rec* recs, float* __restrict__ norms) {
  __shared__ unsigned long long s_t, s_epoch;
  __shared__ double s_part[kWaves][8][3];
  __shared__ int s_tie[kWaves][8][2];
  __shared__ double s_aggS[8], s_exclS[8], s_T[8][2];
  __shared__ int s_g[8][2], s_ok[8][2];
  __shared__ float s_excl[8], s_inc[8];
  __shared__ int s_slow, s_err, s_retry, s_why[3];
  __shared__ __attribute__((aligned(16))) float s_stage[8 * kStageStride];  // also the walker's LDS
  __shared__ unsigned long long s_cand[kMaxD][8][2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c = lane & 7, q = lane >> 3;
  if (tid == 0) {
    s_t = __hip_atomic_fetch_add(&hdr->ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_epoch = __hip_atomic_load(&hdr->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_err = 0;
    s_slow = 0;
    s_retry = 0;
    s_why[0] = s_why[1] = s_why[2] = 0;
  }
  __syncthreads();
  const int64_t t = (int64_t)s_t;
  const unsigned long long epoch = s_epoch;
  const uint32_t tag = (uint32_t)(epoch + 1);  // zeroed scratch: tag 0 is never current
  if (t < ntiles) {
    const int64_t ci = t / kTilesPerChunk;
    const int h = (int)(t % kTilesPerChunk);
    const adfl_slq_chunk ch = chunks[ci];
    const int kc = (int)(ci - ch.first_chunk);
    const int64_t tbase = ch.start - (int64_t)kc * ADFL_SLQ_CHUNK_ELEMS;  // the tensor's first element
    const int64_t n = (int64_t)(ch.nchunks - 1) * ADFL_SLQ_CHUNK_ELEMS + chunks[ch.first_chunk + ch.nchunks - 1].len;
    const int64_t nv = n >= 8 ? n - n % 8 : 0;
    const int64_t e0 = (int64_t)kc * ADFL_SLQ_CHUNK_ELEMS + (int64_t)h * kTile;
    const int len = (int)(nv - e0 <= 0 ? 0 : (nv - e0 < kTile ? nv - e0 : kTile));
    const int ti = kChunksPerTile > 1 ? kc / kChunksPerTile : kc * kTilesPerChunk + h;  // tile index in the tensor
    if (kChunksPerTile > 1 && kc % kChunksPerTile != 0) goto finish;  // not a tile's first chunk
    if (n <= kWalkMax) goto finish;  // block-uniform: short tensors are k_norm_walk's
    {
    Rec* me = recs + t;
    const float* xt = x + tbase + e0;

    float e[kRegs];
    if (len > 0) {  // unconditional loads (index clamped), then zeros past the end: they add nothing
#pragma unroll
      for (int i = 0; i < kRegs; ++i) e[i] = xt[min(wave * 64 * kRegs + 64 * i + lane, len - 1)];
#pragma unroll
      for (int i = 0; i < kRegs; ++i)
        if (wave * 64 * kRegs + 64 * i + lane >= len) e[i] = 0.0f;
    } else {
#pragma unroll
      for (int i = 0; i < kRegs; ++i) e[i] = 0.0f;
    }
    // ---- aggS: fp64 sums of squares per chain, published as fp32
    double S = 0.0;
#pragma unroll
    for (int i = 0; i < kRegs; ++i) {
      const double d = (double)e[i];
      S = __fma_rn(d, d, S);
    }
    S = chain_sum(S);
    if (q == 0) s_part[wave][c][0] = S;
    __syncthreads();
    if (tid < 8) {
      double a = s_part[0][tid][0];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) a += s_part[w][tid][0];
      s_aggS[tid] = a;
      put(&me->aggS[tid], tag, __float_as_uint((float)a));
    }

    // ---- the fp64 sum of all earlier steps of each chain (wave 0; lane = 8 * predecessor slot + chain).
    // Rounds of kBatch windows (64 predecessors): all their granules are loaded at once, so a round costs
    // one memory round trip — the rate at which a tile can see past tiles still in flight.
    if (wave == 0) {
      double accS = 0.0;
      bool done = ti == 0;
      for (int r = 0; __any(!done); ++r) {
        unsigned long long gi[kBatch], ga[kBatch];
        for (long long ns = 0;;) {
#pragma unroll
          for (int j = 0; j < kBatch; ++j) {  // unconditional loads (clamped to the tensor's first tile)
            const int d = min((r * kBatch + j) * kWin + q, ti - 1);
            gi[j] = get(&(me - kChunksPerTile * (1 + d))->inclS[c]);
            ga[j] = get(&(me - kChunksPerTile * (1 + d))->aggS[c]);
          }
          bool ok = true, fnd = done;
#pragma unroll
          for (int j = 0; j < kBatch; ++j) {
            const int d = (r * kBatch + j) * kWin + q;
            const bool valid = ti - 1 - d >= 0;
            const int qb = chain_first(!valid || has(gi[j], tag), c);  // a prefix, or the tensor start
            ok &= fnd || q >= qb || has(ga[j], tag);
            fnd = fnd || qb < kWin;
          }
          if (__all(ok) || !spin(ns, &s_err)) break;
        }
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const int d = (r * kBatch + j) * kWin + q;
          const bool valid = ti - 1 - d >= 0;
          const int qb = chain_first(!valid || has(gi[j], tag), c);
          double v = 0.0;
          if (!done) {
            if (q < qb) v = (double)fval(ga[j]);
            else if (q == qb && valid) v = (double)fval(gi[j]);
          }
          accS += chain_sum(v);
          done = done || qb < kWin;
        }
      }
      if (q == 0) s_exclS[c] = accS;
    }
    __syncthreads();
    // ---- candidate grids for the chain's fp32 accumulator at the tile's start
    if (tid < 8) {
      int g0 = -126, g1 = kNoGrid;
      if (ti > 0) {
        const double Sx = s_exclS[tid];
        g0 = grid_of_d(Sx * (1.0 + 0x1p-16));
        const int gl = grid_of_d(Sx * 0.875);
        if (gl != g0) g1 = gl;
      }
      s_g[tid][0] = g0;
      s_g[tid][1] = g1;
    }
    __syncthreads();
    // ---- integer totals under the candidates
    {
      const int g0 = s_g[c][0], g1 = s_g[c][1];
      bool tie0, tie1 = false;
      const double T0 = chain_sum(lane_total(e, g0, tie0));
      double T1 = 0.0;
      if (__any(g1 != kNoGrid)) T1 = chain_sum(lane_total(e, g1 == kNoGrid ? g0 : g1, tie1));
      const bool a0 = chain_any(tie0, c), a1 = chain_any(tie1, c);
      if (q == 0) {
        s_part[wave][c][1] = T0;
        s_part[wave][c][2] = T1;
        s_tie[wave][c][0] = a0;
        s_tie[wave][c][1] = a1;
      }
    }
    __syncthreads();
    if (tid < 8) {
      const bool nan = __builtin_isnan(s_aggS[tid]);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int g = s_g[tid][k];
        double T = s_part[0][tid][1 + k];
        bool tie = s_tie[0][tid][k];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) {
          T += s_part[w][tid][1 + k];
          tie |= s_tie[w][tid][k];
        }
        const bool ok = g != kNoGrid && !tie && T < kTop;  // NaN fails too
        s_T[tid][k] = T;
        s_ok[tid][k] = ok;
        const uint32_t code = ok ? (uint32_t)(g + 126) : (nan ? kCodeNaN : kCodeBad);
        put(&me->cand[k][tid], tag, (code << 24) | (ok ? (uint32_t)T : 0u));
      }
      put(&me->inclS[tid], tag, __float_as_uint((float)(s_exclS[tid] + s_aggS[tid])));
    }

    // ---- the exact accumulator before the tile (wave 0). The nearest predecessor with its accumulator
    // published (the base) plus the totals the tiles in between hold for the base's grid, if all of them
    // hold one and the sum stays below the binade's top. Otherwise the first tile from the base's side
    // that breaks this (a crossing into the next binade, a tie, a grid it did not predict) must itself
    // become the base: wait until it has published, and look again.
    if (wave == 0) {
      float excl = 0.0f;
      if (ti > 0) {
        for (;;) {
          bool found = false, nan = false;
          float base = 0.0f;
          int dbase = 0;  // predecessors between the base and this tile
          // beyond kMaxD the candidates are not kept: their totals are summed for this tile's own grids
          const int ga = s_g[c][0], gb = s_g[c][1];
          double fa = 0.0, fb = 0.0;
          bool fbada = false, fbadb = gb == kNoGrid;
          for (int r = 0; __any(!found); ++r) {
            unsigned long long g3[kBatch], c0[kBatch], c1[kBatch];
            for (long long ns = 0;;) {
#pragma unroll
              for (int j = 0; j < kBatch; ++j) {
                const int d = min((r * kBatch + j) * kWin + q, ti - 1);
                const Rec* p = me - kChunksPerTile * (1 + d);
                g3[j] = get(&p->incl[c]);
                c0[j] = get(&p->cand[0][c]);
                c1[j] = get(&p->cand[1][c]);
              }
              bool ok2 = true, fnd = found;
#pragma unroll
              for (int j = 0; j < kBatch; ++j) {
                const int d = (r * kBatch + j) * kWin + q;
                const bool valid = ti - 1 - d >= 0;
                const int qb = chain_first(!valid || has(g3[j], tag), c);
                ok2 &= fnd || q >= qb || (has(c0[j], tag) && has(c1[j], tag));
                fnd = fnd || qb < kWin;
              }
              if (__all(ok2) || !spin(ns, &s_err)) break;
            }
#pragma unroll
            for (int j = 0; j < kBatch; ++j) {
              const int d = (r * kBatch + j) * kWin + q;
              const bool valid = !found && ti - 1 - d >= 0;
              const int qb = chain_first(ti - 1 - d < 0 || has(g3[j], tag), c);
              const bool between = !found && q < qb;
              if ((r * kBatch + j) * kWin < kMaxD) {  // the nearest kMaxD predecessors: kept for the composition
                s_cand[d][c][0] = c0[j];
                s_cand[d][c][1] = c1[j];
              } else {
                double va = 0.0, vb = 0.0;
                bool ia = false, ib = false;
                if (between) {
                  ia = !pick(c0[j], c1[j], ga, va);
                  ib = !pick(c0[j], c1[j], gb, vb);
                }
                fa += chain_sum(va);
                fb += chain_sum(vb);
                fbada |= chain_any(ia, c);
                fbadb |= chain_any(ib, c);
              }
              nan |= chain_any(between && ((uint32_t)c0[j] >> 24) == kCodeNaN, c);
              const float b = __shfl(valid ? fval(g3[j]) : 0.0f, (qb < kWin ? qb : 0) * 8 + c, 64);
              if (!found && qb < kWin) {
                base = b;
                dbase = (r * kBatch + j) * kWin + qb;
                found = true;
              }
            }
            if (s_err) break;
          }
          bool ok = true;
          int dwait = kMaxD - 1;  // the tile to wait for when this chain's composition fails
          if (!found) {  // only after a spin ran out
            ok = false;
          } else if (__builtin_isnan(base) || dbase == 0) {
            excl = base;
          } else if (__builtin_isinf(base)) {
            excl = nan ? __builtin_nanf("") : base;
          } else {
            const int G = grid_of(base);
            const double A = (double)base * pow2(23 - G);
            // totals of the in-between tiles (distance d < dbase) for grid G, nearest first
            double sum = 0.0;
            bool bad = false;
            for (int w = 0; w * kWin < kMaxD && __any(w * kWin < dbase); ++w) {
              const int d = w * kWin + q;
              double v = 0.0;
              bool b = false;
              if (d < dbase) b = !pick(s_cand[d][c][0], s_cand[d][c][1], G, v);
              sum += chain_sum(v);
              bad |= chain_any(b, c);
            }
            bool farbad = false;
            if (dbase > kMaxD) {  // the far tiles: through this tile's own candidate for G
              if (G == ga && !fbada) sum += fa;
              else if (G == gb && !fbadb) sum += fb;
              else farbad = true;
            }
            if (!bad && !farbad && A + sum < kTop) {
              excl = (float)((A + sum) * pow2(G - 23));
            } else {
              ok = false;
              if (q == 0) atomicAdd(&s_why[farbad ? 0 : (bad ? 1 : 2)], 1);
              // first break from the base's side: the largest d that is bad for G, or where the running
              // total from the base passes the top: A + sum - (totals of the tiles nearer than d) >= 2^24
              double nearer = 0.0;  // totals of distances below this window
              int brk = 0;
              for (int w = 0; w * kWin < kMaxD && __any(w * kWin < dbase); ++w) {
                const int d = w * kWin + q;
                double v = 0.0;
                bool b = false;
                if (d < dbase) b = !pick(s_cand[d][c][0], s_cand[d][c][1], G, v);
                double pre = v;  // inclusive prefix over this window's slots, nearest first
#pragma unroll
                for (int o = 8; o < 64; o <<= 1) {
                  const double y = __shfl_up(pre, o, 64);
                  if (lane >= o) pre += y;
                }
                const double before = nearer + pre - v;  // totals of distances < d
                const bool br = d < dbase && (b || A + sum - before >= kTop);
                const unsigned long long m = (__ballot(br) >> c) & kChain0;
                if (m) brk = w * kWin + ((63 - __builtin_clzll(m)) >> 3);
                nearer += chain_sum(v);
              }
              dwait = farbad ? kMaxD - 1 : brk;
            }
          }
          if (__all(ok) || s_err) break;
          if (!ok) {  // wait until that tile has published its accumulator
            const Rec* p = me - kChunksPerTile * (1 + dwait);
            for (long long ns = 0; !has(get(&p->incl[c]), tag) && spin(ns, &s_err);) {
            }
          }
          if (lane == 0) atomicAdd(&s_retry, 1);
        }
      }
      if (q == 0) s_excl[c] = excl;
    }
    __syncthreads();
    // ---- the tile's own steps
    if (tid < 8) {
      const float E = s_excl[tid];
      float inc = E;
      if (__builtin_isnan(E)) {
        inc = E;
      } else if (__builtin_isinf(E)) {
        inc = __builtin_isnan(s_aggS[tid]) ? __builtin_nanf("") : E;
      } else {
        const int G = grid_of(E);
        const double A = (double)E * pow2(23 - G);
        bool fast = false;
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (!fast && s_g[tid][k] == G && s_ok[tid][k] && A + s_T[tid][k] < kTop) {
            inc = (float)((A + s_T[tid][k]) * pow2(G - 23));
            fast = true;
          }
        if (!fast) atomicOr(&s_slow, 1 << tid);
      }
      s_inc[tid] = inc;
    }
    __syncthreads();
    if (s_slow) {  // block-uniform: the chains in order, the reference arithmetic itself
      // staged chain-major (s_stage[c][step]); steps past len are zeros, which change nothing
#pragma unroll
      for (int i = 0; i < kRegs; ++i) s_stage[c * kStageStride + 8 * kRegs * wave + 8 * i + q] = e[i];
      __syncthreads();
      if (tid < 8 && ((s_slow >> tid) & 1)) {
        float acc = s_excl[tid];
        const float4* l4 = reinterpret_cast<const float4*>(s_stage + tid * kStageStride);
        float4 a[8], bb[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = l4[k];
#pragma unroll
        for (int k0 = 0; k0 < kTile / 32; k0 += 16) {
#pragma unroll
          for (int k = 0; k < 8; ++k) bb[k] = l4[k0 + 8 + k];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            acc = __builtin_fmaf(a[k].x, a[k].x, acc);
            acc = __builtin_fmaf(a[k].y, a[k].y, acc);
            acc = __builtin_fmaf(a[k].z, a[k].z, acc);
            acc = __builtin_fmaf(a[k].w, a[k].w, acc);
          }
          if (k0 + 16 < kTile / 32) {
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = l4[k0 + 16 + k];
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            acc = __builtin_fmaf(bb[k].x, bb[k].x, acc);
            acc = __builtin_fmaf(bb[k].y, bb[k].y, acc);
            acc = __builtin_fmaf(bb[k].z, bb[k].z, acc);
            acc = __builtin_fmaf(bb[k].w, bb[k].w, acc);
          }
        }
        s_inc[tid] = acc;
      }
      __syncthreads();
    }
    if (tid < 8) put(&me->incl[tid], tag, __float_as_uint(s_inc[tid]));
    if (tid == 0) {
      if (ti == (ch.nchunks * kTilesPerChunk + kChunksPerTile - 1) / kChunksPerTile - 1) {  // last tile: lane sum, tail, sqrt
        const float* xs = x + tbase;
        float b = 0.0f;
        if (n < 8) {
          b = tail_sum(xs, 0, n, 0.0f);
        } else {
          b = s_inc[0];
#pragma unroll
          for (int j = 1; j < 8; ++j) b = b + s_inc[j];
          b = tail_sum(xs, nv, n, b);
        }
        norms[ch.tensor] = s_err ? __builtin_nanf("") : (float)__builtin_sqrt((double)b);
      }
      if (s_err) __hip_atomic_store(&hdr->error, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // counters for tools/torch_norm_bench.py: look-back retries, tiles walked sequentially
      if (s_retry) __hip_atomic_fetch_add(&hdr->stats[0], (unsigned long long)s_retry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (s_slow) __hip_atomic_fetch_add(&hdr->stats[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int k = 0; k < 2; ++k)
        if (s_why[k]) __hip_atomic_fetch_add(&hdr->stats[2 + k], (unsigned long long)s_why[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    }
  }
finish:
  if (tid == 0) {  // the last block out leaves the scratch ready for the next launch
    const unsigned long long d = __hip_atomic_fetch_add(&hdr->done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d + 1 == (unsigned long long)gridDim.x) {
      __hip_atomic_store(&hdr->ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&hdr->done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&hdr->epoch, epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

inline int64_t scratch_bytes(int64_t nchunks) {
  return (int64_t)sizeof(Header) + nchunks * kTilesPerChunk * (int64_t)sizeof(Rec);
}

}  // namespace adfl_tn
