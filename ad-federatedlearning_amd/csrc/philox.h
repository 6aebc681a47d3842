// philox.h — the codecs' counter-based uniform stream, Philox4x32-R (Salmon et al., SC'11), shared by
// stoch_codec.hip (fp32 tensors) and stoch_dtype.hip (fp16 / bf16 / fp64 tensors). Round function,
// multipliers and key schedule are Philox4x32's (pinned by the 10-round known-answer vectors in
// tests/test_stoch_golden.py); the codecs run R = 7 rounds (stoch_codec.hip header).
//
// Why 7: Salmon et al. (SC'11, Table 2) report Philox4x32-7 as the fewest rounds that pass all of TestU01's
// BigCrush ("Crush-resistant"); 10 rounds is Random123's and curand's default safety margin. These codecs
// compare each uniform with a threshold at 24-bit resolution (fp16 / bf16: 11 / 8 bits), and the
// reference's own draws are torch.rand_like's mt19937, so no run is bit-comparable with the reference's
// stream under any R. What is tested here: the 7-round words continued by 3 more rounds give the 10-round
// known answers (round function, multipliers, key schedule pinned), and the 7-round stream's statistics on
// 2^20 draws — a 256-bucket chi-square, lag-1 and lag-4 correlation, each of the 24 used bits at 1/2
// (tests/test_stoch_golden.py: test_philox_7_rounds_is_a_prefix_of_the_known_answer_computation,
// test_philox_7_round_stream_statistics), plus the unbiased-decode and CNAT frequency checks on the GPU.
// BigCrush / PractRand themselves are not in this image. For the standard margin, build with
// ADFL_PHILOX_ROUNDS=10 in the environment (adfl_amd/_build.py passes -DADFL_PHILOX_ROUNDS; the oracle,
// oracle/stoch_oracle.py, reads the same variable; adfl_philox_rounds() reports what was compiled). Streams
// for a fixed (seed, counter) differ between the two builds.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef ADFL_PHILOX_ROUNDS
#define ADFL_PHILOX_ROUNDS 7
#endif

namespace adfl {

constexpr int kPhiloxRounds = ADFL_PHILOX_ROUNDS;

// Block `ctr` of the stream keyed by `seed` (counter words 2, 3 are zero).
__device__ __forceinline__ uint4 philox4x32(uint64_t ctr, uint64_t seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < kPhiloxRounds; ++r) {
    // full 32x32 -> 64 products: one v_mad_u64_u32 each instead of a v_mul_hi_u32 + v_mul_lo_u32 pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    c1 = (uint32_t)p1;
    c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

}  // namespace adfl
