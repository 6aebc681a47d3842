// bucket_copy.hip — the device side of staging a state dict as one bucket (include/adfl_slq.h,
// adfl_bucket_gather / adfl_bucket_scatter): every tensor's elements copied between its own storage and its
// slot of the flat bucket, for the whole dict in one launch. The per-tensor form this replaces cost one
// launch per tensor on the way out (the owned per-tensor payloads and decoded tensors the Channel API
// returns, quant.py:83-92,107-112) — 256 launches for ResNet-18's weights, milliseconds of host time for
// 0.03 ms of copying.
//
// One block per chunk of the bucket's chunk table: the chunk's bytes are copied between bucket + start and
// ptrs[tensor] + (start - the tensor's first element), 16-byte words when source and destination share
// their phase mod 16 (bytes up to the first boundary and after the last), 4-byte words when they share it
// mod 4, bytes otherwise. Pads between tensors in an aligned bucket are in no chunk: never read or written.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "adfl_host.h"
#include "adfl_slq.h"

namespace {

constexpr int kBlock = 256;

template <typename W>
__device__ __forceinline__ void copy_words(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n) {
  constexpr int kW = (int)sizeof(W);
  const int h = (int)((kW - ((uintptr_t)dst & (kW - 1))) & (kW - 1));
  const int64_t head = h < n ? h : n;
  for (int64_t i = threadIdx.x; i < head; i += kBlock) dst[i] = src[i];
  const int64_t nw = (n - head) / kW;
  const W* s = reinterpret_cast<const W*>(src + head);
  W* d = reinterpret_cast<W*>(dst + head);
  int64_t i = threadIdx.x;
  for (; i + 3 * kBlock < nw; i += 4 * kBlock) {  // four words in flight per thread
    const W a = s[i], b = s[i + kBlock], c = s[i + 2 * kBlock], e = s[i + 3 * kBlock];
    d[i] = a;
    d[i + kBlock] = b;
    d[i + 2 * kBlock] = c;
    d[i + 3 * kBlock] = e;
  }
  for (; i < nw; i += kBlock) d[i] = s[i];
  for (int64_t j = head + nw * kW + threadIdx.x; j < n; j += kBlock) dst[j] = src[j];
}

template <bool TO_BUCKET>
__global__ __launch_bounds__(kBlock) void k_bucket_copy(uint8_t* __restrict__ bucket,
                                                        const adfl_slq_chunk* __restrict__ chunks,
                                                        uint8_t* const* __restrict__ ptrs, int eb) {
  const adfl_slq_chunk c = chunks[blockIdx.x];
  const int64_t t0 = chunks[c.first_chunk].start;
  uint8_t* b = bucket + c.start * eb;
  uint8_t* p = ptrs[c.tensor] + (c.start - t0) * eb;
  uint8_t* dst = TO_BUCKET ? b : p;
  const uint8_t* src = TO_BUCKET ? p : b;
  const int64_t n = (int64_t)c.len * eb;
  const uintptr_t phase = (uintptr_t)dst ^ (uintptr_t)src;  // block-uniform
  if ((phase & 15) == 0)
    copy_words<uint4>(dst, src, n);
  else if ((phase & 3) == 0)
    copy_words<uint32_t>(dst, src, n);
  else
    copy_words<uint8_t>(dst, src, n);
}

int launch(bool to_bucket, void* d_bucket, const adfl_slq_chunk* d_chunks, int64_t nchunks, const void* d_ptrs,
           int32_t elem_bytes, void* stream) {
  if (!d_bucket || !d_chunks || !d_ptrs || nchunks < 0 || nchunks > INT32_MAX) return ADFL_E_ARG;
  if (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8) return ADFL_E_ARG;
  if (nchunks == 0) return ADFL_OK;
  auto* bucket = static_cast<uint8_t*>(d_bucket);
  auto* ptrs = static_cast<uint8_t* const*>(d_ptrs);
  if (to_bucket)
    hipLaunchKernelGGL(k_bucket_copy<true>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, bucket,
                       d_chunks, ptrs, (int)elem_bytes);
  else
    hipLaunchKernelGGL(k_bucket_copy<false>, dim3((unsigned)nchunks), dim3(kBlock), 0, (hipStream_t)stream, bucket,
                       d_chunks, ptrs, (int)elem_bytes);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ADFL_OK : (int)e;
}

}  // namespace

extern "C" {

// include/adfl_host.h: the completion wait the host copy pool runs before scattering a staging range.
int adfl_event_synchronize(void* event) {
  const hipError_t e = hipEventSynchronize(static_cast<hipEvent_t>(event));
  return e == hipSuccess ? 0 : (int)e;
}

int adfl_bucket_gather(void* d_bucket, const adfl_slq_chunk* d_chunks, int64_t nchunks, const void* const* d_srcs,
                       int32_t elem_bytes, void* stream) {
  return launch(true, d_bucket, d_chunks, nchunks, d_srcs, elem_bytes, stream);
}

int adfl_bucket_scatter(const void* d_bucket, const adfl_slq_chunk* d_chunks, int64_t nchunks, void* const* d_dsts,
                        int32_t elem_bytes, void* stream) {
  return launch(false, const_cast<void*>(d_bucket), d_chunks, nchunks, d_dsts, elem_bytes, stream);
}

}  // extern "C"
