/*
 * adfl_host.h — host-side runtime of libadfl_slq.so: parallel staging copies for the host-resident
 * channel path (CPU state dict -> pinned bucket -> device, and back).
 *
 * The reference codec runs on CPU tensors (Src/ADFL/Channel/quant.py:74-112; callers .cpu() first,
 * Src/ADFL/model.py:195-197), so a drop-in GPU channel first gathers a whole state dict into one pinned
 * host bucket and at the end scatters the payload back into per-tensor storage. Those two host memcpys
 * dominate the host-to-host call; torch.cat of 256 pieces runs single-stream. This call
 * splits a list of copies into byte ranges across a persistent pool of host threads.
 */
#ifndef ADFL_HOST_H
#define ADFL_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dsts[k] <- srcs[k], nbytes[k] bytes, k < n (HOST pointers; regions must not overlap). The total is split
 * into contiguous byte ranges over min(nthreads, pool size) threads, the caller's thread included;
 * nthreads <= 0 picks the default (hardware threads, at most 16). Blocks until every byte is copied.
 * Returns 0, or ADFL_E_ARG (-1) for a null pointer or negative size. */
int adfl_host_copy(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n, int32_t nthreads);

/* adfl_host_copy with flags. ADFL_HOST_COPY_STREAM: pieces of 64 KiB or more are written with
 * non-temporal (streaming) stores, for destinations nothing reads soon (fresh per-tensor outputs: measured
 * faster for the scatter, slower for the gather into a pinned bucket, tools/hostcopy_ab.py). */
enum { ADFL_HOST_COPY_STREAM = 1 };
int adfl_host_copy_ex(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n, int32_t nthreads,
                      int32_t flags);

/* Threads the pool would use for nthreads <= 0 (for logging and tests). */
int32_t adfl_host_threads(void);

#ifdef __cplusplus
}
#endif

#endif /* ADFL_HOST_H */
