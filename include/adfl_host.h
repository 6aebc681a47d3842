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

#include "adfl_slq.h"

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

/* Asynchronous adfl_host_copy_ex: the copy list is copied, queued behind earlier jobs and run by the pool's
 * worker threads only; the call returns at once with a ticket (> 0) or ADFL_E_ARG. If wait_fn is not null,
 * every part first calls wait_fn(wait_arg) and copies only when it returns 0 (the host-resident channel passes
 * adfl_event_synchronize and a HIP event recorded after the D2H that fills the source, so the scatter of a
 * staging range starts the moment its copy lands while the caller's thread builds the output tensors).
 * The buffers must stay valid until adfl_host_copy_wait(ticket) returns; every ticket is waited exactly once.
 * adfl_host_copy_wait returns 0, or the first nonzero status a wait_fn returned. */
int64_t adfl_host_copy_submit(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n,
                              int32_t nthreads, int32_t flags, int (*wait_fn)(void*), void* wait_arg);
int adfl_host_copy_wait(int64_t ticket);
/* 1 if every part of the job has finished (adfl_host_copy_wait would return at once), 0 if not, ADFL_E_ARG for
 * a bad ticket. Never blocks and does not consume the ticket. */
int adfl_host_copy_done(int64_t ticket);

/* adfl_host_copy_submit that also reduces what it copies: piece k is fp32 (nbytes[k] and srcs[k] multiples of
 * 4) and, when absmax_bits[k] is not null, max over its elements of (bits & 0x7fffffff) is max'ed atomically
 * into *absmax_bits[k] — torch.max(torch.abs(t)) as an unsigned compare of the magnitude bits, NaN winning
 * (Src/ADFL/Channel/quant.py:100), exactly as the device encode reduces it. The host-resident SLQ encode
 * gathers a CPU state dict this way, so every tensor's scale is known on the host when its bytes reach the
 * pinned bucket and its qint8 output can be built while the H2D and the kernels run. ADFL_E_ARG for a piece
 * that is not whole fp32 words. */
int64_t adfl_host_copy_submit_absmax(void* const* dsts, const void* const* srcs, const int64_t* nbytes, int64_t n,
                                     int32_t nthreads, int32_t flags, int (*wait_fn)(void*), void* wait_arg,
                                     uint32_t* const* absmax_bits);

/* Pin the pool's worker threads to the given CPUs (the channel passes the CPUs of the GPU's NUMA node, read
 * from sysfs: measured on the MI355X box, the C3 host round trip takes 3.3 ms bound to the GPU's node against
 * 4.1-4.4 ms on the other one). Returns 0, or ADFL_E_ARG for an empty or unusable set. */
int adfl_host_bind(const int32_t* cpus, int32_t n);

/* hipEventSynchronize(event) as an int-returning callback for adfl_host_copy_submit (0 = complete). */
int adfl_event_synchronize(void* event);

/* ---------------------------------------------------------------------------------------------
 * Device steps of one staging range of the host-resident channel path (csrc/host_stage.hip): what the
 * pipelined SLQChannel encode / decode of a CPU state dict (Src/ADFL/Channel/quant.py:74-112 on the dict
 * Src/ADFL/model.py:195-197 hands over) enqueues as each range of the pinned bucket lands, in one call.
 * Every step is asynchronous; h_* are PINNED host buffers, d_* device buffers, element offsets throughout.
 *   stream:      H2D of elements [lo, hi) (hi == lo: none); if count > 0, then the kernel over chunks
 *                [chunk_begin, chunk_begin + count) of the FULL chunk table d_chunks, then ev_compute
 *   d2h_stream:  waits for ev_compute, D2H of output elements [e0, e1), records ev_copied — the event the
 *                host pool's scatter of those elements waits on (adfl_host_copy_submit + adfl_event_synchronize)
 * Returns 0, ADFL_E_ARG, or a positive hipError_t. count == 0 enqueues the H2D alone.
 * ------------------------------------------------------------------------------------------- */
/* n timing-free HIP events on the current device into events[0..n) (the staging keeps them for its life). */
int adfl_stage_events_create(int32_t n, void** events);
int adfl_stage_events_destroy(void* const* events, int32_t n);

/* The copy-back half alone: record ev_compute on stream, make d2h_stream wait for it, then n D2H copies
 * (d_srcs[i] -> h_dsts[i], nbytes[i] bytes, h_dsts pinned) on d2h_stream, then record ev_copied there. The
 * stochastic encode runs its codec's kernels for the tensors a range completes, then hands both planes'
 * bytes of those tensors back through this. */
int adfl_stage_d2h(const void* const* d_srcs, void* const* h_dsts, const int64_t* nbytes, int32_t n, void* stream,
                   void* d2h_stream, void* ev_compute, void* ev_copied);

/* Encode: x range H2D; then, over the chunk range (whole tensors, every byte of them staged),
 * adfl_slq_absmax_batched_range into d_partials (one uint32 per chunk of the table) and
 * adfl_slq_quantize_batched_range into d_q / d_scales, and payload bytes [e0, e1) back into h_q. */
int adfl_stage_encode_range(const float* h_x, float* d_x, int64_t lo, int64_t hi, uint32_t* d_partials,
                            const adfl_slq_chunk* d_chunks, int64_t chunk_begin, int64_t count, int bits, int8_t* d_q,
                            float* d_scales, int8_t* h_q, int64_t e0, int64_t e1, void* stream, void* d2h_stream,
                            void* ev_compute, void* ev_copied);

/* Decode: payload range H2D; then adfl_slq_dequantize_batched over the chunk range into d_out, and floats
 * [e0, e1) back into h_out. */
int adfl_stage_decode_range(const int8_t* h_q, int8_t* d_q, int64_t lo, int64_t hi, const adfl_slq_chunk* d_chunks,
                            int64_t chunk_begin, int64_t count, const float* d_scales, float* d_out, float* h_out,
                            int64_t e0, int64_t e1, void* stream, void* d2h_stream, void* ev_compute,
                            void* ev_copied);

/* Stochastic decode (codec ADFL_CODEC_QSGD / RQSGD / CNAT of adfl_stoch.h): both byte planes' range H2D; then
 * the codec's dequantize over the chunk range (adfl_qsgd / rqsgd / cnat_dequantize_batched; d_levels holds
 * CNAT's int8 exponents; d_mins only for RQSGD) into d_out, and floats [e0, e1) back into h_out. */
int adfl_stage_stoch_decode_range(int32_t codec, int bits, const uint8_t* h_levels, uint8_t* d_levels,
                                  const int8_t* h_signs, int8_t* d_signs, int64_t lo, int64_t hi,
                                  const adfl_slq_chunk* d_chunks, int64_t chunk_begin, int64_t count,
                                  const float* d_norms, const float* d_mins, float* d_out, float* h_out, int64_t e0,
                                  int64_t e1, void* stream, void* d2h_stream, void* ev_compute, void* ev_copied);

/* Threads the pool would use for nthreads <= 0 (for logging and tests): the CPUs in this process's affinity
 * mask, at most 8, or ADFL_HOST_THREADS when set. */
int32_t adfl_host_threads(void);

#ifdef __cplusplus
}
#endif

#endif /* ADFL_HOST_H */
