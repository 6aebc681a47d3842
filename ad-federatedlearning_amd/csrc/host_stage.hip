// host_stage.hip — the device-side steps of one staging range of the host-resident channel path
// (include/adfl_host.h, adfl_stage_encode_range / adfl_stage_decode_range), as one call.
//
// SLQChannel's host-to-host encode and decode (Src/ADFL/Channel/quant.py:74-112 on the CPU state dict the
// client hands over, Src/ADFL/model.py:195-197), and the QSGD / RQSGD / CNAT decode (quant.py:243-252,
// 385-398,537-545), are pipelined over staging ranges of the pinned bucket
// (adfl_amd/Channel/quant.py, _encode_host_dict / _decode_host_dict): as range r lands in pinned memory, its
// H2D is enqueued, the tensors or chunks it completes are (de)quantized, and their output goes back D2H on a
// second stream behind an event, while the host pool scatters the previous range. A trace of the C3 dict
// (profiles/r05/host_stage/) showed the calling thread, not the link, pacing those ranges, and the torch ops
// that enqueued each one — slices, copies, a stream switch, event objects — cost it ~40 us per range. Here
// they are the HIP calls alone.
//
// Order per range, every step asynchronous:
//   stream:      H2D [lo, hi) of the input (both byte planes for the stochastic decode); if count > 0: (encode)
//                the absmax and quantize kernels, (decode) the codec's dequantize kernel, over chunks
//                [chunk_begin, chunk_begin + count), record ev_compute
//   d2h_stream:  wait ev_compute, D2H [e0, e1) of the output, record ev_copied (the host pool's scatter of
//                that range waits on it through adfl_event_synchronize)

#include <hip/hip_runtime.h>

#include <cstdint>

#include "adfl_host.h"
#include "adfl_slq.h"
#include "adfl_stoch.h"

namespace {

int hip_status(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// The D2H half: d2h_stream waits for the kernel, copies [e0, e1) of `elem` bytes each back, records ev_copied.
int copy_back(const void* d_src, void* h_dst, int64_t e0, int64_t e1, int64_t elem, hipStream_t st, hipStream_t d2h,
              hipEvent_t ev_compute, hipEvent_t ev_copied) {
  if (int s = hip_status(hipEventRecord(ev_compute, st))) return s;
  if (int s = hip_status(hipStreamWaitEvent(d2h, ev_compute, 0))) return s;
  if (int s = hip_status(hipMemcpyAsync(static_cast<char*>(h_dst) + e0 * elem,
                                        static_cast<const char*>(d_src) + e0 * elem, (size_t)((e1 - e0) * elem),
                                        hipMemcpyDeviceToHost, d2h)))
    return s;
  return hip_status(hipEventRecord(ev_copied, d2h));
}

}  // namespace

extern "C" {

int adfl_stage_events_create(int32_t n, void** events) {
  if (n < 0 || (n > 0 && !events)) return ADFL_E_ARG;
  for (int32_t i = 0; i < n; ++i) {
    hipEvent_t e = nullptr;
    if (int s = hip_status(hipEventCreateWithFlags(&e, hipEventDisableTiming))) {
      for (int32_t j = 0; j < i; ++j) (void)hipEventDestroy(static_cast<hipEvent_t>(events[j]));
      return s;
    }
    events[i] = e;
  }
  return 0;
}

int adfl_stage_events_destroy(void* const* events, int32_t n) {
  if (n < 0 || (n > 0 && !events)) return ADFL_E_ARG;
  int first = 0;
  for (int32_t i = 0; i < n; ++i) {
    const int s = hip_status(hipEventDestroy(static_cast<hipEvent_t>(events[i])));
    if (s && !first) first = s;
  }
  return first;
}

int adfl_stage_d2h(const void* const* d_srcs, void* const* h_dsts, const int64_t* nbytes, int32_t n, void* stream,
                   void* d2h_stream, void* ev_compute, void* ev_copied) {
  if (n < 1 || !d_srcs || !h_dsts || !nbytes || !d2h_stream || !ev_compute || !ev_copied) return ADFL_E_ARG;
  for (int32_t i = 0; i < n; ++i)
    if (!d_srcs[i] || !h_dsts[i] || nbytes[i] < 0) return ADFL_E_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream), d2h = static_cast<hipStream_t>(d2h_stream);
  if (int s = hip_status(hipEventRecord(static_cast<hipEvent_t>(ev_compute), st))) return s;
  if (int s = hip_status(hipStreamWaitEvent(d2h, static_cast<hipEvent_t>(ev_compute), 0))) return s;
  for (int32_t i = 0; i < n; ++i)
    if (nbytes[i] > 0)
      if (int s = hip_status(hipMemcpyAsync(h_dsts[i], d_srcs[i], (size_t)nbytes[i], hipMemcpyDeviceToHost, d2h)))
        return s;
  return hip_status(hipEventRecord(static_cast<hipEvent_t>(ev_copied), d2h));
}

int adfl_stage_encode_range(const float* h_x, float* d_x, int64_t lo, int64_t hi, uint32_t* d_partials,
                            const adfl_slq_chunk* d_chunks, int64_t chunk_begin, int64_t count, int bits, int8_t* d_q,
                            float* d_scales, int8_t* h_q, int64_t e0, int64_t e1, void* stream, void* d2h_stream,
                            void* ev_compute, void* ev_copied) {
  if (!h_x || !d_x || lo < 0 || hi < lo || count < 0) return ADFL_E_ARG;
  if (count > 0 && (!d_partials || !d_chunks || !d_q || !d_scales || !h_q || chunk_begin < 0 || e0 < 0 || e1 <= e0 ||
                    !d2h_stream || !ev_compute || !ev_copied))
    return ADFL_E_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hi > lo) {
    if (int s = hip_status(hipMemcpyAsync(d_x + lo, h_x + lo, (size_t)(hi - lo) * 4, hipMemcpyHostToDevice, st)))
      return s;
  }
  if (count == 0) return 0;
  // the device's own max|x| over the completed tensors' chunks (just landed, so read from the caches), then
  // their quantize: the scales and payload never depend on anything the host reduced
  if (int s = adfl_slq_absmax_batched_range(d_x, d_chunks, chunk_begin, count, d_partials, stream)) return s;
  if (int s = adfl_slq_quantize_batched_range(d_x, d_chunks, chunk_begin, count, bits, d_partials, d_q, d_scales,
                                              stream))
    return s;
  return copy_back(d_q, h_q, e0, e1, 1, st, static_cast<hipStream_t>(d2h_stream), static_cast<hipEvent_t>(ev_compute),
                   static_cast<hipEvent_t>(ev_copied));
}

int adfl_stage_decode_range(const int8_t* h_q, int8_t* d_q, int64_t lo, int64_t hi, const adfl_slq_chunk* d_chunks,
                            int64_t chunk_begin, int64_t count, const float* d_scales, float* d_out, float* h_out,
                            int64_t e0, int64_t e1, void* stream, void* d2h_stream, void* ev_compute,
                            void* ev_copied) {
  if (!h_q || !d_q || lo < 0 || hi < lo || count < 0) return ADFL_E_ARG;
  if (count > 0 && (!d_chunks || !d_scales || !d_out || !h_out || chunk_begin < 0 || e0 < 0 || e1 <= e0 ||
                    !d2h_stream || !ev_compute || !ev_copied))
    return ADFL_E_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hi > lo) {
    if (int s = hip_status(hipMemcpyAsync(d_q + lo, h_q + lo, (size_t)(hi - lo), hipMemcpyHostToDevice, st)))
      return s;
  }
  if (count == 0) return 0;
  if (int s = adfl_slq_dequantize_batched(d_q, d_chunks + chunk_begin, count, d_scales, d_out, stream)) return s;
  return copy_back(d_out, h_out, e0, e1, 4, st, static_cast<hipStream_t>(d2h_stream),
                   static_cast<hipEvent_t>(ev_compute), static_cast<hipEvent_t>(ev_copied));
}

int adfl_stage_stoch_decode_range(int32_t codec, int bits, const uint8_t* h_levels, uint8_t* d_levels,
                                  const int8_t* h_signs, int8_t* d_signs, int64_t lo, int64_t hi,
                                  const adfl_slq_chunk* d_chunks, int64_t chunk_begin, int64_t count,
                                  const float* d_norms, const float* d_mins, float* d_out, float* h_out, int64_t e0,
                                  int64_t e1, void* stream, void* d2h_stream, void* ev_compute, void* ev_copied) {
  if (!h_levels || !d_levels || !h_signs || !d_signs || lo < 0 || hi < lo || count < 0) return ADFL_E_ARG;
  if (codec != ADFL_CODEC_QSGD && codec != ADFL_CODEC_RQSGD && codec != ADFL_CODEC_CNAT) return ADFL_E_ARG;
  if (count > 0 && (!d_chunks || !d_norms || !d_out || !h_out || chunk_begin < 0 || e0 < 0 || e1 <= e0 ||
                    !d2h_stream || !ev_compute || !ev_copied || (codec == ADFL_CODEC_RQSGD && !d_mins)))
    return ADFL_E_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hi > lo) {
    if (int s = hip_status(hipMemcpyAsync(d_levels + lo, h_levels + lo, (size_t)(hi - lo), hipMemcpyHostToDevice, st)))
      return s;
    if (int s = hip_status(hipMemcpyAsync(d_signs + lo, h_signs + lo, (size_t)(hi - lo), hipMemcpyHostToDevice, st)))
      return s;
  }
  if (count == 0) return 0;
  const adfl_slq_chunk* c = d_chunks + chunk_begin;
  int s = 0;
  if (codec == ADFL_CODEC_QSGD)
    s = adfl_qsgd_dequantize_batched(d_levels, d_signs, c, count, bits, d_norms, d_out, stream);
  else if (codec == ADFL_CODEC_RQSGD)
    s = adfl_rqsgd_dequantize_batched(d_levels, d_signs, c, count, bits, d_norms, d_mins, d_out, stream);
  else
    s = adfl_cnat_dequantize_batched(reinterpret_cast<const int8_t*>(d_levels), d_signs, c, count, d_norms, d_out,
                                     stream);
  if (s) return s;
  return copy_back(d_out, h_out, e0, e1, 4, st, static_cast<hipStream_t>(d2h_stream),
                   static_cast<hipEvent_t>(ev_compute), static_cast<hipEvent_t>(ev_copied));
}

}  // extern "C"
