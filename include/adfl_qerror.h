/*
 * adfl_qerror.h — the reference's quantization-error metrics, bit for bit, on the device (libadfl_slq.so).
 *
 * Replaces Src/ADFL/model.py:256-323 — parameter_relative_mse (-> parameter_mse, :266-284) and
 * parameter_cosine_similarity (:302-323), both with exclude_bias=True as Src/ADFL/Client/worker.py:186-189
 * calls them on an update and its decode. What torch 2.10 computes there (CPU, fp32):
 *   e[t] = torch.sum((x_t - d_t) ** 2)     s[t] = torch.sum((x_t - 0) ** 2)     per ndim > 1 tensor t
 *   c    = torch.sum((x / max(|x|, 1e-8)) * (d / max(|d|, 1e-8)))               x, d = the concatenations
 * each sum in torch's CPU order (cascade_sum: 8 lanes x 4 ILP partials x a 4-level cascade; above 32,768
 * elements with T > 1 threads the two-pass parallel reduction over at::parallel_for's split), |.| the
 * reference-order fp32 norm (adfl_torch_norms), max NaN-propagating. The caller then forms the Python
 * doubles exactly as model.py does: mse = (sum_t e[t] / N) / (sum_t s[t] / N), cos = c.
 * Restated in oracle/slq_oracle.c (oracle_torch_sum_f32, oracle_qerror_ref), pinned to torch.sum and to the
 * reference executed in place (tests/test_qerror_order.py, tests/golden/qerror_manifest.json).
 *
 * Conventions as adfl_slq.h: d_* device pointers, asynchronous on `stream`, nothing allocated.
 */
#ifndef ADFL_QERROR_H
#define ADFL_QERROR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Plan the sums for tensors of sizes[0..ntensors) laid back to back and `threads` = the caller's
 * torch.get_num_threads(): fills h_plan (host memory, plan_bytes) when it is large enough and returns the
 * plan's size in bytes (call with h_plan == NULL to size it), or a negative ADFL_E_* code. The plan is
 * position independent: copy it to the device once per (sizes, threads) and reuse it. */
int64_t adfl_qerror_ref_plan(const int64_t* sizes, int32_t ntensors, int32_t threads, void* h_plan, int64_t plan_bytes);
/* Device scratch the metrics need for a plan (read from the HOST copy of the plan). */
int64_t adfl_qerror_ref_scratch_bytes(const void* h_plan);
/* d_x: the update, d_d: its decode, both ntensors back to back (the plan's layout), fp32.
 * d_norms: {|x|, |d|} fp32 (adfl_torch_norms over the two concatenations). d_out: 2 * ntensors + 1 floats:
 * e[0..T), s[0..T), c. h_plan / d_plan: the plan in host memory (its counts size the launches) and its copy
 * on the device (what the kernels read). d_scratch 256-byte aligned. */
int adfl_qerror_ref(const float* d_x, const float* d_d, const void* h_plan, const void* d_plan, const float* d_norms,
                    void* d_scratch, int64_t scratch_bytes, float* d_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ADFL_QERROR_H */
