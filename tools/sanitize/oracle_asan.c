/* oracle_asan.c — CPU sanitizer driver for the oracle's C restatement (oracle/slq_oracle.c): every entry
 * point on exactly-sized heap buffers (ragged lengths 1..4099, odd int4 counts, K-row means), so ASan
 * flags any read or write past a buffer. Test infrastructure only (tools/sanitize/run.sh). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

float oracle_slq_absmax(const float* x, int64_t n);
float oracle_slq_scale(float absmax, int bits);
void oracle_slq_quantize(const float* x, int64_t n, float scale, int8_t* q);
float oracle_slq_encode(const float* x, int64_t n, int bits, int8_t* q);
void oracle_slq_dequantize(const int8_t* q, int64_t n, float scale, float* out);
int64_t oracle_pack_int4(const int8_t* q, int64_t n, uint8_t* packed);
void oracle_unpack_int4(const uint8_t* packed, int64_t n, int8_t* q);
void oracle_slq_dequantize_int4(const uint8_t* packed, int64_t n, float scale, float* out);
void oracle_slq_dequantize_mean(const int8_t* const* qs, const float* scales, int32_t k, int64_t n, float* out);
void oracle_slq_dequantize_mean_int4(const uint8_t* const* ps, const float* scales, int32_t k, int64_t n, float* out);
void oracle_slq_dequantize_mean_self(const void* const* rows, const float* scales, int32_t k, int64_t n,
                                     int32_t self_row, const float* self_x, int32_t packed, float* out);
float oracle_torch_l2_norm(const float* x, int64_t n);

int main(void) {
    unsigned s = 7;
    int checked = 0;
    for (int64_t n = 1; n <= 4099; n += (n < 70 ? 1 : 97)) {
        float* x = malloc(n * sizeof(float));
        int8_t* q = malloc(n);
        float* d = malloc(n * sizeof(float));
        uint8_t* p = malloc((n + 1) / 2);
        int8_t* q2 = malloc(n);
        for (int64_t i = 0; i < n; ++i) {
            s = s * 1664525u + 1013904223u;
            x[i] = ((int32_t)s) * 1e-12f;
        }
        const float sc = oracle_slq_encode(x, n, 4, q);
        oracle_slq_quantize(x, n, oracle_slq_scale(oracle_slq_absmax(x, n), 8), q);
        oracle_slq_dequantize(q, n, sc, d);
        oracle_pack_int4(q, n, p);
        oracle_unpack_int4(p, n, q2);
        oracle_slq_dequantize_int4(p, n, sc, d);
        const int8_t* qs[3] = {q, q2, q};
        const uint8_t* ps[3] = {p, p, p};
        const void* rows[3] = {p, p, p};
        const float scs[3] = {sc, sc * 2, sc};
        oracle_slq_dequantize_mean(qs, scs, 3, n, d);
        oracle_slq_dequantize_mean_int4(ps, scs, 3, n, d);
        oracle_slq_dequantize_mean_self(rows, scs, 3, n, 1, x, 1, d);
        (void)oracle_torch_l2_norm(x, n);
        free(x);
        free(q);
        free(d);
        free(p);
        free(q2);
        ++checked;
    }
    printf("oracle_asan: %d lengths, every entry point\n", checked);
    return 0;
}
