/* torch_norm_proto.c — CPU model of the parallel exact torch-order L2 norm (not part of the product).
 *
 * torch's fp32 vector_norm is 8 chains acc_j = fmaf(x, x, acc_j) over the elements 8i + j. Each step is
 * RN32(acc + p) with p = x*x exact (48 bits, exact in fp64). While acc stays in one binade (grid u), the
 * step is acc + u * R(p / u) — an integer increment that does not depend on acc except through the
 * tie-to-even rule — so a tile of steps adds a sum of integers, computable in parallel, as long as it
 * stays below the binade's top. This program checks that model against the plain sequential chain on
 * random and adversarial data, and counts how often a tile takes the fast path when its grid is predicted
 * from an fp64 prefix sum (the look-back kernel's predictor).
 *
 *   gcc -O2 -o /tmp/torch_norm_proto tools/torch_norm_proto.c -lm && /tmp/torch_norm_proto
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* grid exponent of a finite acc >= 0: u = 2^(g - 23); acc = A * u with A < 2^24 */
static int grid_of(float acc) {
    if (acc < 0x1p-125f) return -126;      /* subnormals and the first normal binade share u = 2^-149 */
    int e; frexpf(acc, &e);                 /* acc = m 2^e, m in [0.5, 1) -> binade e - 1 */
    return e - 1;
}

typedef struct { long fast, slow, crossing_steps, tie_tiles, mispredicted; double maxdev, mindev; } stats_t;

/* one chain's tile [0, T): returns new acc. fast path if the (given) grid matches, no special step, no tie,
 * and A + total < 2^24; else the crossing-aware in-tile walk (what the wave scan does on the GPU). */
static float tile_step(float acc, const float* e, int64_t stride, int T, int g_pred, stats_t* st) {
    if (isnan(acc)) return acc;
    if (isinf(acc)) {
        for (int i = 0; i < T; ++i) if (isnan(e[i * stride])) return e[i * stride];
        return acc;
    }
    const int g = grid_of(acc);
    const double A = ldexp((double)acc, 23 - g);
    const double scale = ldexp(1.0, 23 - g);
    if (g == g_pred) {
        double tot = 0.0; int special = 0, tie = 0;
        for (int i = 0; i < T; ++i) {
            const double x = e[i * stride];
            const double v = x * x * scale;
            if (!(v < 0x1p24)) { special = 1; break; }
            const double f = floor(v);
            if (v - f == 0.5) tie = 1;
            tot += rint(v);
        }
        if (!special && !tie && A + tot < 0x1p24) { st->fast++; return (float)ldexp(A + tot, g - 23); }
        if (tie) st->tie_tiles++;
    } else st->mispredicted++;
    st->slow++;
    /* crossing-aware walk: prefix under the current grid, exact fma at the first step that may leave it */
    int i = 0;
    while (i < T) {
        if (isnan(acc) || isinf(acc)) {           /* terminal */
            for (; i < T; ++i) acc = fmaf(e[i * stride], e[i * stride], acc);
            break;
        }
        const int gg = grid_of(acc);
        const double sc = ldexp(1.0, 23 - gg);
        double P = ldexp((double)acc, 23 - gg);   /* A + prefix, an integer */
        for (; i < T; ++i) {
            const double x = e[i * stride];
            const double v = x * x * sc;
            if (!(P + v < 0x1p24)) break;         /* may cross (or NaN / inf): exact step */
            const double f = floor(v);
            double k;
            if (v - f == 0.5) k = f + (double)(((int64_t)(P + f)) & 1);   /* tie: make A + P + k even */
            else k = rint(v);
            P += k;
        }
        acc = (float)ldexp(P, gg - 23);
        if (i < T) {
            acc = fmaf(e[i * stride], e[i * stride], acc);
            st->crossing_steps++;
            ++i;
        }
    }
    return acc;
}

static float ref_norm(const float* x, int64_t n) {
    float b = 0.0f;
    if (n < 8) { for (int64_t i = 0; i < n; ++i) { const float sq = x[i] * x[i]; b = b + sq; } return sqrtf(b); }
    float acc[8] = {0};
    const int64_t nv = n - n % 8;
    for (int64_t i = 0; i < nv; i += 8) for (int j = 0; j < 8; ++j) acc[j] = fmaf(x[i + j], x[i + j], acc[j]);
    b = acc[0];
    for (int j = 1; j < 8; ++j) b = b + acc[j];
    for (int64_t i = nv; i < n; ++i) b = fmaf(x[i], x[i], b);
    return sqrtf(b);
}

/* tiled model; predictor: grid of the fp64 prefix sum scaled by (1 - delta) (delta = 0: the exact state's grid) */
static float model_norm(const float* x, int64_t n, int T, double delta, int oracle_grid, stats_t* st) {
    if (n < 8) return ref_norm(x, n);
    const int64_t nv = n - n % 8, m = nv / 8;
    float acc[8];
    for (int j = 0; j < 8; ++j) {
        float a = 0.0f;
        double S = 0.0;
        for (int64_t t0 = 0; t0 < m; t0 += T) {
            const int len = (int)(m - t0 < T ? m - t0 : T);
            int gp;
            if (oracle_grid) gp = isfinite(a) ? grid_of(a) : 0;
            else gp = grid_of((float)(S * (1.0 - delta)));
            if (isfinite(a) && S > 0) { const double d = (S - a) / S; if (d > st->maxdev) st->maxdev = d; if (d < st->mindev) st->mindev = d; }
            a = tile_step(a, x + t0 * 8 + j, 8, len, gp, st);
            for (int i = 0; i < len; ++i) S += (double)x[(t0 + i) * 8 + j] * x[(t0 + i) * 8 + j];
        }
        acc[j] = a;
    }
    float b = acc[0];
    for (int j = 1; j < 8; ++j) b = b + acc[j];
    for (int64_t i = nv; i < n; ++i) b = fmaf(x[i], x[i], b);
    return sqrtf(b);
}

static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static double urand(void) { return (rnd() >> 11) * 0x1p-53; }
static float nrand(void) {
    double u1 = urand(), u2 = urand();
    if (u1 < 1e-300) u1 = 1e-300;
    return (float)(sqrt(-2 * log(u1)) * cos(6.283185307179586 * u2));
}

static int check(const char* name, float* x, int64_t n, int T, int verbose) {
    stats_t st = {0};
    const float r = ref_norm(x, n);
    const float a = model_norm(x, n, T, 0.0, 1, &st);
    stats_t sp = {0};
    const float b = model_norm(x, n, T, 1.0 / 64, 0, &sp);
    const int ok = bits(r) == bits(a) && bits(r) == bits(b);
    if (verbose || !ok)
        printf("%-28s n=%-10lld T=%-5d %s ref %.9g  exact-grid fast %ld slow %ld (ties %ld, crossings %ld) | "
               "predicted fast %ld slow %ld mispred %ld\n", name, (long long)n, T, ok ? "ok " : "BAD", r, st.fast,
               st.slow, st.tie_tiles, st.crossing_steps, sp.fast, sp.slow, sp.mispredicted);
    if (verbose) printf("   (S - acc) / S at tile starts: min %.3g max %.3g\n", st.mindev, st.maxdev);
    if (!ok) printf("   model %.9g (%08x) predicted %.9g (%08x) ref %08x\n", a, bits(a), b, bits(b), bits(r));
    return ok;
}

int main(int argc, char** argv) {
    const int64_t big = argc > 1 ? atoll(argv[1]) : (1 << 24);
    int bad = 0;
    float* x = malloc(sizeof(float) * (big > 1 << 20 ? big : 1 << 20));
    /* the bench data: randn * 1e-3, C3 tensor size and a big flat tensor */
    for (int64_t i = 0; i < big; ++i) x[i] = nrand() * 1e-3f;
    bad += !check("randn*1e-3 C3 tensor", x, 45662, 128, 1);
    bad += !check("randn*1e-3 big", x, big, 1024, 1);
    /* random sizes and tile lengths */
    for (int trial = 0; trial < 400; ++trial) {
        const int64_t n = 1 + rnd() % 70000;
        const int T = 1 + rnd() % 300;
        const int kind = trial % 10;
        for (int64_t i = 0; i < n; ++i) {
            float v;
            switch (kind) {
                case 0: v = nrand(); break;
                case 1: v = (float)(int)(nrand() * 20); break;                          /* integers: ties */
                case 2: { float f = nrand(); uint32_t u = bits(f) & 0xffff0000u; memcpy(&v, &u, 4); } break;  /* bf16 */
                case 3: v = 0.6f; break;
                case 4: v = nrand() * powf(2.f, (float)((int)(rnd() % 120) - 60)); break;  /* wide scales */
                case 5: v = nrand() * 1e-22f; break;                                      /* squares underflow */
                case 6: v = nrand() * 1e19f; break;                                       /* squares overflow */
                case 7: { uint32_t u = (uint32_t)(rnd() % 0x00800000u); memcpy(&v, &u, 4); } break;  /* subnormal */
                case 8: v = (rnd() % 1000 == 0) ? (rnd() & 1 ? NAN : INFINITY) : nrand(); break;
                default: v = (rnd() % 7 == 0) ? 0.0f : (float)(rnd() % 5) * 0.25f; break;      /* short mantissas */
            }
            x[i] = v;
        }
        char name[64];
        snprintf(name, sizeof name, "trial %d kind %d", trial, kind);
        bad += !check(name, x, n, T, trial < 10);
    }
    printf("%s (%d bad)\n", bad ? "FAIL" : "all bit-identical to the sequential chain", bad);
    free(x);
    return bad != 0;
}
