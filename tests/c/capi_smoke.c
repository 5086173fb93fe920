/*
 * capi_smoke.c — exercises libdpf_hip.so through include/dpf_hip.h from
 * plain C (no Python, no torch), the way a cgo / JNI / FFI caller would.
 * Mirrors the reference's property tests (dpf/dpf_test.go:32-73): the XOR of
 * the two shares is the point function, for Eval and EvalFull, plus a
 * batched EvalFull and the PIR host API.  Exit status 0 = pass.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dpf_hip.h"

#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fprintf(stderr, " (%s)\n", dpf_last_error()); \
            return 1;                         \
        }                                     \
    } while (0)

static int bit(const uint8_t* b, uint64_t x) { return (b[x >> 3] >> (x & 7)) & 1; }

int main(void) {
    CHECK(dpf_gpu_init(1) >= 1, "no gfx950 device");

    /* TestEval shape: logN=8, alpha=123 */
    {
        const uint32_t logN = 8;
        size_t kl = dpf_key_len(logN);
        uint8_t* ka = malloc(kl);
        uint8_t* kb = malloc(kl);
        CHECK(dpf_gen(123, logN, ka, kb) == DPF_OK, "gen");
        for (uint64_t x = 0; x < 256; ++x) {
            uint8_t a, b;
            CHECK(dpf_eval(ka, kl, x, logN, &a) == DPF_OK && dpf_eval(kb, kl, x, logN, &b) == DPF_OK, "eval");
            CHECK((uint8_t)(a ^ b) == (x == 123), "Eval shares at x=%llu", (unsigned long long)x);
        }
        free(ka);
        free(kb);
    }
    /* TestEvalFull / TestEvalFullShort shapes */
    {
        const uint32_t cases[2][2] = {{9, 128}, {3, 1}};
        for (int c = 0; c < 2; ++c) {
            uint32_t logN = cases[c][0];
            uint64_t alpha = cases[c][1];
            size_t kl = dpf_key_len(logN), ol = dpf_evalfull_len(logN);
            uint8_t *ka = malloc(kl), *kb = malloc(kl), *fa = malloc(ol), *fb = malloc(ol);
            CHECK(dpf_gen(alpha, logN, ka, kb) == DPF_OK, "gen");
            CHECK(dpf_evalfull(ka, kl, logN, fa) == DPF_OK && dpf_evalfull(kb, kl, logN, fb) == DPF_OK, "evalfull");
            for (uint64_t x = 0; x < (1ull << logN); ++x)
                CHECK((bit(fa, x) ^ bit(fb, x)) == (x == alpha), "EvalFull shares logN=%u x=%llu", logN,
                      (unsigned long long)x);
            free(ka); free(kb); free(fa); free(fb);
        }
    }
    /* batched EvalFull at logN=20 and PIR through the host API */
    {
        const uint32_t logN = 20;
        const size_t n = 16;
        size_t kl = dpf_key_len(logN), ol = dpf_evalfull_len(logN);
        uint64_t alphas[16];
        uint8_t s0[16 * 16], s1[16 * 16];
        for (size_t i = 0; i < n; ++i) {
            alphas[i] = (i * 0x9E3779B97F4A7C15ull) >> 44;
            for (int j = 0; j < 16; ++j) {
                s0[i * 16 + j] = (uint8_t)(i * 31 + j * 7);
                s1[i * 16 + j] = (uint8_t)(i * 17 + j * 13 + 1);
            }
        }
        uint8_t *ka = malloc(n * kl), *kb = malloc(n * kl);
        uint8_t *fa = malloc(n * ol), *fb = malloc(n * ol);
        CHECK(dpf_gen_batch_seeded(alphas, logN, s0, s1, n, ka, kb, 0) == DPF_OK, "gen batch");
        CHECK(dpf_evalfull_batch(ka, kl, n, logN, fa, 0) == DPF_OK, "evalfull batch a");
        CHECK(dpf_evalfull_batch(kb, kl, n, logN, fb, 0) == DPF_OK, "evalfull batch b");
        for (size_t i = 0; i < n; ++i) {
            size_t ones = 0;
            for (size_t b = 0; b < ol; ++b) ones += (size_t)__builtin_popcount(fa[i * ol + b] ^ fb[i * ol + b]);
            CHECK(ones == 1 && bit(fa + i * ol, alphas[i]) != bit(fb + i * ol, alphas[i]), "batch key %zu", i);
        }
        const uint64_t nrec = 1ull << logN;
        uint8_t* db = malloc(nrec * 32);
        for (uint64_t r = 0; r < nrec * 32; ++r) db[r] = (uint8_t)(r * 2654435761u >> 13);
        void* h = NULL;
        CHECK(dpf_pir_db_create(db, nrec, logN, 1, &h) == DPF_OK, "pir db");
        uint8_t *aa = malloc(n * 32), *ab = malloc(n * 32);
        CHECK(dpf_pir_answer(h, ka, kl, n, aa) == DPF_OK && dpf_pir_answer(h, kb, kl, n, ab) == DPF_OK, "pir answer");
        for (size_t i = 0; i < n; ++i)
            for (int b = 0; b < 32; ++b)
                CHECK((uint8_t)(aa[i * 32 + b] ^ ab[i * 32 + b]) == db[alphas[i] * 32 + b], "PIR record %zu", i);
        dpf_pir_db_free(h);
        free(db); free(aa); free(ab); free(ka); free(kb); free(fa); free(fb);
    }
    /* the reference's panics become error codes */
    {
        uint8_t k[64];
        CHECK(dpf_gen(8, 3, k, k) == DPF_ERR_PARAM, "Gen alpha >= 2^logN must fail");
        CHECK(dpf_gen(0, 64, k, k) == DPF_ERR_PARAM, "Gen logN > 63 must fail");
        uint8_t out[16];
        CHECK(dpf_evalfull(k, 40, 20, out) == DPF_ERR_KEYLEN, "short key must fail");
    }
    dpf_gpu_shutdown();
    printf("capi_smoke: all checks passed\n");
    return 0;
}
