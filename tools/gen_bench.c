/* gen_bench.c — host Gen throughput: key pairs/s at a logN,
 * one thread, for the one-key-at-a-time path (dpf_gen_seeded: one AES-NI
 * block per call, like the reference's Gen) and the pipelined batch path
 * (dpf_gen_batch_seeded, nthreads = 1 and = argv[2]).
 * Usage: gen_bench [logN=20] [threads=16] [nkeys=200000] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dpf_hip.h"

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char** argv) {
    uint32_t logN = argc > 1 ? (uint32_t)atoi(argv[1]) : 20;
    int th = argc > 2 ? atoi(argv[2]) : 16;
    size_t n = argc > 3 ? (size_t)atol(argv[3]) : 200000;
    size_t kl = dpf_key_len(logN);
    uint64_t* al = malloc(n * 8);
    uint8_t* s = malloc(n * 32);
    uint8_t* ka = malloc(n * kl);
    uint8_t* kb = malloc(n * kl);
    for (size_t i = 0; i < n; ++i) {
        al[i] = (i * 0x9E3779B97F4A7C15ull) >> (64 - (logN ? logN : 1));
        if (logN == 0) al[i] = 0;
        for (int j = 0; j < 32; ++j) s[32 * i + j] = (uint8_t)(i * 131 + j * 7);
    }
    memset(ka, 0, n * kl);
    memset(kb, 0, n * kl);
    size_t n1 = n / 4;
    double t0 = now();
    for (size_t i = 0; i < n1; ++i) dpf_gen_seeded(al[i], logN, s + 32 * i, s + 32 * i + 16, ka + kl * i, kb + kl * i);
    double single = n1 / (now() - t0);
    dpf_gen_batch_seeded(al, logN, s, s + 16, 1000, ka, kb, 1);
    t0 = now();
    dpf_gen_batch_seeded(al, logN, s, s + 16, n, ka, kb, 1);
    double batch1 = n / (now() - t0);
    t0 = now();
    dpf_gen_batch_seeded(al, logN, s, s + 16, n, ka, kb, th);
    double batchn = n / (now() - t0);
    printf("{\"logN\": %u, \"single_call_pairs_per_s_1core\": %.0f, \"batch_pairs_per_s_1core\": %.0f, "
           "\"batch_pairs_per_s\": %.0f, \"threads\": %d, \"speedup_1core\": %.2f}\n",
           logN, single, batch1, batchn, th, batch1 / single);
    return 0;
}
