/* small_call_bench.c — per-call latency of the single-key API at C level
 * (no Python): dpf_eval / dpf_evalfull through libdpf_hip.so in a given
 * small-call mode, beside the reference-style restatement (oracle_eval /
 * oracle_evalfull with AES-NI, one aes128MMO per call like dpf.go).
 * Usage: small_call_bench <logN> <mode 0 auto|1 gpu|2 host>.  One JSON line.
 * Build: gcc -O2 -I include tools/small_call_bench.c -Ldpf-go_amd/lib -ldpf_hip -Loracle -loracle */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "dpf_hip.h"

int oracle_eval(const uint8_t* k, size_t klen, uint64_t x, uint64_t logN, int use_aesni);
void oracle_evalfull(const uint8_t* key, size_t klen, uint64_t logN, uint8_t* out, int use_aesni);

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    const uint32_t logN = argc > 1 ? (uint32_t)atoi(argv[1]) : 20;
    const int mode = argc > 2 ? atoi(argv[2]) : DPF_SMALL_HOST;
    if (dpf_gpu_init(1) < 1) { fprintf(stderr, "no gpu: %s\n", dpf_last_error()); return 1; }
    dpf_set_small_call_path(mode);
    const size_t kl = dpf_key_len(logN), ol = dpf_evalfull_len(logN);
    uint8_t *ka = malloc(kl), *kb = malloc(kl), *out = malloc(ol), s0[16], s1[16], bit = 0;
    for (int i = 0; i < 16; ++i) { s0[i] = (uint8_t)(i * 7 + 1); s1[i] = (uint8_t)(i * 13 + 5); }
    const uint64_t alpha = 12345 % (1ull << logN);
    if (dpf_gen_seeded(alpha, logN, s0, s1, ka, kb) != DPF_OK) return 1;
    const int ne = 200000, nf = logN <= 20 ? 2000 : 100;
    unsigned acc = 0;
    double t0 = now();
    for (int i = 0; i < ne; ++i) { dpf_eval(ka, kl, (alpha + (uint64_t)i * 977) & ((1ull << logN) - 1), logN, &bit); acc += bit; }
    const double e_api = (now() - t0) / ne;
    t0 = now();
    for (int i = 0; i < ne; ++i) acc += (unsigned)oracle_eval(ka, kl, (alpha + (uint64_t)i * 977) & ((1ull << logN) - 1), logN, 1);
    const double e_ref = (now() - t0) / ne;
    t0 = now();
    for (int i = 0; i < nf; ++i) { dpf_evalfull(ka, kl, logN, out); acc += out[0]; }
    const double f_api = (now() - t0) / nf;
    t0 = now();
    for (int i = 0; i < nf; ++i) { oracle_evalfull(ka, kl, logN, out, 1); acc += out[0]; }
    const double f_ref = (now() - t0) / nf;
    printf("{\"logN\": %u, \"mode\": %d, \"eval_api_ns\": %.1f, \"eval_ref_style_ns\": %.1f, "
           "\"evalfull_api_us\": %.2f, \"evalfull_ref_style_us\": %.2f, \"chk\": %u}\n",
           logN, mode, e_api * 1e9, e_ref * 1e9, f_api * 1e6, f_ref * 1e6, acc);
    return 0;
}
