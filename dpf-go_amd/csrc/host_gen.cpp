// host_gen.cpp — host-side key generation for the engine (Gen stays on the
// host per the north star).  Restates dpf/dpf.go:71-169 with the PRG of
// dpf.go:59-69 on AES-NI (aes_amd64.s:51-82 semantics), falling back to a
// T-table software AES when the CPU lacks AES-NI.  Batched generation over
// host threads is SURVEY §8(f)1.
#include <errno.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <stdexcept>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "aes_consts.hpp"
#include "dpf_internal.hpp"
#include "../../include/dpf_hip.h"

namespace dpfh {

namespace {

struct RkBytes {
    alignas(16) uint8_t b[176];
};

RkBytes to_bytes(const dpfc::RoundKeys& k) {
    RkBytes r;
    for (int i = 0; i < 44; ++i) memcpy(r.b + 4 * i, &k.w[i], 4);   // words are little-endian columns
    return r;
}

const RkBytes kL = to_bytes(dpfc::kRkL);
const RkBytes kR = to_bytes(dpfc::kRkR);

bool cpu_has_aesni() {
    static const bool v = __builtin_cpu_supports("aes");
    return v;
}

__attribute__((target("aes,sse2"))) void mmo_ni(const RkBytes& rk, uint8_t* dst, const uint8_t* src) {
    __m128i x = _mm_loadu_si128((const __m128i*)src);
    __m128i s = _mm_xor_si128(x, _mm_load_si128((const __m128i*)rk.b));
    for (int r = 1; r < 10; ++r) s = _mm_aesenc_si128(s, _mm_load_si128((const __m128i*)(rk.b + 16 * r)));
    s = _mm_aesenclast_si128(s, _mm_load_si128((const __m128i*)(rk.b + 160)));
    _mm_storeu_si128((__m128i*)dst, _mm_xor_si128(s, x));
}

inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

void mmo_sw(const dpfc::RoundKeys& k, uint8_t* dst, const uint8_t* src) {
    uint32_t x[4], s[4], n[4];
    memcpy(x, src, 16);
    for (int c = 0; c < 4; ++c) s[c] = x[c] ^ k.w[c];
    const uint32_t* T = dpfc::kTe0.v;
    for (int r = 1; r < 10; ++r) {
        for (int c = 0; c < 4; ++c)
            n[c] = T[s[c] & 255] ^ rotl(T[(s[(c + 1) & 3] >> 8) & 255], 8) ^
                   rotl(T[(s[(c + 2) & 3] >> 16) & 255], 16) ^ rotl(T[s[(c + 3) & 3] >> 24], 24) ^ k.w[4 * r + c];
        memcpy(s, n, 16);
    }
    for (int c = 0; c < 4; ++c)
        n[c] = ((uint32_t)dpfc::kSbox.v[s[c] & 255] | ((uint32_t)dpfc::kSbox.v[(s[(c + 1) & 3] >> 8) & 255] << 8) |
                ((uint32_t)dpfc::kSbox.v[(s[(c + 2) & 3] >> 16) & 255] << 16) |
                ((uint32_t)dpfc::kSbox.v[s[(c + 3) & 3] >> 24] << 24)) ^
               k.w[40 + c];
    for (int c = 0; c < 4; ++c) n[c] ^= x[c];
    memcpy(dst, n, 16);
}

inline void mmo(bool right, uint8_t* dst, const uint8_t* src) {
    if (cpu_has_aesni()) mmo_ni(right ? kR : kL, dst, src);
    else mmo_sw(right ? dpfc::kRkR : dpfc::kRkL, dst, src);
}

inline void x16(uint8_t* d, const uint8_t* a, const uint8_t* b) {
    for (int i = 0; i < 16; ++i) d[i] = (uint8_t)(a[i] ^ b[i]);
}

// prg: left/right child with the control bit split off (dpf.go:59-69).
inline void prg(const uint8_t* seed, uint8_t* l, uint8_t* r, uint8_t& tl, uint8_t& tr) {
    mmo(false, l, seed);
    tl = l[0] & 1;
    l[0] &= 0xfe;
    mmo(true, r, seed);
    tr = r[0] & 1;
    r[0] &= 0xfe;
}

}  // namespace

bool host_has_aesni() { return cpu_has_aesni(); }

int gen_seeded(uint64_t alpha, uint32_t logN, const uint8_t seed0[16], const uint8_t seed1[16], uint8_t* ka,
               uint8_t* kb) {
    if (logN > 63 || alpha >= (1ull << logN)) return DPF_ERR_PARAM;   // dpf.go:72-74
    const uint32_t stop = logN >= 7 ? logN - 7 : 0;
    uint8_t s[2][16], ch[2][2][16], cw[16];
    uint8_t t[2];
    memcpy(s[0], seed0, 16);
    memcpy(s[1], seed1, 16);
    t[0] = s[0][0] & 1;                      // dpf.go:83-87
    t[1] = t[0] ^ 1;
    s[0][0] &= 0xfe;
    s[1][0] &= 0xfe;
    memcpy(ka, s[0], 16);
    ka[16] = t[0];
    memcpy(kb, s[1], 16);
    kb[16] = t[1];
    uint8_t* rec = ka + 17;
    for (uint32_t i = 0; i < stop; ++i, rec += 18) {
        uint8_t tc[2][2];
        for (int b = 0; b < 2; ++b) prg(s[b], ch[b][0], ch[b][1], tc[b][0], tc[b][1]);
        // keep = the child on alpha's path; lose = its sibling (dpf.go:106-157)
        const int keep = (alpha >> (logN - 1 - i)) & 1;
        const int lose = keep ^ 1;
        x16(cw, ch[0][lose], ch[1][lose]);
        uint8_t tcw[2];
        tcw[0] = (uint8_t)(tc[0][0] ^ tc[1][0] ^ (keep == 0 ? 1 : 0));
        tcw[1] = (uint8_t)(tc[0][1] ^ tc[1][1] ^ (keep == 1 ? 1 : 0));
        memcpy(rec, cw, 16);
        rec[16] = tcw[0];
        rec[17] = tcw[1];
        for (int b = 0; b < 2; ++b) {
            memcpy(s[b], ch[b][keep], 16);
            if (t[b]) x16(s[b], s[b], cw);
            t[b] = t[b] ? (uint8_t)(tc[b][keep] ^ tcw[keep]) : tc[b][keep];
        }
    }
    mmo(false, s[0], s[0]);                  // dpf.go:160-162
    mmo(false, s[1], s[1]);
    x16(cw, s[0], s[1]);
    cw[(alpha & 127) / 8] ^= (uint8_t)(1u << ((alpha & 127) % 8));
    memcpy(rec, cw, 16);
    memcpy(kb + 17, ka + 17, (size_t)18 * stop + 16);
    return DPF_OK;
}

int gen_random(uint64_t alpha, uint32_t logN, uint8_t* ka, uint8_t* kb) {
    uint8_t seeds[32];
    size_t got = 0;
    while (got < sizeof(seeds)) {
        ssize_t r = getrandom(seeds + got, sizeof(seeds) - got, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            return DPF_ERR_PARAM;
        }
        got += (size_t)r;
    }
    return gen_seeded(alpha, logN, seeds, seeds + 16, ka, kb);
}

static int usable_cpus() {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, CPU_COUNT(&set));
    return (int)std::max(1u, std::thread::hardware_concurrency());
}

int gen_batch_seeded(const uint64_t* alphas, uint32_t logN, const uint8_t* s0s, const uint8_t* s1s, size_t n,
                     uint8_t* kas, uint8_t* kbs, int nthreads) {
    if (logN > 63) return DPF_ERR_PARAM;
    for (size_t i = 0; i < n; ++i)
        if (alphas[i] >= (1ull << logN)) return DPF_ERR_PARAM;
    const size_t kl = 33 + 18 * (size_t)(logN >= 7 ? logN - 7 : 0);
    // Default: the CPUs this process may run on, at most 32; and no more
    // threads than 512-key chunks (a key pair takes ~1-3 us, a thread ~30 us).
    int nt = nthreads > 0 ? nthreads : std::min(32, usable_cpus());
    nt = (int)std::min<size_t>((size_t)nt, std::max<size_t>((n + 511) / 512, 1));
    auto work = [&](int tid) {
        for (size_t i = (size_t)tid; i < n; i += (size_t)nt)
            gen_seeded(alphas[i], logN, s0s + 16 * i, s1s + 16 * i, kas + kl * i, kbs + kl * i);
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& x : th) x.join();
    return DPF_OK;
}

}  // namespace dpfh
