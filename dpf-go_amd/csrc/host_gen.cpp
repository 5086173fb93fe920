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
#include <functional>
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

namespace {
// ---------------------------------------------------------------------------
// Pipelined Gen.  Gen's four MMOs per level (prg of both
// seeds, dpf.go:102-104) are independent, and so are different keys: a
// thread generates kBatch keys at once so that 4*kBatch AES chains are in
// flight.  VAES (AVX-512) carries one key's four MMOs in one zmm
// [s0|s0|s1|s1] under round keys [L|R|L|R]; without VAES the same schedule
// runs as four AES-NI chains per key.  Output is byte-identical to
// gen_seeded (tests: golden keys, host_sanity.c).
constexpr int kBatch = 8;

bool cpu_has_vaes() {
    static const bool v = __builtin_cpu_supports("vaes") && __builtin_cpu_supports("avx512f");
    return v;
}

// Per-key part of one level (dpf.go:106-158), kept in SSE registers (no
// byte stores + wide reloads, which stall store forwarding): c[0]=L(s0)
// c[1]=R(s0) c[2]=L(s1) c[3]=R(s1) are the MMO outputs, control bits still
// in byte 0.
struct KeyState {
    __m128i s[2];
    uint32_t t[2];
    uint64_t alpha;
    uint8_t* rec;
};

inline void level_post(KeyState& k, uint32_t logN, uint32_t i, const __m128i c_in[4]) {
    const __m128i lsb = _mm_cvtsi32_si128(1);
    uint32_t tc[2][2];
    __m128i c[4];
    for (int q = 0; q < 4; ++q) {
        tc[q >> 1][q & 1] = (uint32_t)_mm_cvtsi128_si32(c_in[q]) & 1u;
        c[q] = _mm_andnot_si128(lsb, c_in[q]);
    }
    const int keep = (int)((k.alpha >> (logN - 1 - i)) & 1);
    const int lose = keep ^ 1;
    const __m128i cw = _mm_xor_si128(c[lose], c[2 + lose]);
    const uint32_t tcw0 = tc[0][0] ^ tc[1][0] ^ (keep == 0 ? 1u : 0u);
    const uint32_t tcw1 = tc[0][1] ^ tc[1][1] ^ (keep == 1 ? 1u : 0u);
    _mm_storeu_si128((__m128i*)k.rec, cw);
    k.rec[16] = (uint8_t)tcw0;
    k.rec[17] = (uint8_t)tcw1;
    k.rec += 18;
    const uint32_t tk = keep ? tcw1 : tcw0;
    for (int b = 0; b < 2; ++b) {
        const __m128i m = _mm_set1_epi32(k.t[b] ? -1 : 0);
        k.s[b] = _mm_xor_si128(c[2 * b + keep], _mm_and_si128(m, cw));
        k.t[b] = k.t[b] ? (tc[b][keep] ^ tk) : tc[b][keep];
    }
}

inline void key_init(KeyState& k, uint64_t alpha, const uint8_t* seed0, const uint8_t* seed1, uint8_t* ka,
                     uint8_t* kb) {
    const __m128i lsb = _mm_cvtsi32_si128(1);
    const __m128i a = _mm_loadu_si128((const __m128i*)seed0), b = _mm_loadu_si128((const __m128i*)seed1);
    k.t[0] = seed0[0] & 1u;                  // dpf.go:83-87
    k.t[1] = k.t[0] ^ 1u;
    k.s[0] = _mm_andnot_si128(lsb, a);
    k.s[1] = _mm_andnot_si128(lsb, b);
    _mm_storeu_si128((__m128i*)ka, k.s[0]);
    ka[16] = (uint8_t)k.t[0];
    _mm_storeu_si128((__m128i*)kb, k.s[1]);
    kb[16] = (uint8_t)k.t[1];
    k.alpha = alpha;
    k.rec = ka + 17;
}

inline void key_final(KeyState& k, __m128i f0, __m128i f1, uint32_t stop, uint8_t* ka, uint8_t* kb) {
    alignas(16) uint8_t cw[16];
    _mm_store_si128((__m128i*)cw, _mm_xor_si128(f0, f1));   // dpf.go:160-165
    cw[(k.alpha & 127) / 8] ^= (uint8_t)(1u << ((k.alpha & 127) % 8));
    memcpy(k.rec, cw, 16);
    memcpy(kb + 17, ka + 17, (size_t)18 * stop + 16);
}

__attribute__((target("vaes,avx512f,aes,sse2"))) void gen_group_vaes(const uint64_t* alphas, uint32_t logN,
                                                                      const uint8_t* s0s, const uint8_t* s1s,
                                                                      int n, uint8_t* kas, uint8_t* kbs,
                                                                      size_t kl) {
    const uint32_t stop = logN >= 7 ? logN - 7 : 0;
    KeyState ks[kBatch];
    for (int j = 0; j < n; ++j) key_init(ks[j], alphas[j], s0s + 16 * j, s1s + 16 * j, kas + kl * j, kbs + kl * j);
    __m512i rkLR[11], rkL[11];
    for (int r = 0; r < 11; ++r) {
        const __m128i l = _mm_load_si128((const __m128i*)(kL.b + 16 * r));
        const __m128i rr = _mm_load_si128((const __m128i*)(kR.b + 16 * r));
        rkLR[r] = _mm512_inserti32x4(_mm512_inserti32x4(_mm512_inserti32x4(_mm512_castsi128_si512(l), rr, 1), l, 2),
                                     rr, 3);
        rkL[r] = _mm512_broadcast_i32x4(l);
    }
    for (uint32_t i = 0; i < stop; ++i) {
        __m512i x[kBatch], st[kBatch];
        for (int j = 0; j < n; ++j) {
            const __m512i a = _mm512_broadcast_i32x4(ks[j].s[0]);
            x[j] = _mm512_inserti32x4(_mm512_inserti32x4(a, ks[j].s[1], 2), ks[j].s[1], 3);
            st[j] = _mm512_xor_si512(x[j], rkLR[0]);
        }
        for (int r = 1; r < 10; ++r)
            for (int j = 0; j < n; ++j) st[j] = _mm512_aesenc_epi128(st[j], rkLR[r]);
        for (int j = 0; j < n; ++j) {
            const __m512i o = _mm512_xor_si512(_mm512_aesenclast_epi128(st[j], rkLR[10]), x[j]);
            const __m128i c[4] = {_mm512_castsi512_si128(o), _mm512_extracti32x4_epi32(o, 1),
                                  _mm512_extracti32x4_epi32(o, 2), _mm512_extracti32x4_epi32(o, 3)};
            level_post(ks[j], logN, i, c);
        }
    }
    // final: MMO_L of both seeds (dpf.go:160-162), two keys per zmm
    for (int j0 = 0; j0 < n; j0 += 2) {
        const int q1 = n - j0 < 2 ? j0 : j0 + 1;
        __m512i x = _mm512_castsi128_si512(ks[j0].s[0]);
        x = _mm512_inserti32x4(x, ks[j0].s[1], 1);
        x = _mm512_inserti32x4(x, ks[q1].s[0], 2);
        x = _mm512_inserti32x4(x, ks[q1].s[1], 3);
        __m512i stt = _mm512_xor_si512(x, rkL[0]);
        for (int r = 1; r < 10; ++r) stt = _mm512_aesenc_epi128(stt, rkL[r]);
        stt = _mm512_xor_si512(_mm512_aesenclast_epi128(stt, rkL[10]), x);
        key_final(ks[j0], _mm512_castsi512_si128(stt), _mm512_extracti32x4_epi32(stt, 1), stop, kas + kl * j0,
                  kbs + kl * j0);
        if (q1 != j0)
            key_final(ks[q1], _mm512_extracti32x4_epi32(stt, 2), _mm512_extracti32x4_epi32(stt, 3), stop,
                      kas + kl * q1, kbs + kl * q1);
    }
}

__attribute__((target("aes,sse2"))) void gen_group_ni(const uint64_t* alphas, uint32_t logN, const uint8_t* s0s,
                                                      const uint8_t* s1s, int n, uint8_t* kas, uint8_t* kbs,
                                                      size_t kl) {
    const uint32_t stop = logN >= 7 ? logN - 7 : 0;
    KeyState ks[kBatch];
    for (int j = 0; j < n; ++j) key_init(ks[j], alphas[j], s0s + 16 * j, s1s + 16 * j, kas + kl * j, kbs + kl * j);
    __m128i rl[11], rr[11];
    for (int r = 0; r < 11; ++r) {
        rl[r] = _mm_load_si128((const __m128i*)(kL.b + 16 * r));
        rr[r] = _mm_load_si128((const __m128i*)(kR.b + 16 * r));
    }
    for (uint32_t i = 0; i < stop; ++i) {
        __m128i x[kBatch][4], st[kBatch][4];
        for (int j = 0; j < n; ++j)
            for (int q = 0; q < 4; ++q) {
                x[j][q] = ks[j].s[q >> 1];
                st[j][q] = _mm_xor_si128(x[j][q], (q & 1) ? rr[0] : rl[0]);
            }
        for (int r = 1; r < 10; ++r)
            for (int j = 0; j < n; ++j)
                for (int q = 0; q < 4; ++q) st[j][q] = _mm_aesenc_si128(st[j][q], (q & 1) ? rr[r] : rl[r]);
        for (int j = 0; j < n; ++j) {
            __m128i c[4];
            for (int q = 0; q < 4; ++q)
                c[q] = _mm_xor_si128(_mm_aesenclast_si128(st[j][q], (q & 1) ? rr[10] : rl[10]), x[j][q]);
            level_post(ks[j], logN, i, c);
        }
    }
    for (int j = 0; j < n; ++j) {
        __m128i f[2];
        for (int b = 0; b < 2; ++b) {
            __m128i t = _mm_xor_si128(ks[j].s[b], rl[0]);
            for (int r = 1; r < 10; ++r) t = _mm_aesenc_si128(t, rl[r]);
            f[b] = _mm_xor_si128(_mm_aesenclast_si128(t, rl[10]), ks[j].s[b]);
        }
        key_final(ks[j], f[0], f[1], stop, kas + kl * j, kbs + kl * j);
    }
}

// kBatch keys (or fewer) of one logN; falls back to gen_seeded per key
// without AES-NI.
void gen_group(const uint64_t* alphas, uint32_t logN, const uint8_t* s0s, const uint8_t* s1s, int n, uint8_t* kas,
               uint8_t* kbs) {
    const size_t kl = 33 + 18 * (size_t)(logN >= 7 ? logN - 7 : 0);
    if (cpu_has_vaes())
        gen_group_vaes(alphas, logN, s0s, s1s, n, kas, kbs, kl);
    else if (cpu_has_aesni())
        gen_group_ni(alphas, logN, s0s, s1s, n, kas, kbs, kl);
    else
        for (int j = 0; j < n; ++j)
            gen_seeded(alphas[j], logN, s0s + 16 * j, s1s + 16 * j, kas + kl * j, kbs + kl * j);
}

}  // namespace

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
    // Threads take contiguous ranges, kBatch keys at a time (pipelined Gen).
    auto work = [&](int tid) {
        const size_t lo = n * (size_t)tid / (size_t)nt, hi = n * (size_t)(tid + 1) / (size_t)nt;
        for (size_t i = lo; i < hi; i += kBatch) {
            const int m = (int)std::min<size_t>(kBatch, hi - i);
            gen_group(alphas + i, logN, s0s + 16 * i, s1s + 16 * i, m, kas + kl * i, kbs + kl * i);
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& x : th) x.join();
    return DPF_OK;
}

// Key wire format.  A key is the reference's DPFkey bytes
// (dpf.go:7,89-92,111-112,137-138,165-167) and a batch is [n][key_len]
// contiguous, which is what Gen writes and every evaluation entry reads; so
// (de)serialising a batch is a gather / scatter of whole keys.  Large batches
// are copied on several threads (one 64-key block per task at least).
static void copy_keys(size_t n, size_t kl, const std::function<void(size_t)>& one) {
    const size_t bytes = n * kl;
    int nt = bytes < ((size_t)8 << 20) ? 1 : std::min(16, usable_cpus());
    nt = (int)std::min<size_t>((size_t)nt, std::max<size_t>(n / 64, 1));
    auto work = [&](int tid) {
        const size_t lo = n * (size_t)tid / (size_t)nt, hi = n * (size_t)(tid + 1) / (size_t)nt;
        for (size_t i = lo; i < hi; ++i) one(i);
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& x : th) x.join();
}

int keys_pack(const uint8_t* const* keys, const size_t* lens, size_t n, size_t key_len, uint8_t* out) {
    if (n == 0) return DPF_OK;
    if (!keys || !out || key_len == 0) return DPF_ERR_PARAM;
    for (size_t i = 0; i < n; ++i) {
        if (!keys[i]) return DPF_ERR_PARAM;
        if (lens && lens[i] != key_len) return DPF_ERR_KEYLEN;
    }
    copy_keys(n, key_len, [&](size_t i) { memcpy(out + i * key_len, keys[i], key_len); });
    return DPF_OK;
}

int keys_unpack(const uint8_t* packed, size_t key_len, size_t n, uint8_t* const* keys) {
    if (n == 0) return DPF_OK;
    if (!keys || !packed || key_len == 0) return DPF_ERR_PARAM;
    for (size_t i = 0; i < n; ++i)
        if (!keys[i]) return DPF_ERR_PARAM;
    copy_keys(n, key_len, [&](size_t i) { memcpy(keys[i], packed + i * key_len, key_len); });
    return DPF_OK;
}

}  // namespace dpfh
