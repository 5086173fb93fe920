// host_eval.cpp — the small-call path of the drop-in API: the reference's
// single-key Eval and EvalFull (dpf/dpf.go:171-211, 213-262) on the host's
// AES units, for calls too small to amortise a GPU round trip (SURVEY §8b:
// "Single-key EvalFull/Eval may route to the CPU path below a size
// threshold, since they are latency-bound").  This is product code, not the
// oracle: a pipelined restatement on AES-NI / VAES that evaluates only what
// the output needs, routed by dpf_capi.hip (route_host_*) and only when a
// gfx950 device is open, so it never stands in for a missing GPU.
//
// Exactness rules kept: t values are bytes, XORed as bytes and
// tested != 0 (dpf.go:185-193, 205, 218, 230-237); the root seed is used
// without clearing its LSB (:175, :245); the final CW is k[len-16:] (:206,
// :219); logN < 7 gives 16 output bytes (:248); Eval reads bit x&127 of the
// final block whatever the high bits of x (:207-209).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include <immintrin.h>

#include "aes_consts.hpp"
#include "dpf_internal.hpp"

namespace dpfh {

namespace {

struct alignas(16) Rk {
    uint8_t b[176];
};

Rk rk_bytes(const dpfc::RoundKeys& k) {
    Rk r;
    for (int i = 0; i < 44; ++i) memcpy(r.b + 4 * i, &k.w[i], 4);
    return r;
}

const Rk kRkLb = rk_bytes(dpfc::kRkL);
const Rk kRkRb = rk_bytes(dpfc::kRkR);

// VAES when the CPU has it; DPF_HOST_ISA=aesni forces the 128-bit AES-NI
// form (the tests run both).
bool has_vaes() {
    static const bool hw = __builtin_cpu_supports("vaes") && __builtin_cpu_supports("avx512f");
    const char* e = getenv("DPF_HOST_ISA");
    return hw && !(e && e[0] == 'a');
}

// ---------------------------------------------------------------- Eval ---
// Only the child on x's path is computed: stop + 1 AES-MMO per query (the
// reference computes both children, 2*stop + 1).  kQ queries in flight, so
// kQ independent AES chains hide the AESENC latency.
constexpr int kQ = 8;

__attribute__((target("aes,sse4.1"))) void eval_group(const uint8_t* const* keys, const size_t* klens,
                                                      const uint64_t* xs, int n, uint32_t logN, uint8_t* out) {
    __m128i rl[11], rr[11];
    for (int r = 0; r < 11; ++r) {
        rl[r] = _mm_load_si128((const __m128i*)(kRkLb.b + 16 * r));
        rr[r] = _mm_load_si128((const __m128i*)(kRkRb.b + 16 * r));
    }
    const uint32_t stop = stop_of(logN);
    const __m128i lsb = _mm_cvtsi32_si128(1);
    __m128i s[kQ];
    uint8_t t[kQ];
    for (int q = 0; q < n; ++q) {
        s[q] = _mm_loadu_si128((const __m128i*)keys[q]);          // dpf.go:175: no LSB clear
        t[q] = keys[q][16];
    }
    for (uint32_t i = 0; i < stop; ++i) {
        __m128i st[kQ];
        bool right[kQ];
        const __m128i* rk[kQ];          // the path child's key schedule: no per-round select
        for (int q = 0; q < n; ++q) {
            right[q] = path_bit(xs[q], (uint64_t)logN - 1 - i) != 0;   // dpf.go:194-200
            rk[q] = right[q] ? rr : rl;
            st[q] = _mm_xor_si128(s[q], rk[q][0]);
        }
        for (int r = 1; r < 10; ++r)
            for (int q = 0; q < n; ++q) st[q] = _mm_aesenc_si128(st[q], rk[q][r]);
        for (int q = 0; q < n; ++q) {
            const __m128i c = _mm_xor_si128(_mm_aesenclast_si128(st[q], rk[q][10]), s[q]);
            const uint8_t* rec = keys[q] + 17 + 18 * (size_t)i;
            uint8_t tc = (uint8_t)(_mm_cvtsi128_si32(c) & 1);      // getT (dpf.go:46-48)
            __m128i sc = _mm_andnot_si128(lsb, c);                 // clr (:50-52)
            if (t[q] != 0) {                                       // :185-193
                sc = _mm_xor_si128(sc, _mm_loadu_si128((const __m128i*)rec));
                tc ^= rec[16 + (right[q] ? 1 : 0)];
            }
            s[q] = sc;
            t[q] = tc;
        }
    }
    __m128i st[kQ];
    for (int q = 0; q < n; ++q) st[q] = _mm_xor_si128(s[q], rl[0]);
    for (int r = 1; r < 10; ++r)
        for (int q = 0; q < n; ++q) st[q] = _mm_aesenc_si128(st[q], rl[r]);
    for (int q = 0; q < n; ++q) {
        __m128i c = _mm_xor_si128(_mm_aesenclast_si128(st[q], rl[10]), s[q]);   // :204
        if (t[q] != 0) c = _mm_xor_si128(c, _mm_loadu_si128((const __m128i*)(keys[q] + klens[q] - 16)));   // :205-206
        alignas(16) uint8_t b[16];
        _mm_store_si128((__m128i*)b, c);
        const uint32_t bit = (uint32_t)(xs[q] & 127);
        out[q] = (uint8_t)((b[bit / 8] >> (bit % 8)) & 1);         // :207-209
    }
}

// ------------------------------------------------------------- EvalFull ---
// Breadth-first by level (leaf order = index order, like the reference's
// DFS cursor, dpf.go:239-240), every level's nodes independent: the two
// children of a node are one pair of AES chains, 8 nodes (16 chains) in
// flight per group, and the leaf conversion 4 blocks per zmm under VAES.
struct Level {
    std::vector<__m128i> s;
    std::vector<uint8_t> t;
};

// Children of nodes [0, n) of level i into `nx` (2n nodes); AES-NI form.
__attribute__((target("aes,sse4.1"))) void expand_level_ni(const Level& cur, Level& nx, size_t n, const uint8_t* rec) {
    __m128i rl[11], rr[11];
    for (int r = 0; r < 11; ++r) {
        rl[r] = _mm_load_si128((const __m128i*)(kRkLb.b + 16 * r));
        rr[r] = _mm_load_si128((const __m128i*)(kRkRb.b + 16 * r));
    }
    const __m128i lsb = _mm_cvtsi32_si128(1);
    const __m128i scw = _mm_loadu_si128((const __m128i*)rec);
    const uint8_t tlcw = rec[16], trcw = rec[17];
    constexpr int G = 8;
    for (size_t j0 = 0; j0 < n; j0 += G) {
        const int g = (int)(n - j0 < (size_t)G ? n - j0 : (size_t)G);
        __m128i x[G], a[G], b[G];
        for (int q = 0; q < g; ++q) {
            x[q] = cur.s[j0 + q];
            a[q] = _mm_xor_si128(x[q], rl[0]);
            b[q] = _mm_xor_si128(x[q], rr[0]);
        }
        for (int r = 1; r < 10; ++r)
            for (int q = 0; q < g; ++q) {
                a[q] = _mm_aesenc_si128(a[q], rl[r]);
                b[q] = _mm_aesenc_si128(b[q], rr[r]);
            }
        for (int q = 0; q < g; ++q) {
            const __m128i cl = _mm_xor_si128(_mm_aesenclast_si128(a[q], rl[10]), x[q]);
            const __m128i cr = _mm_xor_si128(_mm_aesenclast_si128(b[q], rr[10]), x[q]);
            const uint8_t tp = cur.t[j0 + q];
            const __m128i m = _mm_set1_epi32(tp != 0 ? -1 : 0);
            const uint8_t tm = tp != 0 ? 0xff : 0;
            const size_t k = 2 * (j0 + q);
            nx.s[k] = _mm_xor_si128(_mm_andnot_si128(lsb, cl), _mm_and_si128(m, scw));   // dpf.go:229-238
            nx.s[k + 1] = _mm_xor_si128(_mm_andnot_si128(lsb, cr), _mm_and_si128(m, scw));
            nx.t[k] = (uint8_t)((_mm_cvtsi128_si32(cl) & 1) ^ (tlcw & tm));
            nx.t[k + 1] = (uint8_t)((_mm_cvtsi128_si32(cr) & 1) ^ (trcw & tm));
        }
    }
}

__attribute__((target("vaes,avx512f,aes,sse4.1"))) void expand_level_vaes(const Level& cur, Level& nx, size_t n,
                                                                          const uint8_t* rec) {
    __m512i rk[11];
    for (int r = 0; r < 11; ++r) {
        const __m128i l = _mm_load_si128((const __m128i*)(kRkLb.b + 16 * r));
        const __m128i rr = _mm_load_si128((const __m128i*)(kRkRb.b + 16 * r));
        rk[r] = _mm512_inserti32x4(_mm512_inserti32x4(_mm512_inserti32x4(_mm512_castsi128_si512(l), rr, 1), l, 2),
                                   rr, 3);                                              // [L|R|L|R]
    }
    const __m128i lsb = _mm_cvtsi32_si128(1);
    const __m128i scw = _mm_loadu_si128((const __m128i*)rec);
    const uint8_t tlcw = rec[16], trcw = rec[17];
    constexpr int Z = 8;   // zmm in flight: 16 nodes
    for (size_t j0 = 0; j0 < n; j0 += 2 * Z) {
        const size_t left = n - j0;
        const int z = (int)(left >= 2 * (size_t)Z ? Z : (left + 1) / 2);
        __m512i x[Z], st[Z];
        for (int q = 0; q < z; ++q) {
            const size_t ja = j0 + 2 * q, jb = ja + 1 < n ? ja + 1 : ja;
            const __m512i a = _mm512_broadcast_i32x4(cur.s[ja]);
            x[q] = _mm512_inserti32x4(_mm512_inserti32x4(a, cur.s[jb], 2), cur.s[jb], 3);   // [sa|sa|sb|sb]
            st[q] = _mm512_xor_si512(x[q], rk[0]);
        }
        for (int r = 1; r < 10; ++r)
            for (int q = 0; q < z; ++q) st[q] = _mm512_aesenc_epi128(st[q], rk[r]);
        for (int q = 0; q < z; ++q) {
            const __m512i o = _mm512_xor_si512(_mm512_aesenclast_epi128(st[q], rk[10]), x[q]);
            const __m128i c[4] = {_mm512_castsi512_si128(o), _mm512_extracti32x4_epi32(o, 1),
                                  _mm512_extracti32x4_epi32(o, 2), _mm512_extracti32x4_epi32(o, 3)};
            for (int h = 0; h < 2; ++h) {
                const size_t j = j0 + 2 * q + h;
                if (j >= n) break;
                const uint8_t tp = cur.t[j];
                const __m128i m = _mm_set1_epi32(tp != 0 ? -1 : 0);
                const uint8_t tm = tp != 0 ? 0xff : 0;
                nx.s[2 * j] = _mm_xor_si128(_mm_andnot_si128(lsb, c[2 * h]), _mm_and_si128(m, scw));
                nx.s[2 * j + 1] = _mm_xor_si128(_mm_andnot_si128(lsb, c[2 * h + 1]), _mm_and_si128(m, scw));
                nx.t[2 * j] = (uint8_t)((_mm_cvtsi128_si32(c[2 * h]) & 1) ^ (tlcw & tm));
                nx.t[2 * j + 1] = (uint8_t)((_mm_cvtsi128_si32(c[2 * h + 1]) & 1) ^ (trcw & tm));
            }
        }
    }
}

// Leaves: out[16j..] = MMO_L(s_j) ^ (t_j != 0 ? finalCW : 0)  (dpf.go:217-223).
__attribute__((target("aes,sse4.1"))) void leaves_ni(const Level& cur, size_t n, const uint8_t* fcw, uint8_t* out) {
    __m128i rl[11];
    for (int r = 0; r < 11; ++r) rl[r] = _mm_load_si128((const __m128i*)(kRkLb.b + 16 * r));
    const __m128i f = _mm_loadu_si128((const __m128i*)fcw);
    constexpr int G = 8;
    for (size_t j0 = 0; j0 < n; j0 += G) {
        const int g = (int)(n - j0 < (size_t)G ? n - j0 : (size_t)G);
        __m128i st[G];
        for (int q = 0; q < g; ++q) st[q] = _mm_xor_si128(cur.s[j0 + q], rl[0]);
        for (int r = 1; r < 10; ++r)
            for (int q = 0; q < g; ++q) st[q] = _mm_aesenc_si128(st[q], rl[r]);
        for (int q = 0; q < g; ++q) {
            const __m128i m = _mm_set1_epi32(cur.t[j0 + q] != 0 ? -1 : 0);
            const __m128i c = _mm_xor_si128(_mm_aesenclast_si128(st[q], rl[10]), cur.s[j0 + q]);
            _mm_storeu_si128((__m128i*)(out + 16 * (j0 + q)), _mm_xor_si128(c, _mm_and_si128(m, f)));
        }
    }
}

__attribute__((target("vaes,avx512f,aes,sse4.1"))) void leaves_vaes(const Level& cur, size_t n, const uint8_t* fcw,
                                                                    uint8_t* out) {
    __m512i rk[11];
    for (int r = 0; r < 11; ++r) rk[r] = _mm512_broadcast_i32x4(_mm_load_si128((const __m128i*)(kRkLb.b + 16 * r)));
    const __m512i f = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)fcw));
    constexpr int Z = 8;   // 32 leaves per group
    size_t j0 = 0;
    for (; j0 + 4 * Z <= n; j0 += 4 * Z) {
        __m512i x[Z], st[Z];
        for (int q = 0; q < Z; ++q) {
            x[q] = _mm512_loadu_si512((const void*)&cur.s[j0 + 4 * q]);
            st[q] = _mm512_xor_si512(x[q], rk[0]);
        }
        for (int r = 1; r < 10; ++r)
            for (int q = 0; q < Z; ++q) st[q] = _mm512_aesenc_epi128(st[q], rk[r]);
        for (int q = 0; q < Z; ++q) {
            const uint8_t* tt = &cur.t[j0 + 4 * q];
            const __mmask16 m = (__mmask16)((tt[0] ? 0x000f : 0) | (tt[1] ? 0x00f0 : 0) | (tt[2] ? 0x0f00 : 0) |
                                            (tt[3] ? 0xf000 : 0));
            __m512i c = _mm512_xor_si512(_mm512_aesenclast_epi128(st[q], rk[10]), x[q]);
            c = _mm512_mask_xor_epi32(c, m, c, f);
            _mm512_storeu_si512((void*)(out + 16 * (j0 + 4 * q)), c);
        }
    }
    if (j0 < n) {   // tail: fewer than 32 leaves
        Level tail;
        tail.s.assign(cur.s.begin() + (ptrdiff_t)j0, cur.s.begin() + (ptrdiff_t)n);
        tail.t.assign(cur.t.begin() + (ptrdiff_t)j0, cur.t.begin() + (ptrdiff_t)n);
        leaves_ni(tail, n - j0, fcw, out + 16 * j0);
    }
}

}  // namespace

bool host_eval_available() { return host_has_aesni(); }
bool host_eval_vaes() { return has_vaes(); }

void eval_batch_host(const uint8_t* keys, size_t klen, size_t nkeys, const uint64_t* xs, size_t ppk, uint32_t logN,
                     uint8_t* out) {
    const uint8_t* kp[kQ];
    size_t kls[kQ];
    uint64_t xq[kQ];
    const size_t nq = nkeys * ppk;
    for (size_t q0 = 0; q0 < nq; q0 += kQ) {
        const int n = (int)(nq - q0 < (size_t)kQ ? nq - q0 : (size_t)kQ);
        for (int q = 0; q < n; ++q) {
            kp[q] = keys + ((q0 + q) / ppk) * klen;
            kls[q] = klen;
            xq[q] = xs[q0 + q];
        }
        eval_group(kp, kls, xq, n, logN, out + q0);
    }
}

void evalfull_host(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out) {
    const uint32_t stop = stop_of(logN);
    const size_t leaves = (size_t)1 << stop;
    Level a, b;
    a.s.resize(leaves);
    a.t.resize(leaves);
    b.s.resize(leaves);
    b.t.resize(leaves);
    a.s[0] = _mm_loadu_si128((const __m128i*)key);               // dpf.go:245: no LSB clear
    a.t[0] = key[16];
    Level* cur = &a;
    Level* nx = &b;
    const bool vaes = has_vaes();
    for (uint32_t i = 0; i < stop; ++i) {
        const size_t n = (size_t)1 << i;
        const uint8_t* rec = key + 17 + 18 * (size_t)i;
        if (vaes) expand_level_vaes(*cur, *nx, n, rec);
        else expand_level_ni(*cur, *nx, n, rec);
        Level* t = cur;
        cur = nx;
        nx = t;
    }
    if (vaes) leaves_vaes(*cur, leaves, key + klen - 16, out);   // final CW at len-16 (:219)
    else leaves_ni(*cur, leaves, key + klen - 16, out);
}

}  // namespace dpfh
