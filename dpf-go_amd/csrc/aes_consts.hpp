// aes_consts.hpp — compile-time AES-128 constants for the DPF PRG.
//
// The reference expands its two fixed PRG keys once at package init
// (dpf/dpf.go:22-35 -> expandKeyAsm, dpf/aes_amd64.s:87-126).  Both keys are
// fixed, so here the whole schedule, the S-box and the T-table are derived by
// constexpr evaluation and become literals in the gfx950 code object and in
// the host library.  Nothing is computed at run time and no table is copied
// from anywhere: the S-box comes from GF(2^8) log/antilog tables (generator 3)
// plus the FIPS-197 affine map.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define DPF_HD __host__ __device__
#else
#define DPF_HD
#endif

namespace dpfc {

// dpf/dpf.go:23-24
constexpr uint8_t kPrfKeyL[16] = {36, 156, 50, 234, 92, 230, 49, 9, 174, 170, 205, 160, 98, 236, 29, 243};
constexpr uint8_t kPrfKeyR[16] = {209, 12, 199, 173, 29, 74, 44, 128, 194, 224, 14, 44, 2, 201, 110, 28};

constexpr uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

struct Bytes256 { uint8_t v[256]; };
struct Words256 { uint32_t v[256]; };
struct RoundKeys { uint32_t w[44]; };   // 11 round keys, 4 little-endian columns each

constexpr Bytes256 make_sbox() {
    uint8_t exp_t[256] = {};
    uint8_t log_t[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {         // 3 generates GF(2^8)*
        exp_t[i] = x;
        log_t[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xt(x));            // x *= 3
    }
    Bytes256 s = {};
    for (int a = 0; a < 256; ++a) {
        uint8_t inv = a ? exp_t[(255 - log_t[a]) % 255] : 0;
        uint8_t r = inv, acc = inv;
        for (int i = 0; i < 4; ++i) {
            r = (uint8_t)((r << 1) | (r >> 7));
            acc ^= r;
        }
        s.v[a] = (uint8_t)(acc ^ 0x63);
    }
    return s;
}

constexpr Bytes256 kSbox = make_sbox();

// Te0 in the little-endian column convention used by the kernels: a state
// column c is the u32 (b[4c] | b[4c+1]<<8 | b[4c+2]<<16 | b[4c+3]<<24), i.e.
// row r lives in byte r.  Te0[x] = MixColumns of (S[x],0,0,0) = (2s, s, s, 3s).
constexpr Words256 make_te0() {
    Words256 t = {};
    for (int a = 0; a < 256; ++a) {
        uint8_t s = kSbox.v[a];
        uint8_t s2 = xt(s);
        uint8_t s3 = (uint8_t)(s2 ^ s);
        t.v[a] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
    return t;
}

constexpr Words256 kTe0 = make_te0();

// FIPS-197 key expansion, words kept little-endian like the state columns.
constexpr RoundKeys expand(const uint8_t* key) {
    uint8_t rk[176] = {};
    const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
    for (int i = 0; i < 16; ++i) rk[i] = key[i];
    for (int i = 4; i < 44; ++i) {
        uint8_t t0 = rk[4 * (i - 1)], t1 = rk[4 * (i - 1) + 1], t2 = rk[4 * (i - 1) + 2], t3 = rk[4 * (i - 1) + 3];
        if (i % 4 == 0) {
            uint8_t u = t0;
            t0 = (uint8_t)(kSbox.v[t1] ^ rcon[i / 4 - 1]);
            t1 = kSbox.v[t2];
            t2 = kSbox.v[t3];
            t3 = kSbox.v[u];
        }
        rk[4 * i + 0] = (uint8_t)(rk[4 * (i - 4) + 0] ^ t0);
        rk[4 * i + 1] = (uint8_t)(rk[4 * (i - 4) + 1] ^ t1);
        rk[4 * i + 2] = (uint8_t)(rk[4 * (i - 4) + 2] ^ t2);
        rk[4 * i + 3] = (uint8_t)(rk[4 * (i - 4) + 3] ^ t3);
    }
    RoundKeys r = {};
    for (int i = 0; i < 44; ++i)
        r.w[i] = (uint32_t)rk[4 * i] | ((uint32_t)rk[4 * i + 1] << 8) | ((uint32_t)rk[4 * i + 2] << 16) |
                 ((uint32_t)rk[4 * i + 3] << 24);
    return r;
}

constexpr RoundKeys kRkL = expand(kPrfKeyL);
constexpr RoundKeys kRkR = expand(kPrfKeyR);

// FIPS-197 Appendix A.1 last round key for 2b7e1516..., guards the schedule.
constexpr uint8_t kFipsKey[16] = {0x2b, 0x7e, 0x15, 0x16, 0x28, 0xae, 0xd2, 0xa6,
                                  0xab, 0xf7, 0x15, 0x88, 0x09, 0xcf, 0x4f, 0x3c};
static_assert(expand(kFipsKey).w[43] == 0xa60c63b6u, "AES-128 key schedule mismatch (FIPS-197 A.1 w[43]=b6630ca6)");
static_assert(kSbox.v[0x00] == 0x63 && kSbox.v[0x53] == 0xed && kSbox.v[0xff] == 0x16, "S-box mismatch");

}  // namespace dpfc
