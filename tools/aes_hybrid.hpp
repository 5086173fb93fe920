// aes_hybrid.hpp — AES-128-MMO with both PRG back ends in ONE instruction
// stream (device code): T-table blocks (LDS lookups, aes_ttable.hpp) and a
// byte-sliced set (VALU only, aes_bytesliced.hpp) advanced round by round in
// lockstep, so each wave keeps the LDS pipe and the VALU busy at once.
//
// Implements aes128MMO (dpf/aes_amd64.s:51-82), dst = AES_k(src) ^ src, for
// the two fixed PRG keys (dpf/dpf.go:23-24).
//
// Why: on gfx950 the T-table back end is LDS-bound (160 ds_read_b32 per
// block; ~0.8 of the LDS array, VALU ~45% idle) and the byte-sliced back end
// is VALU-bound (~533 lane-ops per block, LDS idle).  A wave that runs NT
// T-table blocks and one 8-block byte-sliced set per round loads both pipes;
// NT = 14 balances them.
//
// Round keys change every iteration of the (not unrolled) round loop, so
// they cannot be instruction literals; they come from __constant__ tables
// through scalar loads (wave-uniform).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../dpf-go_amd/csrc/aes_bytesliced.hpp"
#include "../dpf-go_amd/csrc/aes_consts.hpp"
#include "../dpf-go_amd/csrc/aes_ttable.hpp"

namespace dpfk {
namespace hy {

// T-table round keys: rk16[key][round][col] = rotl(rk, 16) (rounds 1..9, the
// pre-rotation XOR of a column, aes_ttable.hpp aes_round), rk[key][round][col]
// plain (rounds 0 and 10).
struct TtKeys {
    uint32_t rk16[2][11][4];
    uint32_t rk[2][11][4];
};
constexpr TtKeys make_ttkeys() {
    TtKeys t = {};
    for (int key = 0; key < 2; ++key) {
        const dpfc::RoundKeys& K = key ? dpfc::kRkR : dpfc::kRkL;
        for (int r = 0; r < 11; ++r)
            for (int c = 0; c < 4; ++c) {
                t.rk[key][r][c] = K.w[4 * r + c];
                t.rk16[key][r][c] = crotl(K.w[4 * r + c], 16);
            }
    }
    return t;
}
static __constant__ TtKeys c_ttk = make_ttkeys();

// One middle T-table round with run-time round key words (already rotl 16).
__device__ __forceinline__ void tt_round(const uint8_t* tab, uint32_t lo, Blk& s, uint32_t k0, uint32_t k1,
                                         uint32_t k2, uint32_t k3) {
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk16) {
        uint32_t ta = tl<0>(tab, a, lo), tb = tl<1, true>(tab, b, lo), tc = tl<2>(tab, c, lo),
                 td = tl<3, true>(tab, d, lo);
        return xor3(ta, tb, rotl(xor3(tc, td, rk16), 16));
    };
    uint32_t n0 = col(s.c0, s.c1, s.c2, s.c3, k0);
    uint32_t n1 = col(s.c1, s.c2, s.c3, s.c0, k1);
    uint32_t n2 = col(s.c2, s.c3, s.c0, s.c1, k2);
    uint32_t n3 = col(s.c3, s.c0, s.c1, s.c2, k3);
    s.c0 = n0; s.c1 = n1; s.c2 = n2; s.c3 = n3;
}

// Final T-table round (S-box from byte 1 of Te0, ShiftRows, AddRoundKey 10).
__device__ __forceinline__ void tt_last(const uint8_t* tab, uint32_t lo, Blk& s, uint32_t k0, uint32_t k1, uint32_t k2,
                                        uint32_t k3) {
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
        uint32_t la = tl<0>(tab, a, lo), lb = tl<1>(tab, b, lo), lc = tl<2>(tab, c, lo), ld = tl<3>(tab, d, lo);
        uint32_t p = __builtin_amdgcn_perm(lb, la, 0x0c0c0501u);   // {la.b1, lb.b1, 0, 0}
        uint32_t q = __builtin_amdgcn_perm(ld, lc, 0x05010c0cu);   // {0, 0, lc.b1, ld.b1}
        return __builtin_amdgcn_bitop3_b32(p, q, rk, kOrXor);
    };
    uint32_t n0 = col(s.c0, s.c1, s.c2, s.c3, k0);
    uint32_t n1 = col(s.c1, s.c2, s.c3, s.c0, k1);
    uint32_t n2 = col(s.c2, s.c3, s.c0, s.c1, k2);
    uint32_t n3 = col(s.c3, s.c0, s.c1, s.c2, k3);
    s.c0 = n0; s.c1 = n1; s.c2 = n2; s.c3 = n3;
}

// Lockstep MMO of NT T-table blocks and one byte-sliced set (8 blocks).
// T-table block b has key (b & 1) (0 = L, 1 = R) and input x[b >> 1]: the
// two PRG halves of NT/2 parent seeds (dpf.go:59-69).  The byte-sliced set
// X (aes_bytesliced.hpp layout) uses key L: leaf conversions (dpf.go:215-217).
// On return s[b] = AES(x[b>>1]) ^ x[b>>1] and O = AES_L(X) ^ X.
template <int NT>
__device__ __forceinline__ void mmo_lockstep(const uint8_t* tab, uint32_t lo, const Blk (&x)[NT / 2], Blk (&s)[NT],
                                             const uint32_t (&X)[32], uint32_t (&O)[32]) {
    static_assert(NT % 2 == 0, "T-table blocks come in L/R pairs");
    const uint32_t* rkb = &bs::c_rkbs.w[0][0][0];          // key L
    const uint32_t* mkb = &bs::c_mcks.w[0][0][0];
#pragma unroll
    for (int b = 0; b < NT; ++b) {
        const uint32_t k = b & 1;
        s[b] = {x[b >> 1].c0 ^ c_ttk.rk[k][0][0], x[b >> 1].c1 ^ c_ttk.rk[k][0][1],
                x[b >> 1].c2 ^ c_ttk.rk[k][0][2], x[b >> 1].c3 ^ c_ttk.rk[k][0][3]};
    }
    uint32_t st[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) st[w] = X[w] ^ rkb[w];
    bs::sub_bytes(st);
#pragma nounroll
    for (int rnd = 1; rnd < 10; ++rnd) {
        const uint32_t l0 = c_ttk.rk16[0][rnd][0], l1 = c_ttk.rk16[0][rnd][1], l2 = c_ttk.rk16[0][rnd][2],
                       l3 = c_ttk.rk16[0][rnd][3];
        const uint32_t r0 = c_ttk.rk16[1][rnd][0], r1 = c_ttk.rk16[1][rnd][1], r2 = c_ttk.rk16[1][rnd][2],
                       r3 = c_ttk.rk16[1][rnd][3];
#pragma unroll
        for (int b = 0; b < NT; ++b) {
            if (b & 1)
                tt_round(tab, lo, s[b], r0, r1, r2, r3);
            else
                tt_round(tab, lo, s[b], l0, l1, l2, l3);
        }
        bs::shift_rows(st);
        bs::mix_columns(st, mkb + 32 * rnd);
        bs::sub_bytes(st);
    }
#pragma unroll
    for (int b = 0; b < NT; ++b) {
        const uint32_t k = b & 1;
        tt_last(tab, lo, s[b], c_ttk.rk[k][10][0], c_ttk.rk[k][10][1], c_ttk.rk[k][10][2], c_ttk.rk[k][10][3]);
        s[b] = bxor(s[b], x[b >> 1]);
    }
    bs::shift_rows(st);
#pragma unroll
    for (int w = 0; w < 32; ++w) O[w] = bs::x3(st[w], rkb[320 + w], X[w]);
}

}  // namespace hy
}  // namespace dpfk
