// aes_bytesliced.hpp — AES-128-MMO on gfx950 VALU, byte-sliced: 8 blocks per
// lane, no tables (device code).  The "bitsliced" back end of the north star
// (BASELINE configs[1] asks for bitsliced vs LDS T-table).
//
// Implements aes128MMO (dpf/aes_amd64.s:51-82), dst = AES_k(src) ^ src, for
// the two fixed PRG keys (dpf/dpf.go:23-24), on 8 independent blocks at once.
//
// Layout: a set of 8 blocks is 32 words w[8*row + plane]; bit (8*col + i)
// of w[8*row + plane] is bit `plane` of state byte (col, row) of block i.
// So one word is one bit plane of one state row for all 4 columns x 8
// blocks, and
//   SubBytes   = the S-box circuit over the 8 plane words of a row (82
//                v_bitop3_b32, aes_sbox_lut3.inc), 4 rows;
//   ShiftRows  = rotate row r's words right by 8r bits (v_alignbit);
//   MixColumns = XORs between rows (xtime is a renaming of planes), with
//                AddRoundKey folded into its constants (make_mcks);
//   AddRoundKey= scalar-operand XORs, only before round 1 and in round 10.
// A set is only 32 registers, so a lane can keep a depth-first stack of sets
// and the MMO feed-forward input in VGPRs (the 128-word layout of 32-block
// bitslicing cannot).  Block i of a memory block word c is bit q = 8c + i of
// a 32x32 bit-matrix transpose (transpose32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "aes_consts.hpp"

namespace dpfk {
namespace bs {

// Byte-sliced round keys: w[key][round][8*row + plane], byte c = 0xFF when
// bit `plane` of round-key byte (column c, row) is set.  key 0 = L, 1 = R.
struct RkBs {
    uint32_t w[2][11][32];
};

constexpr RkBs make_rkbs() {
    RkBs r = {};
    for (int key = 0; key < 2; ++key) {
        const dpfc::RoundKeys& K = key ? dpfc::kRkR : dpfc::kRkL;
        for (int rnd = 0; rnd < 11; ++rnd)
            for (int row = 0; row < 4; ++row)
                for (int plane = 0; plane < 8; ++plane) {
                    uint32_t v = 0;
                    for (int c = 0; c < 4; ++c) {
                        const uint32_t byte = (K.w[4 * rnd + c] >> (8 * row)) & 0xFFu;
                        if ((byte >> plane) & 1u) v |= 0xFFu << (8 * c);
                    }
                    r.w[key][rnd][8 * row + plane] = v;
                }
    }
    return r;
}

static __constant__ RkBs c_rkbs = make_rkbs();

// AddRoundKey folded into MixColumns.  MixColumns computes t_r = a_r ^
// a_{r+1} and out_r = xtime(t_r) ^ a_{r+1} ^ t_{r+2}; computing instead
// t'_r = t_r ^ c_r (same one v_bitop3) gives out_r ^ xtime(c_r) ^ c_{r+2}.
// Per column byte, xtime(c_r) ^ c_{r+2} = K_r (rounds 1..9) is solved as
// c_r = 5^-1 (K_{r+2} ^ 2 K_r) (the 2x2 system [[2,1],[1,2]] has det 5 != 0
// in GF(2^8)), so the 32 round-key XORs per round disappear.
constexpr uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        a = dpfc::xt(a);
        b >>= 1;
    }
    return p;
}
constexpr uint8_t ginv(uint8_t a) {
    for (int x = 1; x < 256; ++x)
        if (gmul(a, (uint8_t)x) == 1) return (uint8_t)x;
    return 0;
}
constexpr RkBs make_mcks() {
    RkBs r = {};
    const uint8_t inv5 = ginv(5);
    for (int key = 0; key < 2; ++key) {
        const dpfc::RoundKeys& K = key ? dpfc::kRkR : dpfc::kRkL;
        for (int rnd = 1; rnd < 10; ++rnd)
            for (int c = 0; c < 4; ++c) {
                uint8_t k[4] = {}, cc[4] = {};
                for (int row = 0; row < 4; ++row) k[row] = (uint8_t)(K.w[4 * rnd + c] >> (8 * row));
                for (int row = 0; row < 4; ++row) cc[row] = gmul(inv5, (uint8_t)(k[(row + 2) & 3] ^ gmul(2, k[row])));
                for (int row = 0; row < 4; ++row)
                    for (int plane = 0; plane < 8; ++plane)
                        if ((cc[row] >> plane) & 1u) r.w[key][rnd][8 * row + plane] |= 0xFFu << (8 * c);
            }
    }
    return r;
}
constexpr bool mck_ok() {   // xtime(c_r) ^ c_{r+2} == K_r for every byte
    const RkBs m = make_mcks();
    for (int key = 0; key < 2; ++key)
        for (int rnd = 1; rnd < 10; ++rnd)
            for (int c = 0; c < 4; ++c)
                for (int row = 0; row < 4; ++row) {
                    uint8_t cr = 0, c2 = 0;
                    for (int p = 0; p < 8; ++p) {
                        cr |= (uint8_t)(((m.w[key][rnd][8 * row + p] >> (8 * c)) & 1u) << p);
                        c2 |= (uint8_t)(((m.w[key][rnd][8 * ((row + 2) & 3) + p] >> (8 * c)) & 1u) << p);
                    }
                    const dpfc::RoundKeys& K = key ? dpfc::kRkR : dpfc::kRkL;
                    if ((uint8_t)(dpfc::xt(cr) ^ c2) != (uint8_t)(K.w[4 * rnd + c] >> (8 * row))) return false;
                }
    return true;
}
static_assert(mck_ok(), "MixColumns-folded round keys");
static __constant__ RkBs c_mcks = make_mcks();

// S-box over one row: st[j] = plane j (st[7] = MSB plane = circuit input U0).
__device__ __forceinline__ void sub_row(uint32_t* st) {
    const uint32_t u0 = st[7], u1 = st[6], u2 = st[5], u3 = st[4], u4 = st[3], u5 = st[2], u6 = st[1], u7 = st[0];
    uint32_t o0, o1, o2, o3, o4, o5, o6, o7;
#include "aes_sbox_lut3.inc"
    st[7] = o0; st[6] = o1; st[5] = o2; st[4] = o3; st[3] = o4; st[2] = o5; st[1] = o6; st[0] = o7;
}

__device__ __forceinline__ void sub_bytes(uint32_t (&st)[32]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sub_row(st + 8 * r);
}

// ShiftRows: new column c of row r = old column c + r -> rotate right 8r.
__device__ __forceinline__ void shift_rows(uint32_t (&st)[32]) {
#pragma unroll
    for (int r = 1; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) st[8 * r + j] = __builtin_amdgcn_alignbit(st[8 * r + j], st[8 * r + j], 8 * r);
}

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// MixColumns: out_r = xtime(a_r ^ a_{r+1}) ^ a_{r+1} ^ a_{r+2} ^ a_{r+3}
//           = xtime(t_r) ^ a_{r+1} ^ t_{r+2},  t_r = a_r ^ a_{r+1};
// xtime on planes: out0 = t7, out_j = t_{j-1} (^ t7 for j = 1, 3, 4).
// Planes are done from 7 down to 0 so that only t_*[7], t_*[j], t_*[j-1]
// and four outputs are live beside the state (16 words, not 64).
__device__ __forceinline__ void mix_columns(uint32_t (&st)[32], const uint32_t* __restrict__ ck) {
    uint32_t t7[4], tj[4], tm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) t7[r] = x3(st[8 * r + 7], st[8 * ((r + 1) & 3) + 7], ck[8 * r + 7]);
#pragma unroll
    for (int r = 0; r < 4; ++r) tj[r] = t7[r];
#pragma unroll
    for (int j = 7; j >= 0; --j) {
        if (j > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) tm[r] = x3(st[8 * r + j - 1], st[8 * ((r + 1) & 3) + j - 1], ck[8 * r + j - 1]);
        }
        uint32_t o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t lo = j == 0 ? t7[r] : tm[r];
            uint32_t v = x3(lo, st[8 * ((r + 1) & 3) + j], tj[(r + 2) & 3]);
            if (j == 1 || j == 3 || j == 4) v ^= t7[r];
            o[r] = v;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) st[8 * r + j] = o[r];
#pragma unroll
        for (int r = 0; r < 4; ++r) tj[r] = tm[r];
    }
}

// AES-128-MMO of the 8 blocks in x under key `key` (0 = L, 1 = R): o = AES(x) ^ x.
// Rounds 1..9 are one loop body (code size ~ one round).
__device__ __forceinline__ void aes_mmo8(const uint32_t (&x)[32], uint32_t (&o)[32], uint32_t key) {
    const uint32_t* rk = &c_rkbs.w[0][0][0] + key * (11 * 32);
    const uint32_t* mk = &c_mcks.w[0][0][0] + key * (11 * 32);
    uint32_t st[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) st[w] = x[w] ^ rk[w];
    sub_bytes(st);
#pragma nounroll
    for (int rnd = 1; rnd < 10; ++rnd) {
        shift_rows(st);
        mix_columns(st, mk + 32 * rnd);   // includes AddRoundKey(rk[rnd])
        sub_bytes(st);
    }
    shift_rows(st);
#pragma unroll
    for (int w = 0; w < 32; ++w) o[w] = x3(st[w], rk[320 + w], x[w]);
}

// In-place 32x32 bit-matrix transpose: m[q] bit b <-> m[b] bit q.
__device__ __forceinline__ void transpose32(uint32_t (&m)[32]) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {                 // s = 16: 16-bit halves
        const uint32_t x = m[k], y = m[k + 16];
        m[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);
        m[k + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {                 // s = 8: bytes
        if (k & 8) continue;
        const uint32_t x = m[k], y = m[k + 8];
        m[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);
        m[k + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);
    }
#define DPF_BS_SWAP(S, MASK)                                                           \
    _Pragma("unroll") for (int k = 0; k < 32; ++k) {                                   \
        if (k & S) continue;                                                           \
        const uint32_t x = m[k], y = m[k + S];                                         \
        m[k] = __builtin_amdgcn_bitop3_b32(x, y << S, MASK, 0xe4); /* MASK ? x : y<<S */ \
        m[k + S] = __builtin_amdgcn_bitop3_b32(x >> S, y, MASK, 0xe4);                 \
    }
    DPF_BS_SWAP(4, 0x0F0F0F0Fu)
    DPF_BS_SWAP(2, 0x33333333u)
    DPF_BS_SWAP(1, 0x55555555u)
#undef DPF_BS_SWAP
}

}  // namespace bs
}  // namespace dpfk
