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
//   MixColumns = XORs between rows (xtime is a renaming of planes);
//   AddRoundKey= XOR with 32 per-round constant words (scalar operands).
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
__device__ __forceinline__ void mix_columns(uint32_t (&st)[32]) {
    uint32_t t7[4], tj[4], tm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) t7[r] = st[8 * r + 7] ^ st[8 * ((r + 1) & 3) + 7];
#pragma unroll
    for (int r = 0; r < 4; ++r) tj[r] = t7[r];
#pragma unroll
    for (int j = 7; j >= 0; --j) {
        if (j > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) tm[r] = st[8 * r + j - 1] ^ st[8 * ((r + 1) & 3) + j - 1];
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
    uint32_t st[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) st[w] = x[w] ^ rk[w];
    sub_bytes(st);
#pragma nounroll
    for (int rnd = 1; rnd < 10; ++rnd) {
        shift_rows(st);
        mix_columns(st);
        const uint32_t* k = rk + 32 * rnd;
#pragma unroll
        for (int w = 0; w < 32; ++w) st[w] ^= k[w];
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
