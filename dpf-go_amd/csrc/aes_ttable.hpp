// aes_ttable.hpp — AES-128-MMO on gfx950 with LDS T-tables (device code).
//
// Implements aes128MMO (dpf/aes_amd64.s:51-82): dst = AES_k(src) ^ src for
// the two fixed PRG keys (dpf/dpf.go:23-24).
//
// PRG back end ("T-table"): AES-128 as four lookups per column into Te0 held
// in LDS.  Row e (256 B) holds 32 lane copies of Te0[e] followed by 32 copies
// of rotl8(Te0[e]); lane l reads copy (l mod 32) at byte e*256 + 4*(l mod 32)
// (+128 for the rotated word).  ds_read_b32 serves each 32-lane half in one
// pass over banks (a/4) mod 32, so every lookup is conflict-free whatever the
// indices.  The LDS address of byte k of a column is one v_perm_b32
// {0, 0, x.byte_k, lane offset}.  With the rotated copy a column needs one
// rotation instead of three:
//   out = Ta ^ R8Tb ^ R16(Tc ^ R8Td) ^ rk.
// v_perm / v_alignbit issue at ~0.6x the rate of v_xor / v_bitop3 on gfx950
// (tools/valu_peak.hip), so rotations and address math dominate the VALU
// budget.  Round keys are compile-time literals: the two PRG keys are fixed
// (dpf/dpf.go:23-24).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "aes_consts.hpp"

namespace dpfk {

// LDS footprint of one table: 256 rows x 256 B.
constexpr uint32_t kTabWords = 256 * 64;

// Te0, the source of the LDS table (one copy per code object).
static __constant__ dpfc::Words256 c_te0 = dpfc::kTe0;

struct Blk {
    uint32_t c0, c1, c2, c3;
};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
constexpr uint32_t crotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// v_bitop3_b32 truth tables (src0 = 0xF0, src1 = 0xCC, src2 = 0xAA).
constexpr uint32_t kXor3 = 0x96;     // a ^ b ^ c
constexpr uint32_t kOrXor = 0x56;    // (a | b) ^ c
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, kXor3);
}

// LDS address of the Te0 pair for byte K of x in this lane's copy.
template <int K>
__device__ __forceinline__ uint32_t taddr(uint32_t x, uint32_t laneoff) {
    // v_perm_b32 selector: result byte0 = src1.byte0 (lane offset), byte1 =
    // src0.byte K, bytes 2-3 = 0x00 (selector 0x0c).
    return __builtin_amdgcn_perm(x, laneoff, 0x0c0c0000u | ((4u + K) << 8));
}

// Te0[x.byte K] (ROT = false) or rotl8(Te0[x.byte K]) (ROT = true).
template <int K, bool ROT = false>
__device__ __forceinline__ uint32_t tl(const uint8_t* tab, uint32_t x, uint32_t laneoff) {
    return *reinterpret_cast<const uint32_t*>(tab + taddr<K>(x, laneoff) + (ROT ? 128 : 0));
}

// Round-key sources.  KeyFixed<R>: the fixed left/right PRG key (literal).
// KeySel: per-lane choice, rk = rkL ^ (m & (rkL ^ rkR)), m = 0 or ~0.
// get16<I>() = rotl(rk_I, 16), folded into the pre-rotation XOR of a column.
template <bool RIGHT>
struct KeyFixed {
    template <int I>
    __device__ __forceinline__ uint32_t get() const {
        return RIGHT ? dpfc::kRkR.w[I] : dpfc::kRkL.w[I];
    }
    template <int I>
    __device__ __forceinline__ uint32_t get16() const {
        constexpr uint32_t v = crotl(RIGHT ? dpfc::kRkR.w[I] : dpfc::kRkL.w[I], 16);
        return v;
    }
};
struct KeySel {
    uint32_t m;
    template <int I>
    __device__ __forceinline__ uint32_t get() const {
        constexpr uint32_t l = dpfc::kRkL.w[I];
        constexpr uint32_t d = dpfc::kRkL.w[I] ^ dpfc::kRkR.w[I];
        return l ^ (m & d);
    }
    template <int I>
    __device__ __forceinline__ uint32_t get16() const {
        constexpr uint32_t l = crotl(dpfc::kRkL.w[I], 16);
        constexpr uint32_t d = crotl(dpfc::kRkL.w[I] ^ dpfc::kRkR.w[I], 16);
        return l ^ (m & d);
    }
};

template <int R, class K>
__device__ __forceinline__ void aes_round(const uint8_t* tab, uint32_t lo, const K& k, Blk& s) {
    // column j: Te0[s_j.b0] ^ Te1[s_{j+1}.b1] ^ Te2[s_{j+2}.b2] ^ Te3[s_{j+3}.b3] ^ rk_j, Te_i = rotl(Te0, 8i)
    // = Ta ^ R8Tb ^ R16(Tc ^ R8Td ^ R16 rk): two v_bitop3 + one v_alignbit.
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk16) {
        uint32_t ta = tl<0>(tab, a, lo), tb = tl<1, true>(tab, b, lo), tc = tl<2>(tab, c, lo),
                 td = tl<3, true>(tab, d, lo);
        return xor3(ta, tb, rotl(xor3(tc, td, rk16), 16));
    };
    uint32_t n0 = col(s.c0, s.c1, s.c2, s.c3, k.template get16<4 * R + 0>());
    uint32_t n1 = col(s.c1, s.c2, s.c3, s.c0, k.template get16<4 * R + 1>());
    uint32_t n2 = col(s.c2, s.c3, s.c0, s.c1, k.template get16<4 * R + 2>());
    uint32_t n3 = col(s.c3, s.c0, s.c1, s.c2, k.template get16<4 * R + 3>());
    s.c0 = n0; s.c1 = n1; s.c2 = n2; s.c3 = n3;
}

// Final round: SubBytes via byte 1 of Te0 (= S[x]), ShiftRows, AddRoundKey.
template <class K>
__device__ __forceinline__ void aes_last(const uint8_t* tab, uint32_t lo, const K& k, Blk& s) {
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
        uint32_t la = tl<0>(tab, a, lo), lb = tl<1>(tab, b, lo), lc = tl<2>(tab, c, lo), ld = tl<3>(tab, d, lo);
        uint32_t p = __builtin_amdgcn_perm(lb, la, 0x0c0c0501u);   // {la.b1, lb.b1, 0, 0}
        uint32_t q = __builtin_amdgcn_perm(ld, lc, 0x05010c0cu);   // {0, 0, lc.b1, ld.b1}
        return __builtin_amdgcn_bitop3_b32(p, q, rk, kOrXor);
    };
    uint32_t n0 = col(s.c0, s.c1, s.c2, s.c3, k.template get<40>());
    uint32_t n1 = col(s.c1, s.c2, s.c3, s.c0, k.template get<41>());
    uint32_t n2 = col(s.c2, s.c3, s.c0, s.c1, k.template get<42>());
    uint32_t n3 = col(s.c3, s.c0, s.c1, s.c2, k.template get<43>());
    s.c0 = n0; s.c1 = n1; s.c2 = n2; s.c3 = n3;
}

// A round as two phases: the 16 lookups of a block issued together, then
// its 4 columns.  aes2_rounds<BATCH = true> issues both blocks' 32 lookups
// before any XOR, with scheduling fences between the phases, so a wave keeps
// up to 32 LDS reads in flight; left alone the compiler consumes them in
// groups of 4-8 (r03: 95.7-96.1 vs 93.1-93.4 G blocks/s in the configs[1]
// tree kernel).  Needs ~16 more VGPRs: the tree kernels use it where they
// fit (one key per wave) and the interleaved form elsewhere.
template <int C0 = 0, int C1 = 4>
__device__ __forceinline__ void round_loads(const uint8_t* tab, uint32_t lo, const Blk& s, uint32_t (&t)[16]) {
    const uint32_t c[4] = {s.c0, s.c1, s.c2, s.c3};
#pragma unroll
    for (int j = C0; j < C1; ++j) {
        t[4 * j + 0] = tl<0>(tab, c[j], lo);
        t[4 * j + 1] = tl<1, true>(tab, c[(j + 1) & 3], lo);
        t[4 * j + 2] = tl<2>(tab, c[(j + 2) & 3], lo);
        t[4 * j + 3] = tl<3, true>(tab, c[(j + 3) & 3], lo);
    }
}
template <int R, class K>
__device__ __forceinline__ void round_mix(const K& k, const uint32_t (&t)[16], Blk& s) {
    auto col = [&](int j, uint32_t rk16) {
        return xor3(t[4 * j], t[4 * j + 1], rotl(xor3(t[4 * j + 2], t[4 * j + 3], rk16), 16));
    };
    s.c0 = col(0, k.template get16<4 * R + 0>());
    s.c1 = col(1, k.template get16<4 * R + 1>());
    s.c2 = col(2, k.template get16<4 * R + 2>());
    s.c3 = col(3, k.template get16<4 * R + 3>());
}

template <int R, bool BATCH = false, class K>
__device__ __forceinline__ void aes_rounds(const uint8_t* tab, uint32_t lo, const K& k, Blk& s) {
    if constexpr (R <= 9) {
        if constexpr (BATCH) {
            uint32_t t[16];
            round_loads(tab, lo, s, t);
            __builtin_amdgcn_sched_barrier(0);
            round_mix<R>(k, t, s);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            aes_round<R>(tab, lo, k, s);
        }
        aes_rounds<R + 1, BATCH>(tab, lo, k, s);
    }
}

// Two independent AES-MMO blocks, rounds interleaved for ILP.
template <int R, bool BATCH, class KA, class KB>
__device__ __forceinline__ void aes2_rounds(const uint8_t* tab, uint32_t lo, const KA& ka, Blk& a, const KB& kb,
                                            Blk& b) {
    if constexpr (R <= 9) {
        if constexpr (BATCH) {
            uint32_t ta[16], tb[16];
            round_loads(tab, lo, a, ta);
            round_loads(tab, lo, b, tb);
            __builtin_amdgcn_sched_barrier(0);
            round_mix<R>(ka, ta, a);
            round_mix<R>(kb, tb, b);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            aes_round<R>(tab, lo, ka, a);
            aes_round<R>(tab, lo, kb, b);
        }
        aes2_rounds<R + 1, BATCH>(tab, lo, ka, a, kb, b);
    }
}

__device__ __forceinline__ Blk bxor(Blk a, Blk b) { return {a.c0 ^ b.c0, a.c1 ^ b.c1, a.c2 ^ b.c2, a.c3 ^ b.c3}; }
__device__ __forceinline__ Blk bkey4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return {a, b, c, d}; }

// aes128MMO (aes_amd64.s:51-82): AES_k(x) ^ x.
template <bool BATCH = false, class K>
__device__ __forceinline__ Blk mmo1(const uint8_t* tab, uint32_t lo, const K& k, Blk x) {
    Blk s = bxor(x, bkey4(k.template get<0>(), k.template get<1>(), k.template get<2>(), k.template get<3>()));
    aes_rounds<1, BATCH>(tab, lo, k, s);
    aes_last(tab, lo, k, s);
    return bxor(s, x);
}

template <bool BATCH = false, class KA, class KB>
__device__ __forceinline__ void mmo2(const uint8_t* tab, uint32_t lo, const KA& ka, Blk xa, Blk& oa, const KB& kb,
                                     Blk xb, Blk& ob) {
    Blk a = bxor(xa, bkey4(ka.template get<0>(), ka.template get<1>(), ka.template get<2>(), ka.template get<3>()));
    Blk b = bxor(xb, bkey4(kb.template get<0>(), kb.template get<1>(), kb.template get<2>(), kb.template get<3>()));
    aes2_rounds<1, BATCH>(tab, lo, ka, a, kb, b);
    aes_last(tab, lo, ka, a);
    aes_last(tab, lo, kb, b);
    oa = bxor(a, xa);
    ob = bxor(b, xb);
}

// ---- Latency form: one block per quad of lanes (r05) --------------------
// The serial root-to-subtree walks of small launches run one dependent
// AES-MMO per level on a nearly idle CU (profiles/r05/wave_times: the walk
// was half of a 51 us PIR-rank launch at N = 8), so their time is the
// latency of a round, not the LDS rate.  Here lane j = lane & 3 of a quad
// holds column j of the state: a round is 3 DPP quad permutes (columns j+1,
// j+2, j+3), 4 lookups and 3 XOR ops per lane instead of 16 lookups and
// their address math on one lane.  Round keys are per lane (column j), for
// the left key and the left^right difference, so a per-quad key select is
// one v_bitop3 per round.
struct QuadKeys {
    uint32_t l[11], d[11];   // rk_L[r][j], (rk_L ^ rk_R)[r][j]; rounds 1..9 pre-rotated by 16
};
__device__ __forceinline__ QuadKeys quad_keys(uint32_t j) {
    QuadKeys k;
#pragma unroll
    for (int r = 0; r < 11; ++r) {
        const uint32_t l0 = dpfc::kRkL.w[4 * r], l1 = dpfc::kRkL.w[4 * r + 1], l2 = dpfc::kRkL.w[4 * r + 2],
                       l3 = dpfc::kRkL.w[4 * r + 3];
        const uint32_t d0 = l0 ^ dpfc::kRkR.w[4 * r], d1 = l1 ^ dpfc::kRkR.w[4 * r + 1],
                       d2 = l2 ^ dpfc::kRkR.w[4 * r + 2], d3 = l3 ^ dpfc::kRkR.w[4 * r + 3];
        uint32_t l = j == 0 ? l0 : j == 1 ? l1 : j == 2 ? l2 : l3;
        uint32_t d = j == 0 ? d0 : j == 1 ? d1 : j == 2 ? d2 : d3;
        if (r >= 1 && r <= 9) {
            l = rotl(l, 16);
            d = rotl(d, 16);
        }
        k.l[r] = l;
        k.d[r] = d;
    }
    return k;
}
template <int CTRL>
__device__ __forceinline__ uint32_t quad_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// aes128MMO (aes_amd64.s:51-82) of the quad's block under rk_L ^ (m & d):
// m = 0 (left key) or ~0 (right key), uniform over the quad.  x = this
// lane's column of the input; returns its column of the output.
__device__ __forceinline__ uint32_t mmo_quad(const uint8_t* tab, uint32_t lo, const QuadKeys& k, uint32_t m,
                                             uint32_t x) {
    uint32_t s = x ^ k.l[0] ^ (m & k.d[0]);
#pragma unroll
    for (int r = 1; r <= 9; ++r) {
        const uint32_t b = quad_mov<0x39>(s), c = quad_mov<0x4E>(s), d = quad_mov<0x93>(s);   // columns j+1, j+2, j+3
        const uint32_t ta = tl<0>(tab, s, lo), tb = tl<1, true>(tab, b, lo), tc = tl<2>(tab, c, lo),
                       td = tl<3, true>(tab, d, lo);
        const uint32_t rk16 = k.l[r] ^ (m & k.d[r]);
        s = xor3(ta, tb, rotl(xor3(tc, td, rk16), 16));
    }
    const uint32_t b = quad_mov<0x39>(s), c = quad_mov<0x4E>(s), d = quad_mov<0x93>(s);
    const uint32_t la = tl<0>(tab, s, lo), lb = tl<1>(tab, b, lo), lc = tl<2>(tab, c, lo), ld = tl<3>(tab, d, lo);
    const uint32_t p = __builtin_amdgcn_perm(lb, la, 0x0c0c0501u);   // {la.b1, lb.b1, 0, 0}
    const uint32_t q = __builtin_amdgcn_perm(ld, lc, 0x05010c0cu);   // {0, 0, lc.b1, ld.b1}
    s = __builtin_amdgcn_bitop3_b32(p, q, k.l[10] ^ (m & k.d[10]), kOrXor);
    return s ^ x;
}

// Without the closing barrier: the caller adds its own LDS writes first.
__device__ __forceinline__ void fill_table_nobar(uint32_t* tab) {
    // Row e: 32 copies of Te0[e], then 32 copies of rotl8(Te0[e]); 16-byte stores.
    for (uint32_t i = threadIdx.x; i < 256 * 16; i += blockDim.x) {
        uint32_t e = i >> 4, q = i & 15;
        uint32_t v = c_te0.v[e];
        if (q >= 8) v = rotl(v, 8);
        reinterpret_cast<uint4*>(tab)[e * 16 + q] = make_uint4(v, v, v, v);
    }
}
__device__ __forceinline__ void fill_table(uint32_t* tab) {
    fill_table_nobar(tab);
    __syncthreads();
}

}  // namespace dpfk
