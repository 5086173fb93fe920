// tree_ops.hpp — device building blocks of the GGM tree walks shared by the
// tree / Eval kernels (dpf_kernels.hip) and the fused PIR kernel
// (pir_kernels.hip): nodes, correction words, the PRG step and the leaf
// conversion.  Reference: dpf/dpf.go:46-69 (getT/clr/prg), :171-241 (Eval,
// evalFullRecursive) and the key layout :89-92,111-112,137-138,165-167.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "aes_ttable.hpp"

#ifndef DPF_MMO_INTERLEAVE
#define DPF_MMO_INTERLEAVE 1
#endif

namespace dpfk {

struct Node {
    Blk s;
    uint32_t t;   // control "bit": a full byte value, tested != 0 (dpf.go:185,218,230)
};

struct CW {
    Blk s;
    uint32_t tl, tr;
};

__device__ __forceinline__ uint32_t tmask(uint32_t t) { return t != 0 ? 0xffffffffu : 0u; }
// Eval's path bit with Go's shift semantics (dpf.go:194: a shift of 64 or
// more gives 0, so logN > 63 keys go left on their top logN-64 levels).
__device__ __forceinline__ uint32_t path_bit(uint64_t x, uint32_t s) { return s < 64 ? (uint32_t)(x >> s) & 1u : 0u; }

// Expanded key record (words): [0..3] root seed, [4] root t, [8+8l..] level l
// {sCW[4], tLCW, tRCW, 0, 0}, [8+8*stop..+3] final CW.
__device__ __forceinline__ CW load_cw(const uint32_t* ek, uint32_t lvl) {
    const uint4* p = reinterpret_cast<const uint4*>(ek + 8 + 8 * lvl);
    uint4 a = p[0];
    uint2 b = *reinterpret_cast<const uint2*>(ek + 8 + 8 * lvl + 4);
    return {{a.x, a.y, a.z, a.w}, b.x, b.y};
}
__device__ __forceinline__ Blk load_blk(const uint32_t* p) {
    uint4 a = *reinterpret_cast<const uint4*>(p);
    return {a.x, a.y, a.z, a.w};
}

// Where a thread's key comes from: its expanded records (k_unpack), or --
// RAW, wave-uniform keys only -- the reference's key bytes themselves
// (dpf.go:89-92,111-112,137-138,165-167), read with scalar loads of the
// aligned words around each field and 64-bit funnel shifts, so a one-shot
// EvalFull needs no unpack launch.  Every load stays inside the dword that
// holds a key byte, so nothing is read past the batch's last dword.
struct KeySrc {
    const uint32_t* ek;    // expanded records of this key
    const uint32_t* kw;    // RAW: the key batch as 4-byte words (4-byte-aligned base)
    uint64_t kb, klen;     // RAW: this key's byte offset in the batch; key length
};
__device__ __forceinline__ uint32_t funnel(uint32_t a, uint32_t b, uint32_t sh) {
    return (uint32_t)((((uint64_t)b << 32) | a) >> sh);
}
template <bool RAW>
__device__ __forceinline__ CW key_cw(const KeySrc& k, uint32_t lvl) {
    if constexpr (!RAW) {
        return load_cw(k.ek, lvl);
    } else {
        const uint64_t o = k.kb + 17 + 18ull * lvl;           // sCW_lvl, tLCW, tRCW (dpf.go:231-233)
        const uint32_t* p = k.kw + (o >> 2);
        const uint32_t sh = (uint32_t)(o & 3) * 8;
        const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
        const uint32_t w5 = sh == 24 ? p[5] : 0u;             // byte o+17 lies in word 5 only then
        const uint32_t t = funnel(w4, w5, sh);
        return {{funnel(w0, w1, sh), funnel(w1, w2, sh), funnel(w2, w3, sh), funnel(w3, w4, sh)}, t & 0xffu,
                (t >> 8) & 0xffu};
    }
}
template <bool RAW>
__device__ __forceinline__ Blk key_root(const KeySrc& k, uint32_t& t) {
    if constexpr (!RAW) {
        t = k.ek[4];
        return load_blk(k.ek);
    } else {                                                   // seed k[0:16], t = k[16] (dpf.go:244-246)
        const uint32_t* p = k.kw + (k.kb >> 2);
        const uint32_t sh = (uint32_t)(k.kb & 3) * 8;
        const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
        t = (w4 >> sh) & 0xffu;
        return {funnel(w0, w1, sh), funnel(w1, w2, sh), funnel(w2, w3, sh), funnel(w3, w4, sh)};
    }
}
template <bool RAW>
__device__ __forceinline__ Blk key_fcw(const KeySrc& k, uint32_t stop) {
    if constexpr (!RAW) {
        return load_blk(k.ek + 8 + 8 * stop);
    } else {                                                   // final CW = k[len-16:] (dpf.go:206,219)
        const uint64_t o = k.kb + k.klen - 16;
        const uint32_t* p = k.kw + (o >> 2);
        const uint32_t sh = (uint32_t)(o & 3) * 8;
        const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3];
        const uint32_t w4 = sh ? p[4] : 0u;
        return {funnel(w0, w1, sh), funnel(w1, w2, sh), funnel(w2, w3, sh), funnel(w3, w4, sh)};
    }
}

// prg (dpf.go:59-69) plus the parent's CW correction (dpf.go:230-238).
// The two independent MMOs of a PRG call (or of a leaf pair), written as two
// plain mmo1 calls so the scheduler interleaves them freely: 98.9 G blocks/s
// in tools/aes_variants.hip, against 88.4 for a round-by-round interleave
// and 93.3 fully serialized (r01 A/B, profiles/r01/full_ilp*).  An explicit
// software pipeline (each block's 16 lookups issued while the other block's
// are in flight, up to 32 per wave) was slower again: 93.1 vs 93.8 in-tree,
// 21 VGPRs spilled (profiles/r02/pipe).
template <bool B = false, class KA, class KB>
__device__ __forceinline__ void mmo_pair(const uint8_t* tab, uint32_t lo, const KA& ka, Blk xa, Blk& oa,
                                         const KB& kb, Blk xb, Blk& ob) {
#if DPF_MMO_INTERLEAVE
    mmo2<B>(tab, lo, ka, xa, oa, kb, xb, ob);
#else
    oa = mmo1(tab, lo, ka, xa);
    ob = mmo1(tab, lo, kb, xb);
#endif
}

template <bool B = false>
__device__ __forceinline__ void expand(const uint8_t* tab, uint32_t lo, const Node& n, const CW& cw, Node& L,
                                       Node& R) {
    mmo_pair<B>(tab, lo, KeyFixed<false>{}, n.s, L.s, KeyFixed<true>{}, n.s, R.s);
    uint32_t tL = L.s.c0 & 1u, tR = R.s.c0 & 1u;
    L.s.c0 &= ~1u;
    R.s.c0 &= ~1u;
    uint32_t m = tmask(n.t);
    L.s.c0 ^= m & cw.s.c0; L.s.c1 ^= m & cw.s.c1; L.s.c2 ^= m & cw.s.c2; L.s.c3 ^= m & cw.s.c3;
    R.s.c0 ^= m & cw.s.c0; R.s.c1 ^= m & cw.s.c1; R.s.c2 ^= m & cw.s.c2; R.s.c3 ^= m & cw.s.c3;
    L.t = tL ^ (m & cw.tl);
    R.t = tR ^ (m & cw.tr);
}

// One step of a root-to-node walk that computes only the child selected by
// `bit` (dpf.go:183-201, minus the unused sibling).
__device__ __forceinline__ void walk_fix(Node& n, Blk c, const CW& cw, uint32_t bit) {
    uint32_t tc = c.c0 & 1u;
    c.c0 &= ~1u;
    uint32_t m = tmask(n.t);
    c.c0 ^= m & cw.s.c0; c.c1 ^= m & cw.s.c1; c.c2 ^= m & cw.s.c2; c.c3 ^= m & cw.s.c3;
    n.s = c;
    n.t = tc ^ (m & (bit ? cw.tr : cw.tl));
}
template <bool B = false>
__device__ __forceinline__ void walk_step(const uint8_t* tab, uint32_t lo, Node& n, const CW& cw, uint32_t bit) {
    walk_fix(n, mmo1<B>(tab, lo, KeySel{bit ? 0xffffffffu : 0u}, n.s), cw, bit);
}
// Two independent walks advanced together (two queries per thread).
template <bool B = false>
__device__ __forceinline__ void walk_step2(const uint8_t* tab, uint32_t lo, Node& n0, const CW& cw0, uint32_t bit0,
                                           Node& n1, const CW& cw1, uint32_t bit1) {
    Blk c0, c1;
#if DPF_EXP_NOSEL
    // Measurement only (wrong answers): the walk with a wave-uniform key, to
    // bound what the per-lane key select costs.
    mmo2<B>(tab, lo, KeyFixed<false>{}, n0.s, c0, KeyFixed<false>{}, n1.s, c1);
#else
    mmo2<B>(tab, lo, KeySel{bit0 ? 0xffffffffu : 0u}, n0.s, c0, KeySel{bit1 ? 0xffffffffu : 0u}, n1.s, c1);
#endif
    walk_fix(n0, c0, cw0, bit0);
    walk_fix(n1, c1, cw1, bit1);
}

// walk_step in the quad latency form (aes_ttable.hpp mmo_quad): lane j of the
// quad holds column j of the node's seed in `col`, and the t byte in `t`
// (the same on the quad's 4 lanes).  cwj = column j of the level's sCW.
__device__ __forceinline__ void walk_step_quad(const uint8_t* tab, uint32_t lo, const QuadKeys& k, uint32_t j,
                                               uint32_t& col, uint32_t& t, uint32_t cwj, uint32_t tl_, uint32_t tr_,
                                               uint32_t bit) {
    uint32_t c = mmo_quad(tab, lo, k, bit ? 0xffffffffu : 0u, col);
    const uint32_t tc = quad_mov<0x00>(c) & 1u;          // getT of column 0 (dpf.go:46-48), on every lane
    if (j == 0) c &= ~1u;                                // clr (dpf.go:50-52)
    const uint32_t m = tmask(t);
    col = c ^ (m & cwj);                                  // dpf.go:185-193
    t = tc ^ (m & (bit ? tr_ : tl_));
}

__device__ __forceinline__ void store16(uint8_t* p, Blk v) {
    *reinterpret_cast<uint4*>(p) = make_uint4(v.c0, v.c1, v.c2, v.c3);
}

// Leaf conversion (dpf.go:214-224): MMO_L(s) ^ (t != 0 ? finalCW : 0).
__device__ __forceinline__ Blk leaf_fix(Blk o, uint32_t t, Blk fcw) {
    uint32_t m = tmask(t);
    return {o.c0 ^ (m & fcw.c0), o.c1 ^ (m & fcw.c1), o.c2 ^ (m & fcw.c2), o.c3 ^ (m & fcw.c3)};
}

}  // namespace dpfk
