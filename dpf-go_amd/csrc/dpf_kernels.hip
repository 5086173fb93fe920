// dpf_kernels.hip — gfx950 kernels for DPF evaluation (EvalFull / Eval).
//
// Reference semantics: dpf/dpf.go:171-262 (Eval, evalFullRecursive, EvalFull)
// and the PRG dpf/dpf.go:59-69 over aes128MMO (dpf/aes_amd64.s:51-82); the
// AES back end is aes_ttable.hpp.
//
// Tree: a thread owns a subtree of 2^D leaves (D <= 7).  It walks from the
// root to its subtree root computing only the child on its path (one AES per
// level), then expands the subtree depth-first with the right siblings kept
// in registers (one statically-allocated slot per level), writing leaves in
// ascending order exactly like evalFullRecursive's cursor (dpf.go:213-241).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <mutex>
#include "aes_consts.hpp"
#include "aes_ttable.hpp"
#include "dpf_kernels.hpp"
#include "wave_prio.hpp"
#include "tree_ops.hpp"

#ifndef DPF_COOP_WALK
#define DPF_COOP_WALK 1
#endif
#ifndef DPF_QUAD_WALK
#define DPF_QUAD_WALK 1  // shared walk: one block per quad of lanes on 4 waves (latency form, mmo_quad)
#endif
#ifndef DPF_QUAD_FAN
#define DPF_QUAD_FAN 6   // log2 of the shared walk's paths in the quad form: 6 (4 waves) or 7 (8 waves)
#endif
#ifndef DPF_COOP_BFS
#define DPF_COOP_BFS 0   // 1: the last W - 6 levels of the shared walk breadth-first in LDS (measured slower, r05)
#endif
#ifndef DPF_PAIR_STORES
#define DPF_PAIR_STORES 1
#endif
#ifndef DPF_EVAL_STRIDE
#define DPF_EVAL_STRIDE 0   // 1: k_eval2 grid = resident workgroups only (slower: 3667 vs 3489 us)
#endif
#ifndef DPF_EVAL_PAIRS
#define DPF_EVAL_PAIRS 1   // batched Eval: two queries per thread (k_eval2)
#endif
#ifndef DPF_EVAL_BATCH
#define DPF_EVAL_BATCH 1
#endif
#ifndef DPF_PRIO_STEPS
#define DPF_PRIO_STEPS 3   // wave issue priority lowered by progress (prio_step)
#endif
#ifndef DPF_DEPTH_MODEL_COOP
#define DPF_DEPTH_MODEL_COOP 1   // pick_shape prices the shared walk (latency once + W - 6 per thread)
#endif
#ifndef DPF_WALK_BATCH
#define DPF_WALK_BATCH 1   // tree kernels' root-to-subtree walks: batched single-block rounds
#endif
#ifndef DPF_WALK_CW_LDS
#define DPF_WALK_CW_LDS 1  // walks of a one-key workgroup read their correction words from LDS (staged once)
#endif
#ifndef DPF_DFS_CW_LDS
#define DPF_DFS_CW_LDS 0   // ... and so does the subtree expansion below them (A/B)
#endif

namespace dpfk {

#ifdef DPF_WAVE_TIMES
constexpr uint64_t kWaveTimesMax = 1u << 16;
__device__ uint64_t g_wave_times[5 * kWaveTimesMax];   // start, end, HW_ID, XCC_ID, walk end
#endif

struct Ctx {
    const uint8_t* tab;
    uint32_t lo;
    KeySrc ks;
    Blk fcw;
    uint8_t* outp;      // leaf mode: 16-byte leaf cursor
    uint4* nseed;       // node mode: seed cursor
    uint8_t* nt;        // node mode: t cursor
    uint32_t groups;    // 4-leaf groups finished (wave priority steps, prio_step)
    const uint32_t* cwl;   // the key's CWs staged in LDS (8 words per level), or nullptr
    bool sync = false;     // workgroup-uniform: every thread runs the same DFS (DPF_TREE_SYNC barriers)
    uint32_t* prog = nullptr;   // DPF_PRIO_FEEDBACK: this SIMD's 16 wave-progress slots in LDS
    uint32_t pslot = 0;         // ... and this wave's slot (hardware wave id)
};

// Level lvl's correction word for the expansion: from the LDS copy when the
// workgroup staged one (DPF_DFS_CW_LDS), else from the key.
template <bool RAW>
__device__ __forceinline__ CW ctx_cw(const Ctx& c, uint32_t lvl) {
#if DPF_DFS_CW_LDS
    if (c.cwl != nullptr) {
        const uint4 a = *reinterpret_cast<const uint4*>(c.cwl + 8 * lvl);
        const uint2 b = *reinterpret_cast<const uint2*>(c.cwl + 8 * lvl + 4);
        return CW{{a.x, a.y, a.z, a.w}, b.x, b.y};
    }
#endif
    return key_cw<RAW>(c.ks, lvl);
}

// Issue priority by progress.  A SIMD's waves issue oldest-first, so of the
// 4 waves sharing one, the oldest finishes its subtree first and the
// youngest runs alone at the end, when the CU's LDS idles (per-wave wall
// clock, tools/wave_times.hip, configs[1]: the 4 slots of every SIMD end at
// 455 / 635 / 825 / 1015 us; waves busy 71% of the kernel's span).  Waves
// lower their priority as they pass progress thresholds (fractions of the
// thread's 4-leaf groups), so waves that are ahead yield the issue slots to
// the ones behind and a SIMD's waves finish close together (busy 95%;
// kernel 1048 -> 948 us on one box, profiles/r03/prio/).
//   DPF_PRIO_STEPS 3: thresholds 3/4, 7/8, 15/16 (default);
//   2: 1/2, 3/4, 7/8;  1: 1/4, 1/2, 3/4;  5: 7/8, 15/16, 31/32;  0: off.
//   Subtrees of <= 2^5 leaf blocks (8 or fewer groups: the PIR tree, strong-
//   scaling ranks) step at 1/2, 3/4, 7/8 (DPF_PRIO_STEPS_SMALL 2): at the
//   PIR shape waves are busy 0.945-0.949 of the span instead of 0.914-0.922
//   and the span is 244 vs 250-256 us (profiles/r04/prio/).
#ifndef DPF_TREE_SYNC
#define DPF_TREE_SYNC 0
#endif
#ifndef DPF_PRIO_FEEDBACK
#define DPF_PRIO_FEEDBACK 3   // priority from the wave's lead over the slowest wave of its SIMD; 0: static steps
#endif
#ifndef DPF_PRIO_STEPS_SMALL
#define DPF_PRIO_STEPS_SMALL 2
#endif
template <int DMAX>
__device__ __forceinline__ void prio_step(Ctx& c) {
#if DPF_PRIO_FEEDBACK
    // Feedback form (progress = finished 4-leaf groups).
    if (c.prog != nullptr) {
        prio_by_lead(c.prog, c.pslot, ++c.groups, 1, DPF_PRIO_FEEDBACK);
        return;
    }
#endif
#if DPF_PRIO_STEPS
    constexpr int S = DMAX <= 5 ? DPF_PRIO_STEPS_SMALL : DPF_PRIO_STEPS;
    constexpr uint32_t total = DMAX >= 2 ? 1u << (DMAX - 2) : 1u;   // 4-leaf groups per thread
    const uint32_t d = ++c.groups;
    constexpr uint32_t den = S == 1 ? 4 : S == 2 ? 8 : S == 5 ? 32 : 16;
    constexpr uint32_t t1 = S == 1 ? 1 : S == 2 ? 4 : S == 5 ? 28 : 12;
    constexpr uint32_t t2 = S == 1 ? 2 : S == 2 ? 6 : S == 5 ? 30 : 14;
    constexpr uint32_t t3 = S == 1 ? 3 : S == 2 ? 7 : S == 5 ? 31 : 15;
    const uint32_t x = d * den;
    if (x >= t3 * total) __builtin_amdgcn_s_setprio(0);
    else if (x >= t2 * total) __builtin_amdgcn_s_setprio(1);
    else if (x >= t1 * total) __builtin_amdgcn_s_setprio(2);
#else
    (void)c;
#endif
#if DPF_TREE_SYNC
    // Measurement: a workgroup barrier every DPF_TREE_SYNC groups keeps the
    // workgroup's waves within one period of each other.
    if (c.sync && (c.groups % DPF_TREE_SYNC) == 0) __syncthreads();
#endif
}

__device__ __forceinline__ void emit_node(Ctx& c, const Node& n) {
    *c.nseed++ = make_uint4(n.s.c0, n.s.c1, n.s.c2, n.s.c3);
    *c.nt++ = (uint8_t)n.t;
}

// Exchange a value with the other lane of the pair (lane ^ 1): DPP
// quad_perm [1,0,3,2], VALU only (no LDS traffic; the T-table owns the LDS).
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ Node pair_swap(const Node& n) {
    return {{pair_swap(n.s.c0), pair_swap(n.s.c1), pair_swap(n.s.c2), pair_swap(n.s.c3)}, pair_swap(n.t)};
}
__device__ __forceinline__ Node sel(bool b, const Node& x, const Node& y) {
    return {{b ? x.s.c0 : y.s.c0, b ? x.s.c1 : y.s.c1, b ? x.s.c2 : y.s.c2, b ? x.s.c3 : y.s.c3}, b ? x.t : y.t};
}

__device__ __forceinline__ Blk bsel(bool b, const Blk& x, const Blk& y) {
    return {b ? x.c0 : y.c0, b ? x.c1 : y.c1, b ? x.c2 : y.c2, b ? x.c3 : y.c3};
}

// Bottom two levels below node n: 4 leaves = 64 contiguous bytes at p
// (dpf.go:214-224 for each), stored back to back once all four are done.
// The two children are finished by one loop body (expand + leaf pair), not
// two inlined copies: the tree kernel's innermost loop must fit the
// instruction cache (64 KiB per two CUs).  Fully inlined, the PAIR path's
// loop body was ~85 KiB of code (22 AES-MMO bodies).
template <bool B, bool RAW>
__device__ __forceinline__ void leaves4(const Ctx& c, uint32_t lvl, const Node& n, uint8_t* p) {
    CW cw = ctx_cw<RAW>(c, lvl);
    Node L, R;
    expand<B>(c.tab, c.lo, n, cw, L, R);
    CW cw1 = ctx_cw<RAW>(c, lvl + 1);
    Blk o0 = {}, o1 = {}, o2, o3;
    // Only the pending child stays live through the first iteration (a
    // select of L or R at the top of each iteration kept both live: 5 more
    // VGPRs at every level of the expansion).
    Node m = L;
    const Node pend = R;
#pragma nounroll
    for (int h = 0; h < 2; ++h) {
        Node a, b;
        expand<B>(c.tab, c.lo, m, cw1, a, b);
        Blk oa, ob;
        mmo_pair<B>(c.tab, c.lo, KeyFixed<false>{}, a.s, oa, KeyFixed<false>{}, b.s, ob);
        oa = leaf_fix(oa, a.t, c.fcw);
        ob = leaf_fix(ob, b.t, c.fcw);
        o2 = oa;
        o3 = ob;
        if (h == 0) {
            o0 = oa;
            o1 = ob;
        }
        m = pend;
    }
    store16(p, o0);
    store16(p + 16, o1);
    store16(p + 32, o2);
    store16(p + 48, o3);
}

// Depth-first expansion of D more levels below node n at tree level `lvl0 +
// (DMAX - D)`; the right child of every internal node stays live in
// registers while the left subtree is expanded.  Leaf mode writes the
// converted leaves (dpf.go:214-224); node mode (NODES) writes the 2^D nodes
// D levels down instead: the frontier a batched Eval continues from.
// B: batched AES rounds (aes_ttable.hpp aes2_rounds) where the registers
// allow it: the one-key-per-wave kernels.
template <int DMAX, int D, bool NODES, bool PAIR, bool B, bool RAW = false>
__device__ __forceinline__ void dfs(Ctx& c, uint32_t lvl0, const Node& n) {
    if constexpr (PAIR && D == 3) {
        // Lane pairs write whole 128-B lines.  Lanes 2i and 2i+1 own adjacent
        // subtrees a and b of one key (same CWs), 16 << DMAX bytes apart, and
        // reach their depth-3 nodes Na, Nb in lockstep.  After expanding, the
        // even lane trades R(Na) for the odd lane's L(Nb): first the pair
        // computes Na's 8 leaves (even: 0-3, odd: 4-7) and stores the line in
        // one instruction, then Nb's.  Storing a line as two 64-B halves 8 AES
        // apart left ~4 MiB of half-written lines per XCD (its whole L2) and
        // made WRITE_SIZE 1.26x the output.  Leaves are unchanged, only which
        // lane computes them.
        CW cw = ctx_cw<RAW>(c, lvl0 + DMAX - 3);
        Node L, R;
        expand<B>(c.tab, c.lo, n, cw, L, R);
        const bool odd = (threadIdx.x & 1u) != 0;
        const Node got = pair_swap(sel(odd, L, R));   // even gets L(Nb), odd gets R(Na)
        const int64_t sub = 16ll << DMAX;
        Node cur = sel(odd, got, L);
        const Node second = sel(odd, R, got);
#pragma nounroll
        for (int h = 0; h < 2; ++h) {   // one code copy of leaves4 (instruction cache)
            leaves4<B, RAW>(c, lvl0 + DMAX - 2, cur, c.outp + (h == 0 ? (odd ? 64 - sub : 0) : (odd ? 64 : sub)));
            prio_step<DMAX>(c);
            cur = second;
        }
        c.outp += 128;
    } else if constexpr (D == 0) {
        if constexpr (NODES) {
            emit_node(c, n);
        } else {
            Blk o = mmo1(c.tab, c.lo, KeyFixed<false>{}, n.s);
            store16(c.outp, leaf_fix(o, n.t, c.fcw));
            c.outp += 16;
        }
    } else if constexpr (D == 2 && !NODES) {
        // Bottom two levels at once: 4 leaves = 64 contiguous bytes stored back
        // to back (subtrees too shallow or lanes of different keys for PAIR).
        leaves4<B, RAW>(c, lvl0 + DMAX - 2, n, c.outp);
        prio_step<DMAX>(c);
        c.outp += 64;
    } else if constexpr (D == 2 && NODES) {
        // Bottom two levels of a frontier at once: 4 seeds = 64 contiguous
        // bytes and their 4 t bytes as one 32-bit store (one byte store per
        // node made the NODES pass write 2.2x its 17 B per node).
        CW cw = ctx_cw<RAW>(c, lvl0 + DMAX - 2);
        Node L, R;
        expand<B>(c.tab, c.lo, n, cw, L, R);
        CW cw1 = ctx_cw<RAW>(c, lvl0 + DMAX - 1);
        Node q[4];
        expand<B>(c.tab, c.lo, L, cw1, q[0], q[1]);
        expand<B>(c.tab, c.lo, R, cw1, q[2], q[3]);
#pragma unroll
        for (int i = 0; i < 4; ++i) c.nseed[i] = make_uint4(q[i].s.c0, q[i].s.c1, q[i].s.c2, q[i].s.c3);
        *reinterpret_cast<uint32_t*>(c.nt) = (q[0].t & 0xffu) | ((q[1].t & 0xffu) << 8) | ((q[2].t & 0xffu) << 16) |
                                             ((q[3].t & 0xffu) << 24);
        c.nseed += 4;
        c.nt += 4;
        prio_step<DMAX>(c);
    } else if constexpr (D == 1) {
        CW cw = ctx_cw<RAW>(c, lvl0 + DMAX - 1);
        Node L, R;
        expand<B>(c.tab, c.lo, n, cw, L, R);
        if constexpr (NODES) {
            emit_node(c, L);
            emit_node(c, R);
        } else {
            Blk oL, oR;
            mmo_pair<B>(c.tab, c.lo, KeyFixed<false>{}, L.s, oL, KeyFixed<false>{}, R.s, oR);
            store16(c.outp, leaf_fix(oL, L.t, c.fcw));
            store16(c.outp + 16, leaf_fix(oR, R.t, c.fcw));
            c.outp += 32;
        }
    } else {
        CW cw = ctx_cw<RAW>(c, lvl0 + DMAX - D);
        Node L, R;
        expand<B>(c.tab, c.lo, n, cw, L, R);
        // The right child is the only node live across the left subtree.
        Node ch = L;
        const Node pend = R;
#pragma nounroll
        for (int side = 0; side < 2; ++side) {
            dfs<DMAX, D - 1, NODES, PAIR, B, RAW>(c, lvl0, ch);
            ch = pend;
        }
    }
}

// Expand byte-layout DPF keys (dpf.go:89-92,111-112,137-138,165-167) into
// the aligned word records above.  One thread per (key, record).
__global__ void k_unpack(const uint8_t* __restrict__ keys, uint64_t key_len, uint64_t nkeys, uint32_t stop,
                         uint32_t* __restrict__ ek) {
    const uint64_t recs = (uint64_t)stop + 2;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys * recs) return;
    const uint64_t k = i / recs, r = i % recs;
    const uint8_t* kp = keys + k * key_len;
    uint32_t* o = ek + k * (recs * 8) + r * 8;
    auto w = [](const uint8_t* p) {
        return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    };
    if (r == 0) {                         // root seed + t (dpf.go:244-246 / :175-176)
        o[0] = w(kp); o[1] = w(kp + 4); o[2] = w(kp + 8); o[3] = w(kp + 12);
        o[4] = kp[16]; o[5] = 0; o[6] = 0; o[7] = 0;
    } else if (r <= stop) {               // level r-1 CW (dpf.go:231-233)
        const uint8_t* p = kp + 17 + 18 * (r - 1);
        o[0] = w(p); o[1] = w(p + 4); o[2] = w(p + 8); o[3] = w(p + 12);
        o[4] = p[16]; o[5] = p[17]; o[6] = 0; o[7] = 0;
    } else {                              // final CW at len(k)-16 (dpf.go:206,219)
        const uint8_t* p = kp + key_len - 16;
        o[0] = w(p); o[1] = w(p + 4); o[2] = w(p + 8); o[3] = w(p + 12);
        o[4] = 0; o[5] = 0; o[6] = 0; o[7] = 0;
    }
}

// Batched / split EvalFull.  Thread u evaluates subtree `sub_base + (u mod
// 2^units_log)` at level ltop of key (u >> units_log), a block of 2^D leaves
// written at out + key*out_stride + (u mod 2^units_log) * 16 * 2^D.
// NODES: the same walk, but the 2^D nodes at level ltop + D are written to
// (uint4*)out / out_t at [key*out_stride + (u mod 2^units_log) * 2^D].
template <int D, bool UNIFORM, bool NODES, bool RAW = false>
__global__ __launch_bounds__(kTreeBlockMax, kTreeWaves) void k_evalfull(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                        uint64_t nunits, uint32_t units_log, uint32_t ltop,
                                                        uint64_t sub_base, uint8_t* __restrict__ out,
                                                        uint8_t* __restrict__ out_t, uint64_t out_stride,
                                                        uint64_t klen = 0, uint64_t kboff = 0) {
    static_assert(!RAW || (UNIFORM && !NODES), "raw keys: wave-uniform leaf launches only");
#ifdef DPF_WAVE_TIMES
    const uint64_t t_start = wall_clock64();
#endif
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;   // blockDim: 64..kTreeBlockMax
    uint64_t key = u >> units_log;
    if constexpr (UNIFORM) key = __builtin_amdgcn_readfirstlane((uint32_t)key);
    const uint64_t local = u & ((1ull << units_log) - 1);
    const uint64_t sub = sub_base + local;
    Ctx c;
    if constexpr (RAW) {
        c.ks = {nullptr, ekeys, kboff + key * klen, klen};   // ekeys: the raw key batch, 4-byte-aligned base
    } else {
        c.ks = {ekeys + key * ((uint64_t)(stop + 2) * 8), nullptr, 0, 0};
    }
    // Correction words of the walk levels 0..ltop-1 staged in LDS when the
    // whole workgroup evaluates one key (r05).  Read in the walk by scalar
    // loads, each level's CW put an s_waitcnt lgkmcnt(0) -- the counter the
    // T-table lookups also use -- into the middle of the level's dependent
    // AES rounds, exposing an L2 (or HBM) round trip per level of a walk
    // that runs while the CU is otherwise idle.  Here lane l of wave 0 loads
    // level l's CW with vector loads issued before the table fill, and the
    // walks read it from LDS (in-order returns: no wait beyond the round's own).
    __shared__ __attribute__((aligned(16))) uint32_t s_cw[8 * 64];
    const uint32_t Bw = blockDim.x;
    const bool cw_lds = DPF_WALK_CW_LDS && UNIFORM && (Bw & (Bw - 1)) == 0 && stop <= 64 &&
                        units_log >= 31u - (uint32_t)__builtin_clz(Bw) &&
                        (uint64_t)blockIdx.x * Bw < nunits;   // workgroup-uniform
    const bool cw_mine = cw_lds && threadIdx.x < (DPF_DFS_CW_LDS ? stop : ltop);
    CW cw_pre{};
    if (cw_mine) cw_pre = key_cw<RAW>(c.ks, threadIdx.x);   // per-lane level: vector loads
#if DPF_PRIO_FEEDBACK
    __shared__ __attribute__((aligned(16))) uint32_t s_prog[64];
    if (threadIdx.x < 64) s_prog[threadIdx.x] = 0xffffffffu;
#endif
    fill_table_nobar(s_tab);
    if (cw_mine) {
        *reinterpret_cast<uint4*>(s_cw + 8 * threadIdx.x) = make_uint4(cw_pre.s.c0, cw_pre.s.c1, cw_pre.s.c2, cw_pre.s.c3);
        *reinterpret_cast<uint2*>(s_cw + 8 * threadIdx.x + 4) = make_uint2(cw_pre.tl, cw_pre.tr);
    }
    __syncthreads();
    if (u >= nunits) return;
    auto lds_cw = [&](uint32_t lvl) __attribute__((always_inline)) {
        const uint4 a = *reinterpret_cast<const uint4*>(s_cw + 8 * lvl);
        const uint2 b = *reinterpret_cast<const uint2*>(s_cw + 8 * lvl + 4);
        return CW{{a.x, a.y, a.z, a.w}, b.x, b.y};
    };
    // The shared walk below runs only in one-key workgroups, where cw_lds holds.
    auto shared_cw = [&](uint32_t lvl) __attribute__((always_inline)) {
        return DPF_WALK_CW_LDS ? lds_cw(lvl) : key_cw<RAW>(c.ks, lvl);
    };
    c.groups = 0;
    c.cwl = DPF_DFS_CW_LDS && cw_lds ? s_cw : nullptr;
    c.sync = DPF_TREE_SYNC && UNIFORM && !NODES && (uint64_t)(blockIdx.x + 1) * Bw <= nunits;
#if DPF_PRIO_FEEDBACK
    // Only where the workgroup holds all 16 waves of its CU (one
    // kTreeBlockBig-thread workgroup per CU): with two workgroups per CU a
    // wave sees half of its SIMD's waves, and steering by them was 3% slower.
    if (UNIFORM && !NODES && D >= (int)kFeedbackMinD && Bw == 1024u) {
        c.prog = prog_slots(s_prog, c.pslot);
        c.prog[c.pslot] = 0;
    }
#endif
#if DPF_PRIO_STEPS
    __builtin_amdgcn_s_setprio(3);
#endif
    c.tab = reinterpret_cast<const uint8_t*>(s_tab);
    c.lo = (threadIdx.x & 31u) * 4u;
    if constexpr (NODES) {
        c.nseed = reinterpret_cast<uint4*>(out) + key * out_stride + (local << D);
        c.nt = out_t + key * out_stride + (local << D);
    } else {
        c.fcw = key_fcw<RAW>(c.ks, stop);
        c.outp = out + key * out_stride + local * (16ull << D);
    }

    Node n;
    n.s = key_root<RAW>(c.ks, n.t);
    uint32_t lvl = 0;
    if constexpr (UNIFORM) {
        // Shared walk: when the whole workgroup (B = 2^W threads) evaluates
        // consecutive subtrees of one key, its threads' paths agree on the
        // top ltop - W levels and fan out to B nodes below.  Wave 0 walks
        // 64 paths down to level l1 = ltop - W + 6 (one per group of B/64
        // threads) and leaves them in LDS; every thread then walks only the
        // last W - 6 levels.  Wave-AES per workgroup: l1 + (B/64)(W - 6)
        // instead of (B/64) ltop (configs[4]: 33 vs 96, configs[3]: 39 vs 144).
        //
        // Breadth-first finish (DPF_COOP_BFS, r05): instead of every thread
        // walking the last W - 6 levels itself (8 waves x (W - 6) AES, with
        // paths that share 1/2, 1/4, ... of their nodes), the workgroup
        // expands the 64 nodes level by level in LDS: step s has 64 * 2^s
        // parents, one expand (both children, dpf.go:227-240) on each of the
        // first 2^s waves, so W - 6 = 3 steps are 1 + 2 + 4 wave-expands.  At
        // the small per-rank shapes the per-thread walk was ~25% of the tree
        // kernel's AES and ran with all 16 waves of a CU contending for LDS
        // (tools/wave_times.hip, profiles/r05/wave_times: mean walk 25 us of a
        // 51 us PIR-rank launch at N = 8).  Node j of step s sits in slot j
        // (left child 2j, right 2j + 1), so after the last step slot i is
        // thread i's subtree root.
        constexpr uint32_t kFs = DPF_COOP_BFS ? kTreeBlockMax : (1u << (DPF_QUAD_FAN > 6 ? DPF_QUAD_FAN : 6));
        __shared__ uint32_t s_front[5 * kFs];   // SoA: word k of node j at k * kFs + j
        const uint32_t B = blockDim.x;
        const uint32_t W = 31u - (uint32_t)__builtin_clz(B);
        if (DPF_COOP_WALK && (B & (B - 1)) == 0 && W >= 7 && units_log >= W && B <= (uint32_t)kTreeBlockMax &&
            (cw_lds || !DPF_WALK_CW_LDS)) {   // uniform
            // Paths of the shared walk: 2^F, F = 6, or DPF_QUAD_FAN with the
            // quad form when the workgroup has the 4 * 2^F lanes for it.
            const uint32_t F = DPF_QUAD_WALK && DPF_QUAD_FAN > 6 && W >= DPF_QUAD_FAN + 2 ? DPF_QUAD_FAN : 6;
            const uint32_t l1 = ltop - W + F;
            auto put = [&](uint32_t j, const Node& m) {
                s_front[j] = m.s.c0; s_front[kFs + j] = m.s.c1; s_front[2 * kFs + j] = m.s.c2;
                s_front[3 * kFs + j] = m.s.c3; s_front[4 * kFs + j] = m.t;
            };
            auto get = [&](uint32_t j) {
                Node m;
                m.s = {s_front[j], s_front[kFs + j], s_front[2 * kFs + j], s_front[3 * kFs + j]};
                m.t = s_front[4 * kFs + j];
                return m;
            };
            if (DPF_QUAD_WALK && W >= 8) {
                // 2^F paths on the first 2^(F-4) waves, one quad of lanes per
                // path (the latency form: the walk is serial, the CU nearly idle).
                if (threadIdx.x < (4u << F)) {
                    const uint32_t path = threadIdx.x >> 2, j = threadIdx.x & 3u;
                    const uint64_t subj = (sub - threadIdx.x) + ((uint64_t)path << (W - F));
                    const QuadKeys qk = quad_keys(j);
                    uint32_t col = j == 0 ? n.s.c0 : j == 1 ? n.s.c1 : j == 2 ? n.s.c2 : n.s.c3;
                    uint32_t t = n.t;
                    for (uint32_t i = 0; i < l1; ++i) {
                        const CW cw = shared_cw(i);
                        const uint32_t cwj = j == 0 ? cw.s.c0 : j == 1 ? cw.s.c1 : j == 2 ? cw.s.c2 : cw.s.c3;
                        walk_step_quad(c.tab, c.lo, qk, j, col, t, cwj, cw.tl, cw.tr,
                                       (uint32_t)(subj >> (ltop - 1 - i)) & 1u);
                    }
                    s_front[j * kFs + path] = col;
                    if (j == 0) s_front[4 * kFs + path] = t;
                }
            } else if (threadIdx.x < 64) {
                const uint64_t subj = (sub - threadIdx.x) + ((uint64_t)threadIdx.x << (W - 6));
                Node m = n;
                for (uint32_t i = 0; i < l1; ++i) {
                    CW cw = shared_cw(i);
                    walk_step<DPF_WALK_BATCH>(c.tab, c.lo, m, cw, (uint32_t)(subj >> (ltop - 1 - i)) & 1u);
                }
                put(threadIdx.x, m);
            }
            __syncthreads();
#if DPF_COOP_BFS
            for (uint32_t st = 0; st < W - 6; ++st) {
                const bool act = threadIdx.x < (64u << st);           // the first 2^st waves (uniform per wave)
                Node m{};
                if (act) m = get(threadIdx.x);
                __syncthreads();                                       // every parent read before a child lands
                if (act) {
                    const CW cw = key_cw<RAW>(c.ks, l1 + st);
                    Node L, R;
                    expand<DPF_WALK_BATCH>(c.tab, c.lo, m, cw, L, R);
                    put(2 * threadIdx.x, L);
                    put(2 * threadIdx.x + 1, R);
                }
                __syncthreads();
            }
            n = get(threadIdx.x);
            lvl = ltop;
#else
            n = get(threadIdx.x >> (W - F));
            lvl = l1;
#endif
        }
    }
    if (cw_lds) {
        for (uint32_t i = lvl; i < ltop; ++i)
            walk_step<DPF_WALK_BATCH>(c.tab, c.lo, n, lds_cw(i), (uint32_t)(sub >> (ltop - 1 - i)) & 1u);
    } else {
        for (uint32_t i = lvl; i < ltop; ++i)
            walk_step<DPF_WALK_BATCH>(c.tab, c.lo, n, key_cw<RAW>(c.ks, i), (uint32_t)(sub >> (ltop - 1 - i)) & 1u);
    }
#ifdef DPF_WAVE_TIMES
    const uint64_t t_walk = wall_clock64();
#endif
    // Lane pairs share a key when a wave owns one key (UNIFORM): whole-line
    // leaf stores (dfs PAIR).  DPF_PAIR_STORES=0 builds the r02 half-line
    // stores for A/B runs.
    constexpr bool kPair = DPF_PAIR_STORES && UNIFORM && !NODES && D >= 3;
    dfs<D, D, NODES, kPair, UNIFORM, RAW>(c, ltop, n);
#if DPF_PRIO_FEEDBACK
    if (c.prog != nullptr) c.prog[c.pslot] = 0xffffffffu;   // done: no longer the slowest
#endif
#ifdef DPF_WAVE_TIMES
    // Measurement build only (tools/wave_times.hip): per wave, start / end
    // (wall clock) and the hardware ids of the CU it ran on.
    if ((threadIdx.x & 63) == 0) {
        const uint64_t wv = u >> 6;
        if (wv < kWaveTimesMax) {
            g_wave_times[5 * wv] = t_start;
            g_wave_times[5 * wv + 1] = wall_clock64();
            g_wave_times[5 * wv + 2] = __builtin_amdgcn_s_getreg(0xF804);   // HW_ID
            g_wave_times[5 * wv + 3] = __builtin_amdgcn_s_getreg(0xF814);   // XCC_ID
            g_wave_times[5 * wv + 4] = t_walk;                              // root-to-subtree walk done
        }
    }
#endif
}

// Batched Eval: one thread per query, independent walks that compute only
// the child on the path (the reference computes both children, dpf.go:184).
// Without a frontier a walk starts at the root: stop+1 AES per query.  With
// one (fseed != nullptr) it starts from the query's level-L node, written
// by the NODES pass: stop-L+1 AES.  Output: one 0/1 byte per query.
__global__ __launch_bounds__(kBlock, 4) void k_eval(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                    uint32_t logN, const uint64_t* __restrict__ xs, uint64_t nq,
                                                    uint64_t pts_per_key, const uint4* __restrict__ fseed,
                                                    const uint8_t* __restrict__ ft, uint32_t L,
                                                    uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;   // blockDim: 64..kBlock
    if (q >= nq) return;
    const uint64_t key = q / pts_per_key;
    const uint32_t* ek = ekeys + key * ((uint64_t)(stop + 2) * 8);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint64_t x = xs[q];
    Node n;
    uint32_t lvl = 0;
    if (fseed != nullptr) {
        const uint64_t idx = (key << L) + ((x >> (logN - L)) & ((1ull << L) - 1));
        const uint4 v = fseed[idx];
        n.s = {v.x, v.y, v.z, v.w};
        n.t = ft[idx];
        lvl = L;
    } else {
        n.s = load_blk(ek);
        n.t = ek[4];
    }
    for (uint32_t i = lvl; i < stop; ++i) {
        CW cw = load_cw(ek, i);
        walk_step<DPF_EVAL_BATCH>(tab, lo, n, cw, path_bit(x, logN - 1 - i));
    }
    Blk o = mmo1<DPF_EVAL_BATCH>(tab, lo, KeyFixed<false>{}, n.s);
    o = leaf_fix(o, n.t, load_blk(ek + 8 + 8 * stop));
    const uint32_t b = (uint32_t)(x & 127);
    const uint32_t w = (b >> 5) == 0 ? o.c0 : (b >> 5) == 1 ? o.c1 : (b >> 5) == 2 ? o.c2 : o.c3;
    out[q] = (uint8_t)((w >> (b & 31)) & 1u);
}

// Batched Eval, two queries per thread (q = 2u, 2u + 1): the two walks run
// in lockstep (same start level and length), so every AES round issues 32
// lookups per wave instead of 16.  Same output as k_eval.
__device__ __forceinline__ Node eval_start(const uint32_t* ek, uint64_t key, uint64_t x, uint32_t logN,
                                           const uint4* fseed, const uint8_t* ft, uint32_t L) {
    Node n;
    if (fseed != nullptr) {
        const uint64_t idx = (key << L) + ((x >> (logN - L)) & ((1ull << L) - 1));
        const uint4 v = fseed[idx];
        n.s = {v.x, v.y, v.z, v.w};
        n.t = ft[idx];
    } else {
        n.s = load_blk(ek);
        n.t = ek[4];
    }
    return n;
}
__device__ __forceinline__ uint8_t eval_bit(Blk o, uint64_t x) {
    const uint32_t b = (uint32_t)(x & 127);
    const uint32_t w = (b >> 5) == 0 ? o.c0 : (b >> 5) == 1 ? o.c1 : (b >> 5) == 2 ? o.c2 : o.c3;
    return (uint8_t)((w >> (b & 31)) & 1u);
}
struct PairIn {
    uint64_t x0, x1;
    Node n0, n1;
};
// UNI: every wave's 64 pairs (128 consecutive queries) belong to one key
// (pts_per_key a multiple of 128, launch_eval): the key index is wave-uniform,
// so its correction words come through scalar loads into SGPRs instead of
// two per-lane copies in VGPRs (12 fewer VGPRs in the walk: the kernel sits
// at the 128-VGPR limit of 4 waves per SIMD and spilled 35 without it).
template <bool UNI>
__device__ __forceinline__ uint64_t pair_key(uint64_t q, uint64_t pts_per_key) {
    const uint64_t k = q / pts_per_key;
    if constexpr (UNI) return __builtin_amdgcn_readfirstlane((uint32_t)k);
    return k;
}
// The pair's points and start nodes (frontier gathers): issued before the
// workgroup fills its table, so their HBM latency overlaps the fill
// (DPF_EVAL_EARLY; the first pair of every thread).
template <bool UNI>
__device__ __forceinline__ PairIn eval_pair_in(const uint32_t* __restrict__ ekeys, uint32_t stop, uint32_t logN,
                                               const uint64_t* __restrict__ xs, uint64_t nq, uint64_t pts_per_key,
                                               const uint4* __restrict__ fseed, const uint8_t* __restrict__ ft,
                                               uint32_t L, uint64_t q0) {
    const uint64_t qa = q0 < nq ? q0 : nq - 1;
    const uint64_t q1 = qa + 1 < nq ? qa + 1 : qa;
    const uint64_t key0 = pair_key<UNI>(qa, pts_per_key), key1 = UNI ? key0 : q1 / pts_per_key;
    const uint64_t rec = (uint64_t)(stop + 2) * 8;
    PairIn p;
    p.x0 = xs[qa];
    p.x1 = xs[q1];
    p.n0 = eval_start(ekeys + key0 * rec, key0, p.x0, logN, fseed, ft, L);
    p.n1 = eval_start(ekeys + key1 * rec, key1, p.x1, logN, fseed, ft, L);
    return p;
}
// The pair's two answer bits (bit 0: query q0, bit 8: q0 + 1).
template <bool UNI>
__device__ __forceinline__ uint32_t eval_pair_bits(const uint32_t* __restrict__ ekeys, uint32_t stop, uint32_t logN,
                                                   uint64_t nq, uint64_t pts_per_key, const uint4* __restrict__ fseed,
                                                   uint32_t L, const uint32_t* s_tab, uint64_t q0, PairIn p,
                                                   const uint32_t* cwp = nullptr) {
    const uint64_t q1 = q0 + 1 < nq ? q0 + 1 : q0;
    const uint64_t key0 = pair_key<UNI>(q0, pts_per_key), key1 = UNI ? key0 : q1 / pts_per_key;
    const uint64_t rec = (uint64_t)(stop + 2) * 8;
    const uint32_t* ek0 = ekeys + key0 * rec;
    const uint32_t* ek1 = ekeys + key1 * rec;
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t i0 = fseed != nullptr ? L : 0;
    if (UNI && cwp != nullptr) {
        // The key's records from level i0 on, staged in LDS by the caller
        // (k_eval_persist): no scalar load -- whose lgkmcnt(0) would stall
        // the level's first AES round -- inside the walk.
        for (uint32_t i = i0; i < stop; ++i) {
            const uint4 a = *reinterpret_cast<const uint4*>(cwp + 8 * (i - i0));
            const uint2 b = *reinterpret_cast<const uint2*>(cwp + 8 * (i - i0) + 4);
            const CW cw{{a.x, a.y, a.z, a.w}, b.x, b.y};
            walk_step2<DPF_EVAL_BATCH>(tab, lo, p.n0, cw, path_bit(p.x0, logN - 1 - i), p.n1, cw,
                                       path_bit(p.x1, logN - 1 - i));
        }
    } else {
        for (uint32_t i = i0; i < stop; ++i) {
            const CW cw0 = load_cw(ek0, i), cw1 = UNI ? cw0 : load_cw(ek1, i);
            walk_step2<DPF_EVAL_BATCH>(tab, lo, p.n0, cw0, path_bit(p.x0, logN - 1 - i), p.n1, cw1,
                                       path_bit(p.x1, logN - 1 - i));
        }
    }
    Blk o0, o1;
    mmo2<DPF_EVAL_BATCH>(tab, lo, KeyFixed<false>{}, p.n0.s, o0, KeyFixed<false>{}, p.n1.s, o1);
    const Blk f0 = UNI && cwp != nullptr ? load_blk(cwp + 8 * (stop - i0)) : load_blk(ek0 + 8 + 8 * stop);
    o0 = leaf_fix(o0, p.n0.t, f0);
    o1 = leaf_fix(o1, p.n1.t, UNI ? f0 : load_blk(ek1 + 8 + 8 * stop));
    return (uint32_t)eval_bit(o0, p.x0) | ((uint32_t)eval_bit(o1, p.x1) << 8);
}
template <bool UNI>
__device__ __forceinline__ void eval_pair_walk(const uint32_t* __restrict__ ekeys, uint32_t stop, uint32_t logN,
                                               uint64_t nq, uint64_t pts_per_key, const uint4* __restrict__ fseed,
                                               uint32_t L, uint8_t* __restrict__ out, const uint32_t* s_tab,
                                               uint64_t q0, PairIn p) {
    const uint32_t b = eval_pair_bits<UNI>(ekeys, stop, logN, nq, pts_per_key, fseed, L, s_tab, q0, p);
    out[q0] = (uint8_t)b;
    if (q0 + 1 < nq) out[q0 + 1] = (uint8_t)(b >> 8);
}

#ifndef DPF_EVAL_EARLY
#define DPF_EVAL_EARLY 1
#endif
#ifndef DPF_EVAL_PERSIST
#define DPF_EVAL_PERSIST 1   // k_eval_persist for frontier Eval with wave-uniform keys (env DPF_EVAL_PERSIST=0: k_eval2)
#endif
#ifndef DPF_EVAL_FEEDBACK
#define DPF_EVAL_FEEDBACK 3   // k_eval_persist: priority from the wave's lead over its SIMD's slowest; 0: fixed steps
#endif
#ifndef DPF_EVAL_CW_LDS
#define DPF_EVAL_CW_LDS 1   // k_eval_persist: each pair's key records staged in LDS by LDS-DMA (A/B: 0)
#endif
#ifndef DPF_EVAL_PREFETCH
#define DPF_EVAL_PREFETCH 0   // strided k_eval2: next pair's inputs requested before the current walk (A/B)
#endif
template <bool UNI>
__global__ __launch_bounds__(kBlock, 4) void k_eval2(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                     uint32_t logN, const uint64_t* __restrict__ xs, uint64_t nq,
                                                     uint64_t pts_per_key, const uint4* __restrict__ fseed,
                                                     const uint8_t* __restrict__ ft, uint32_t L,
                                                     uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    // Grid-stride loop.  launch_eval launches one thread per query pair
    // (iters = 1); DPF_EVAL_STRIDE=1 caps the grid at the resident
    // workgroups so each fills its 64 KiB table once, with the issue priority
    // stepped down by progress like the tree kernels -- measured slower
    // (3667 vs 3489 us at configs[2]): a thread's frontier gathers are then
    // serialised, where short-lived waves overlap them.
    const uint64_t stride = 2 * (uint64_t)gridDim.x * blockDim.x;
    const uint64_t first = 2 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
    const uint64_t iters = first < nq ? (nq - first + stride - 1) / stride : 0;
#if DPF_EVAL_EARLY
    // The first pair's points and frontier nodes are requested before the
    // table fill (a short-lived wave otherwise waits out their HBM latency
    // after it).
    PairIn p0{};
    if (iters) p0 = eval_pair_in<UNI>(ekeys, stop, logN, xs, nq, pts_per_key, fseed, ft, L, first);
#endif
    fill_table(s_tab);
    __builtin_amdgcn_s_setprio(3);
#if DPF_EVAL_EARLY
    if (iters) eval_pair_walk<UNI>(ekeys, stop, logN, nq, pts_per_key, fseed, L, out, s_tab, first, p0);
    const uint64_t it0 = 1;
#else
    const uint64_t it0 = 0;
#endif
#if DPF_EVAL_PREFETCH
    // Strided form with the next pair's points and frontier nodes requested
    // before the current pair's walk, so their HBM latency hides under it.
    PairIn nx{};
    if (it0 < iters) nx = eval_pair_in<UNI>(ekeys, stop, logN, xs, nq, pts_per_key, fseed, ft, L, first + it0 * stride);
    for (uint64_t it = it0; it < iters; ++it) {
        if (it * 16 >= 15 * iters) __builtin_amdgcn_s_setprio(0);
        else if (it * 16 >= 14 * iters) __builtin_amdgcn_s_setprio(1);
        else if (it * 16 >= 12 * iters) __builtin_amdgcn_s_setprio(2);
        const uint64_t q0 = first + it * stride;
        const PairIn cur = nx;
        if (it + 1 < iters) nx = eval_pair_in<UNI>(ekeys, stop, logN, xs, nq, pts_per_key, fseed, ft, L, q0 + stride);
        eval_pair_walk<UNI>(ekeys, stop, logN, nq, pts_per_key, fseed, L, out, s_tab, q0, cur);
    }
#else
    for (uint64_t it = it0; it < iters; ++it) {
        if (it * 16 >= 15 * iters) __builtin_amdgcn_s_setprio(0);
        else if (it * 16 >= 14 * iters) __builtin_amdgcn_s_setprio(1);
        else if (it * 16 >= 12 * iters) __builtin_amdgcn_s_setprio(2);
        const uint64_t q0 = first + it * stride;
        eval_pair_walk<UNI>(ekeys, stop, logN, nq, pts_per_key, fseed, L, out, s_tab, q0,
                            eval_pair_in<UNI>(ekeys, stop, logN, xs, nq, pts_per_key, fseed, ft, L, q0));
    }
#endif
}

// Persistent batched Eval (r05): one 1024-thread workgroup per CU fills its
// T-table once and strides over the query pairs; the next pair's points and
// frontier nodes move into per-wave LDS slots by LDS-DMA
// (global_load_lds_dwordx4 / _dword) while the current pair walks, so they
// cost no VGPRs (k_eval2 sits at the 128-VGPR limit; a register prefetch of
// the next pair spilled and ran slower, DPF_EVAL_PREFETCH above) and no
// workgroup waits out a fresh table fill or its first gathers.
// Pipeline per thread, iteration i: read x(i) and node(i) from LDS; read
// x(i+1), issue node(i+1)'s gathers; issue x(i+2); walk pair i.  The slots are
// this wave's own, so no barrier: the compiler waits vmcnt(0) before the first
// slot read of an iteration (the DMAs issued one walk earlier), and T-table
// reads (a different LDS object) never wait on them.
// UNI only: a wave's 64 pairs are 128 consecutive queries of one key, and nq
// is even (pts_per_key % 128 == 0), so a pair's points are one 16-byte load.
constexpr int kEvalPBlock = 1024;
struct EvalSlots {
    uint4 x[2][64];      // x(i), x(i+1): {x0, x1} as two uint64
    uint4 n0[64], n1[64]; // frontier seeds of pair i's two queries
    uint32_t t0[64], t1[64];   // aligned dwords holding their t bytes
#if DPF_EVAL_CW_LDS
    uint32_t cw[2][64];  // pair i's key records, levels L..stop-1 and the final CW (parity of i)
#endif
};
// s_waitcnt vmcnt(0) as a compiler memory barrier: the slot DMAs have
// landed and no slot read is hoisted above the wait (hipcc's own waits did
// not cover every slot read once the loop was rotated).
__device__ __forceinline__ void eval_vm0() {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}
// s_waitcnt lgkmcnt(0) that is also a compiler memory barrier: this wave's
// LDS reads of a slot stay above it (and complete before it ends), and the
// LDS-DMA that overwrites the slot stays below it.
__device__ __forceinline__ void eval_lgkm0() {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
}
__device__ __forceinline__ void glds(const void* g, void* l, int size) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (size == 16)
        __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
    else
        __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 4, 0, 0);
#else
    (void)g;
    (void)l;
    (void)size;
#endif
}
__global__ __launch_bounds__(kEvalPBlock, 1) void k_eval_persist(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                                 uint32_t logN, const uint64_t* __restrict__ xs,
                                                                 uint64_t nq, uint64_t pts_per_key,
                                                                 const uint4* __restrict__ fseed,
                                                                 const uint8_t* __restrict__ ft, uint32_t L,
                                                                 uint8_t* __restrict__ out) {
    // The table must sit at LDS address 0, where every lookup's address is
    // its byte index (the ds_read offset field is 16 bits): the stricter
    // alignment places it first.  Behind the 72 KiB of slots it cost one
    // v_add_u32 per lookup, 320 per walk level.
    __shared__ __attribute__((aligned(256))) uint32_t s_tab[kTabWords];
    __shared__ __attribute__((aligned(16))) EvalSlots s_sl[kEvalPBlock / 64];
    const uint32_t lane = threadIdx.x & 63;
    EvalSlots& sl = s_sl[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
    const uint64_t npairs = nq / 2;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // every wave runs the same number of iterations (tail pairs clamped, not stored)
    const uint64_t iters = (npairs + nthr - 1) / nthr;
    auto pair_of = [&](uint64_t i) __attribute__((always_inline)) {
        const uint64_t p = i * nthr + gt;
        return p < npairs ? p : npairs - 1;
    };
    const uint64_t rec = (uint64_t)(stop + 2) * 8;
    const uint32_t ncw = (stop - L) * 8 + 4;
    const bool cw_slots = DPF_EVAL_CW_LDS && ncw <= 64;      // uniform
    (void)rec;
    (void)cw_slots;
    auto issue_x = [&](uint64_t i, int slot) __attribute__((always_inline)) {
        glds(xs + 2 * pair_of(i), &sl.x[slot][0], 16);
    };
    auto issue_nodes = [&](uint64_t i, int slot) __attribute__((always_inline)) {
        const uint4 xv = sl.x[slot][lane];
        const uint64_t x0 = ((uint64_t)xv.y << 32) | xv.x, x1 = ((uint64_t)xv.w << 32) | xv.z;
        const uint64_t key = pair_key<true>(2 * pair_of(i), pts_per_key);
        const uint64_t m = (1ull << L) - 1;
        const uint64_t i0 = (key << L) + ((x0 >> (logN - L)) & m), i1 = (key << L) + ((x1 >> (logN - L)) & m);
        eval_lgkm0();                                    // this wave's reads of the node slots are done
        glds(fseed + i0, &sl.n0[0], 16);
        glds(fseed + i1, &sl.n1[0], 16);
        glds(ft + (i0 & ~3ull), &sl.t0[0], 4);
        glds(ft + (i1 & ~3ull), &sl.t1[0], 4);
#if DPF_EVAL_CW_LDS
        // The key's records from level L: 8 words per level, then the final
        // CW (dpf.go:186-188, :206), one word per lane.  Slot parity i & 1:
        // walk i - 2 (the slot's last reader) is done, by the wait above.
        if (cw_slots && lane < ncw) glds(ekeys + key * rec + 8 + 8 * L + lane, &sl.cw[slot][0], 4);
#endif
    };
    // Pair i's points and nodes into registers, after vmcnt(0): the slot
    // DMAs, issued one walk earlier, and the previous pair's output stores,
    // issued after the previous wait -- so a walk's stores are never waited
    // on right after they issue.
    auto read_pair = [&](uint64_t i) __attribute__((always_inline)) {
        eval_vm0();
        PairIn p;
        const uint4 xv = sl.x[i & 1][lane];
        p.x0 = ((uint64_t)xv.y << 32) | xv.x;
        p.x1 = ((uint64_t)xv.w << 32) | xv.z;
        const uint4 a = sl.n0[lane], b = sl.n1[lane];
        const uint64_t key = pair_key<true>(2 * pair_of(i), pts_per_key);
        const uint64_t m = (1ull << L) - 1;
        const uint32_t i0 = (uint32_t)((key << L) + ((p.x0 >> (logN - L)) & m)) & 3u;
        const uint32_t i1 = (uint32_t)((key << L) + ((p.x1 >> (logN - L)) & m)) & 3u;
        p.n0.s = {a.x, a.y, a.z, a.w};
        p.n1.s = {b.x, b.y, b.z, b.w};
        p.n0.t = (sl.t0[lane] >> (8 * i0)) & 0xffu;
        p.n1.t = (sl.t1[lane] >> (8 * i1)) & 0xffu;
        return p;
    };
    if (iters == 0) return;                               // uniform over the grid
#if DPF_EVAL_FEEDBACK
    // Wave-progress slots per SIMD, as the tree kernel's prio_step feedback form.
    __shared__ __attribute__((aligned(16))) uint32_t s_prog[64];
    if (threadIdx.x < 64) s_prog[threadIdx.x] = 0xffffffffu;
#endif
    issue_x(0, 0);
    if (iters > 1) issue_x(1, 1);
    fill_table(s_tab);
    __builtin_amdgcn_s_setprio(3);
#if DPF_EVAL_FEEDBACK
    uint32_t pslot;
    uint32_t* prog = prog_slots(s_prog, pslot);
    prog[pslot] = 0;
#endif
    issue_nodes(0, 0);
    PairIn p = read_pair(0);
    if (iters > 1) issue_nodes(1, 1);
    if (iters > 2) {
        eval_lgkm0();
        issue_x(2, 0);
    }
    for (uint64_t it = 0; it < iters; ++it) {
#if DPF_EVAL_FEEDBACK
        if ((it & 3) == 0) prio_by_lead(prog, pslot, (uint32_t)it, 4, 4 * DPF_EVAL_FEEDBACK);   // progress: pairs walked
#else
        if (it * 16 >= 15 * iters) __builtin_amdgcn_s_setprio(0);
        else if (it * 16 >= 14 * iters) __builtin_amdgcn_s_setprio(1);
        else if (it * 16 >= 12 * iters) __builtin_amdgcn_s_setprio(2);
#endif
        const uint64_t pr = it * nthr + gt;
#if DPF_EVAL_CW_LDS
        const uint32_t* cwp = cw_slots ? &sl.cw[it & 1][0] : nullptr;
#else
        const uint32_t* cwp = nullptr;
#endif
        const uint32_t b = eval_pair_bits<true>(ekeys, stop, logN, nq, pts_per_key, fseed, L, s_tab, 2 * pair_of(it), p,
                                                cwp);
        // unconditional (the last iteration rereads its own slots): a
        // conditional read leaves the DMAs possibly pending at the join, and
        // the compiler then waits on this pair's stores before issue_nodes
        p = read_pair(it + 1 < iters ? it + 1 : it);
        if (pr < npairs) {
            out[2 * pr] = (uint8_t)b;
            out[2 * pr + 1] = (uint8_t)(b >> 8);
        }
        if (it + 2 < iters) issue_nodes(it + 2, (int)(it & 1));
        if (it + 3 < iters) {
            eval_lgkm0();
            issue_x(it + 3, (int)((it + 1) & 1));
        }
    }
#if DPF_EVAL_FEEDBACK
    prog[pslot] = 0xffffffffu;
#endif
}

#ifndef DPF_EVAL_TRIE_KERNEL
#define DPF_EVAL_TRIE_KERNEL 0   // k_eval_trie is built only in the experimental build (make experimental)
#endif
#if DPF_EVAL_TRIE_KERNEL
// Batched Eval as a visited-node trie below the frontier.
// A key's queries share prefixes: at configs[2] (1024 points per key, stop
// 13) levels 10-13 hold only 647 / 806 / 906 / 963 distinct nodes and 963
// distinct leaf blocks, where per-query walks compute 1024 of each.
//
// r05 layout (k_eval_trie): one key per 512-thread workgroup, the shape and
// LDS budget of k_eval2 (the 64 KiB table plus ~6 KiB of trie metadata: two
// workgroups per CU).  The r04 kernel kept the node seeds of 4 keys in LDS
// too (~88 KiB), so one workgroup filled a CU and every per-level barrier
// idled it (24% slower than the walks).  Here the seeds of the level being
// built live in a scratch slot in global memory that stays in the CU's L2:
// the slot is named by the workgroup's hardware id (XCC, SE, SH, CU, TG
// slot), which no two resident workgroups share, so every CU reuses the same
// few slots and the nodes never need to reach HBM.
//   1. each query marks its node at every level L+1..stop in per-level
//      bitmaps (LDS atomics); one wave per level turns a bitmap into per-word
//      prefix counts: rank(pos) = prefix[pos/32] + popc(bits below);
//   2. per level l = L+1..stop: a map pass (thread per bitmap word) gives
//      each visited node (by rank) its parent: a level-L frontier index
//      (the NODES pass, in HBM) or the parent's rank; then every thread reads
//      the parents of its (<= 2) nodes, a barrier, and computes them, one AES
//      each: dpf.go:183-201's on-path child; at l = stop the leaf MMO and the
//      final CW follow at once (dpf.go:214-224);
//   3. each query reads bit x & 127 of its leaf block by rank.
// AES per key at configs[2]: 1022 (frontier) + 4285 = 5307, against 6142 for
// frontier + per-query walks; wave-AES per key 71 against 80 for k_eval2
// (a wave runs its second AES of a level only if one of its lanes has two
// nodes).  Output: one 0/1 byte per query, as k_eval.
constexpr uint32_t kTrieBlock = 512;        // threads per workgroup (one key)
constexpr uint32_t kTrieCap = 1024;         // points per key (and nodes per level)
constexpr uint32_t kTrieItems = kTrieCap / kTrieBlock;   // nodes per thread per level (2)
constexpr uint32_t kTrieMaxStop = 13;       // bitmaps: 2^l bits per level l <= 13
constexpr uint32_t kTrieWords = 512;        // bitmap words, levels L+1..stop (<= 2^(stop-4))
constexpr uint32_t kTrieMaxLevels = 12;
constexpr uint64_t kTrieSlots = 1ull << 15; // hardware workgroup ids: XCC 3 | SE 3 | SH 1 | CU 4 | TG 4 bits

__host__ __device__ __forceinline__ uint32_t trie_words(uint32_t l) { return l >= 5 ? 1u << (l - 5) : 1u; }

// This workgroup's scratch slot: HW_ID (hwreg 4) fields CU_ID [11:8], SH_ID
// [12], SE_ID [15:13], TG_ID [19:16], and XCC_ID (hwreg 20) [2:0].
__device__ __forceinline__ uint32_t trie_slot() {
    const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804);
    const uint32_t xcc = __builtin_amdgcn_s_getreg(0xF814) & 7u;
    return (xcc << 12) | (((hw >> 13) & 7u) << 9) | (((hw >> 12) & 1u) << 8) | (((hw >> 8) & 15u) << 4) |
           ((hw >> 16) & 15u);
}

__global__ __launch_bounds__(kTrieBlock, 4) void k_eval_trie(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                              uint32_t logN, const uint64_t* __restrict__ xs,
                                                              uint32_t ppk, const uint4* __restrict__ fseed,
                                                              const uint8_t* __restrict__ ft, uint32_t L,
                                                              uint4* __restrict__ scratch,
                                                              uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    __shared__ uint32_t s_bm[kTrieWords];
    __shared__ uint16_t s_pre[kTrieWords];
    __shared__ uint16_t s_map[kTrieCap];          // parent (rank or frontier index) * 2 + side
    __shared__ uint8_t s_t[kTrieCap];             // t bytes of the stored nodes, by rank
    __shared__ uint32_t s_cnt[kTrieMaxLevels];    // visited nodes per level
    const uint32_t tid = threadIdx.x;
    const uint64_t key = blockIdx.x;
    const uint64_t q0 = key * ppk;
    uint4* const scr = scratch + (uint64_t)trie_slot() * kTrieCap;
    const uint32_t* ek = ekeys + key * ((uint64_t)(stop + 2) * 8);
    // Word offset of level l's bitmap (levels L+1..stop).
    auto woff = [&](uint32_t l) {
        uint32_t o = 0;
        for (uint32_t i = L + 1; i < l; ++i) o += trie_words(i);
        return o;
    };
    auto pos_at = [&](uint64_t x, uint32_t l) { return (uint32_t)(x >> (logN - l)) & ((1u << l) - 1u); };
    auto rank = [&](uint32_t wo, uint32_t p) {
        const uint32_t w = wo + (p >> 5);
        return (uint32_t)s_pre[w] + (uint32_t)__builtin_popcount(s_bm[w] & ((1u << (p & 31)) - 1u));
    };
    uint64_t x[kTrieItems];
#pragma unroll
    for (uint32_t j = 0; j < kTrieItems; ++j) {
        const uint32_t i = tid + j * kTrieBlock;
        x[j] = i < ppk ? xs[q0 + i] : 0;                  // issued before the table fill
    }
    for (uint32_t i = tid; i < kTrieWords; i += kTrieBlock) s_bm[i] = 0;
    fill_table(s_tab);                                    // ends with a barrier
    // 1. Mark every query's node at each level L+1..stop.
#pragma unroll
    for (uint32_t j = 0; j < kTrieItems; ++j) {
        if (tid + j * kTrieBlock >= ppk) continue;
        uint32_t wo = 0;
        for (uint32_t l = L + 1; l <= stop; ++l) {
            const uint32_t p = pos_at(x[j], l);
            atomicOr(&s_bm[wo + (p >> 5)], 1u << (p & 31));
            wo += trie_words(l);
        }
    }
    __syncthreads();
    {   // Prefix counts: one wave per level.
        const uint32_t wave = tid >> 6, lane = tid & 63, nlev = stop - L;
        for (uint32_t sg = wave; sg < nlev; sg += kTrieBlock / 64) {
            const uint32_t l = L + 1 + sg;
            const uint32_t base = woff(l), nw = trie_words(l);
            uint32_t carry = 0;
            for (uint32_t c = 0; c < nw; c += 64) {
                const uint32_t w = c + lane;
                const uint32_t v = w < nw ? (uint32_t)__builtin_popcount(s_bm[base + w]) : 0u;
                uint32_t inc = v;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t o = __shfl_up(inc, d, 64);
                    if (lane >= (uint32_t)d) inc += o;
                }
                if (w < nw) s_pre[base + w] = (uint16_t)(carry + inc - v);
                carry += __shfl(inc, 63, 64);
            }
            if (lane == 0) s_cnt[sg] = carry;
        }
    }
    __syncthreads();
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (tid & 31u) * 4u;
    const Blk fcw = load_blk(ek + 8 + 8 * stop);
    uint32_t wo_par = 0;
    for (uint32_t l = L + 1; l <= stop; ++l) {
        const uint32_t wo = l == L + 1 ? 0u : wo_par + trie_words(l - 1), nw = trie_words(l);
        // 2a. Map pass: node rank -> parent * 2 + side.
        for (uint32_t w = tid; w < nw; w += kTrieBlock) {
            uint32_t bits = s_bm[wo + w];
            uint32_t r = s_pre[wo + w];
            while (bits) {
                const uint32_t b = (uint32_t)__builtin_ctz(bits);
                bits &= bits - 1u;
                const uint32_t c = 32u * w + b;
                const uint32_t par = l == L + 1 ? c >> 1 : rank(wo_par, c >> 1);
                s_map[r++] = (uint16_t)((par << 1) | (c & 1u));
            }
        }
        __syncthreads();
        // 2b. Parents of this thread's nodes (rank tid, tid + 512), then a
        // barrier before any node of this level overwrites the slot.
        const uint32_t cnt = s_cnt[l - L - 1];
        Node n[kTrieItems];
        uint32_t side[kTrieItems];
#pragma unroll
        for (uint32_t j = 0; j < kTrieItems; ++j) {
            const uint32_t r = tid + j * kTrieBlock;
            n[j] = {{0, 0, 0, 0}, 0};
            side[j] = 0;
            if (r < cnt) {
                const uint32_t v = s_map[r], par = v >> 1;
                side[j] = v & 1u;
                if (l == L + 1) {
                    const uint64_t idx = (key << L) + par;
                    const uint4 sd = fseed[idx];
                    n[j] = {{sd.x, sd.y, sd.z, sd.w}, ft[idx]};
                } else {
                    const uint4 sd = scr[par];
                    n[j] = {{sd.x, sd.y, sd.z, sd.w}, s_t[par]};
                }
            }
        }
        __syncthreads();
        const CW cw = load_cw(ek, l - 1);
        const uint32_t r1 = tid + kTrieBlock;
        const bool has0 = tid < cnt, has1 = r1 < cnt;
        // A wave runs the second AES of the level only if a lane has a
        // second node (ranks are dense: only the first waves do).
        if (__builtin_amdgcn_read_exec() & __ballot(has1)) {
            walk_step2<DPF_EVAL_BATCH>(tab, lo, n[0], cw, side[0], n[1], cw, side[1]);
            if (l == stop) {                                   // leaf blocks (dpf.go:214-224)
                Blk oa, ob;
                mmo2<DPF_EVAL_BATCH>(tab, lo, KeyFixed<false>{}, n[0].s, oa, KeyFixed<false>{}, n[1].s, ob);
                n[0].s = leaf_fix(oa, n[0].t, fcw);
                n[1].s = leaf_fix(ob, n[1].t, fcw);
            }
        } else if (__builtin_amdgcn_read_exec() & __ballot(has0)) {
            walk_step<DPF_EVAL_BATCH>(tab, lo, n[0], cw, side[0]);
            if (l == stop) n[0].s = leaf_fix(mmo1<DPF_EVAL_BATCH>(tab, lo, KeyFixed<false>{}, n[0].s), n[0].t, fcw);
        }
        if (has0) {
            scr[tid] = make_uint4(n[0].s.c0, n[0].s.c1, n[0].s.c2, n[0].s.c3);
            s_t[tid] = (uint8_t)n[0].t;
        }
        if (has1) {
            scr[r1] = make_uint4(n[1].s.c0, n[1].s.c1, n[1].s.c2, n[1].s.c3);
            s_t[r1] = (uint8_t)n[1].t;
        }
        wo_par = wo;
        __syncthreads();   // this level's nodes stored before the next level reads them
    }
    // 3. Each query's bit of its leaf block.
#pragma unroll
    for (uint32_t j = 0; j < kTrieItems; ++j) {
        const uint32_t i = tid + j * kTrieBlock;
        if (i >= ppk) continue;
        const uint4 o = scr[rank(wo_par, pos_at(x[j], stop))];
        out[q0 + i] = eval_bit({o.x, o.y, o.z, o.w}, x[j]);
    }
}

#endif  // DPF_EVAL_TRIE_KERNEL

// aes128MMO microbenchmark / self-test on the T-table back end: two
// independent blocks per thread (the PRG's own ILP), iterated `reps` times.
template <bool RIGHT>
__global__ __launch_bounds__(kBlock, 4) void k_mmo_tt(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                      uint64_t npairs, uint32_t reps) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= npairs) return;
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint4 va = in[2 * u], vb = in[2 * u + 1];
    Blk a = {va.x, va.y, va.z, va.w}, b = {vb.x, vb.y, vb.z, vb.w};
    for (uint32_t r = 0; r < reps; ++r) mmo_pair<true>(tab, lo, KeyFixed<RIGHT>{}, a, a, KeyFixed<RIGHT>{}, b, b);
    out[2 * u] = make_uint4(a.c0, a.c1, a.c2, a.c3);
    out[2 * u + 1] = make_uint4(b.c0, b.c1, b.c2, b.c3);
}

// ------------------------------------------------------------ launchers ---

hipError_t launch_mmo_tt(const uint8_t* in, uint8_t* out, uint64_t nblocks, uint32_t right, uint32_t reps,
                         hipStream_t st) {
    const uint64_t pairs = nblocks / 2;
    if (pairs == 0) return hipSuccess;
    const dim3 grid((uint32_t)((pairs + kBlock - 1) / kBlock));
    if (right)
        hipLaunchKernelGGL(k_mmo_tt<true>, grid, dim3(kBlock), 0, st, reinterpret_cast<const uint4*>(in),
                           reinterpret_cast<uint4*>(out), pairs, reps);
    else
        hipLaunchKernelGGL(k_mmo_tt<false>, grid, dim3(kBlock), 0, st, reinterpret_cast<const uint4*>(in),
                           reinterpret_cast<uint4*>(out), pairs, reps);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ek,
                         hipStream_t st) {
    const uint64_t n = nkeys * ((uint64_t)stop + 2);
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_unpack, dim3(blocks), dim3(256), 0, st, keys, key_len, nkeys, stop, ek);
    return hipGetLastError();
}

template <int D, bool NODES>
static hipError_t launch_full_d(const uint32_t* ek, uint32_t stop, uint64_t nunits, uint32_t units_log,
                                uint32_t ltop, uint64_t sub_base, uint8_t* out, uint8_t* out_t,
                                uint64_t out_stride, uint32_t block, hipStream_t st) {
    const uint64_t blocks = (nunits + block - 1) / block;
    if (units_log >= 6)
        hipLaunchKernelGGL((k_evalfull<D, true, NODES>), dim3((uint32_t)blocks), dim3(block), 0, st, ek, stop,
                           nunits, units_log, ltop, sub_base, out, out_t, out_stride);
    else
        hipLaunchKernelGGL((k_evalfull<D, false, NODES>), dim3((uint32_t)blocks), dim3(block), 0, st, ek, stop,
                           nunits, units_log, ltop, sub_base, out, out_t, out_stride);
    return hipGetLastError();
}

// CUs a launch may occupy: the calling thread's budget when the C ABI set
// one (a stream created with a CU mask, dpf_stream_create_cu_masked), else
// the device's.  Grid shapes (one round of resident waves, the depth model)
// are sized to it, so a kernel on a 64-CU stream does not queue 4 rounds.
static thread_local int t_cu_budget = 0;
void set_cu_budget(int cus) { t_cu_budget = cus; }
int cu_budget() { return t_cu_budget; }
int cu_count() {
    if (t_cu_budget > 0) return t_cu_budget;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return cus;
}

// Workgroup size for a grid of n threads: full kTreeBlock-thread groups once
// the grid covers every CU, otherwise the smallest power of two (>= one
// wave) that spreads it over all CUs, so that a small batch is not packed
// onto a few CUs whose LDS pipe then serialises it.
static uint32_t pick_block(uint64_t n, uint32_t maxb) {
    const uint64_t cus = (uint64_t)cu_count();
    uint32_t b = 64;
    while (b < maxb && n > cus * b) b <<= 1;
    return b < maxb ? b : maxb;   // maxb need not be a power of two (occ5 variant: 640)
}

// Per-thread subtree depth D and workgroup size.  A thread walks span - D
// levels (one AES each) and expands 3 * 2^D - 2 AES depth-first: deeper
// subtrees amortise the walk, shallower ones give more, shorter threads.
// Time model fitted to tools/archive/exp_latency.sh on MI355X (all batch shapes
// within ~8%): a thread's AES take max(kLat, w * kPerWave) each, w = waves
// per CU (<= 16; more threads run in further rounds).  The throughput regime
// (4096 keys x logN=20) takes D = 7; one key at logN=20 takes D = 0, 14 AES
// deep per thread instead of 197 at D = 7.
// DPF_SUBTREE_DEPTH overrides the choice (measurement only).
struct TreeShape {
    uint32_t d, block;
};
static TreeShape pick_shape(uint32_t span, uint64_t nkeys, bool nodes, uint32_t prefix_bits) {
    static const int forced = [] {
        const char* e = getenv("DPF_SUBTREE_DEPTH");
        return e ? atoi(e) : -1;
    }();
    const uint32_t dmax = span < kMaxD ? span : kMaxD;
    auto threads = [&](uint32_t dd) { return span - dd >= 40 ? ~0ull : nkeys << (span - dd); };
    auto block = [&](uint32_t dd) {
        return pick_block(threads(dd), !nodes && dd >= kBigMinD ? (uint32_t)kTreeBlockBig : (uint32_t)kTreeBlock);
    };
    if (forced >= 0) {
        const uint32_t d = dmax < (uint32_t)forced ? dmax : (uint32_t)forced;
        return {d, block(d)};
    }
    constexpr double kLat = 1.9e-6;       // one AES-MMO of a thread on a lightly loaded CU
    constexpr double kPerWave = 0.2e-6;   // ... per resident wave when the CU's LDS pipe is shared
    const double wave_slots = 64.0 * cu_count();
    uint32_t best = dmax;
    double best_t = 1e30;
    for (int dd = (int)dmax; dd >= 0; --dd) {
        const uint32_t d = (uint32_t)dd;
        double walk = (double)(span - d), lat = 0.0;
        const double w = (double)threads(d) / wave_slots;                 // waves per CU
        const double rounds = w > 16.0 ? std::ceil(w / 16.0) : 1.0;
        const double per = w > 16.0 ? 16.0 * kPerWave : std::max(kLat, w * kPerWave);
#if DPF_DEPTH_MODEL_COOP
        // The shared workgroup walk (k_evalfull, DPF_COOP_WALK): one wave walks
        // the top ltop - W + 6 levels alone (latency, once per round of
        // workgroups), every thread the last W - 6.
        const uint32_t bl = block(d);
        const uint32_t W = 31u - (uint32_t)__builtin_clz(bl);
        if (DPF_COOP_WALK && span - d >= 6 && (bl & (bl - 1)) == 0 && W >= 7 && span - d >= W) {
            walk = DPF_COOP_BFS ? 0.0 : (double)(W - 6);               // BFS: W - 6 lightly loaded steps instead
            lat = (double)(span + prefix_bits - d - W + 6 + (DPF_COOP_BFS ? W - 6 : 0)) * kLat;
        }
#else
        (void)prefix_bits;
#endif
        const double work = walk + (nodes ? 2.0 : 3.0) * (double)(1u << d) - 2.0;   // NODES: no leaf AES
        const double t = rounds * (lat + work * std::max(kLat, per));
        if (t < best_t * 0.98) {          // prefer the deeper subtree on near-ties (less total work)
            best_t = t;
            best = d;
        }
    }
    return {best, block(best)};
}

// Tree pass over every key: leaves of the subtree (prefix_bits, prefix) when
// NODES is false, the 2^depth nodes at level `depth` (prefix 0) when true.
template <bool NODES>
static hipError_t launch_tree(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t depth,
                              uint32_t prefix_bits, uint64_t prefix, uint8_t* out, uint8_t* out_t,
                              uint64_t out_stride, hipStream_t st) {
    const uint32_t span = depth - prefix_bits;          // levels below the prefix node
    const TreeShape sh = pick_shape(span, nkeys, NODES, prefix_bits);
    const uint32_t d = sh.d;                             // per-thread subtree depth
    const uint32_t ltop = depth - d;                     // levels walked per thread
    const uint32_t units_log = ltop - prefix_bits;       // threads per key = 2^units_log
    const uint64_t nunits = nkeys << units_log;
    const uint64_t sub_base = prefix << units_log;
    if (nunits == 0) return hipSuccess;
#define DPF_LAUNCH(DD) \
    return launch_full_d<DD, NODES>(ek, stop, nunits, units_log, ltop, sub_base, out, out_t, out_stride, sh.block, st)
    switch (d) {
        case 0: DPF_LAUNCH(0);
        case 1: DPF_LAUNCH(1);
        case 2: DPF_LAUNCH(2);
        case 3: DPF_LAUNCH(3);
        case 4: DPF_LAUNCH(4);
        case 5: DPF_LAUNCH(5);
        case 6: DPF_LAUNCH(6);
        default: DPF_LAUNCH(7);
    }
#undef DPF_LAUNCH
}

// One-shot EvalFull straight from the key bytes (RAW): only where every wave
// owns one key (the shape launch_tree would pick has >= 64 threads per key)
// and DPF_RAW_KEYS is not 0 (measurement switch).  Any key alignment: the
// kernel reads from the 4-byte-aligned base below `keys`.
bool evalfull_raw_ok(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits) {
    static const bool on = [] {
        const char* e = getenv("DPF_RAW_KEYS");
        return !(e && e[0] == '0');
    }();
    if (!on || nkeys == 0 || prefix_bits > stop) return false;
    const uint32_t span = stop - prefix_bits;
    const TreeShape sh = pick_shape(span, nkeys, false, prefix_bits);
    return span - sh.d >= 6;                             // units_log >= 6: UNIFORM
}

hipError_t launch_evalfull_raw(const uint8_t* keys, uint64_t klen, uint64_t nkeys, uint32_t stop, uint32_t prefix_bits,
                               uint64_t prefix, uint8_t* out, uint64_t out_stride, hipStream_t st) {
    const uint32_t span = stop - prefix_bits;
    const TreeShape sh = pick_shape(span, nkeys, false, prefix_bits);
    const uint32_t d = sh.d, ltop = stop - d, units_log = ltop - prefix_bits;
    if (units_log < 6) return hipErrorInvalidValue;
    const uint64_t nunits = nkeys << units_log, sub_base = prefix << units_log;
    const uint64_t blocks = (nunits + sh.block - 1) / sh.block;
    // Aligned base below the batch, the batch's offset from it in kboff.
    const uint64_t kboff = (uintptr_t)keys & 3;
    const uint32_t* kw = reinterpret_cast<const uint32_t*>(keys - kboff);
#define DPF_RAW(DD)                                                                                                  \
    hipLaunchKernelGGL((k_evalfull<DD, true, false, true>), dim3((uint32_t)blocks), dim3(sh.block), 0, st, kw, stop, \
                       nunits, units_log, ltop, sub_base, out, nullptr, out_stride, klen, kboff);                   \
    break
    switch (d) {
        case 0: DPF_RAW(0);
        case 1: DPF_RAW(1);
        case 2: DPF_RAW(2);
        case 3: DPF_RAW(3);
        case 4: DPF_RAW(4);
        case 5: DPF_RAW(5);
        case 6: DPF_RAW(6);
        default: DPF_RAW(7);
    }
#undef DPF_RAW
    return hipGetLastError();
}

hipError_t launch_nodes(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t depth, uint32_t prefix_bits,
                        uint64_t prefix, uint8_t* seeds, uint8_t* ts, uint64_t stride, hipStream_t st) {
    return launch_tree<true>(ek, nkeys, stop, depth, prefix_bits, prefix, seeds, ts, stride, st);
}

hipError_t launch_evalfull(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t prefix_bits,
                           uint64_t prefix, uint8_t* out, uint64_t out_stride, hipStream_t st) {
    return launch_tree<false>(ek, nkeys, stop, stop, prefix_bits, prefix, out, nullptr, out_stride, st);
}

uint32_t eval_frontier_level(uint32_t stop, uint64_t pts_per_key) {
    // Shared frontier at the deepest level L whose nodes a key's points cover
    // twice over on average: 2^(L+1) <= ppk, i.e. >= 2 points per frontier
    // node (L = 9 at 1024 points per key), used when L >= 4.
    uint32_t L = 0;
    while (L < kMaxFrontierHbm && L < stop && (2ull << (L + 1)) <= pts_per_key) ++L;
    // DPF_EVAL_LEVEL_SHIFT=n (measurement only): the frontier n levels deeper.
    static const int shift = [] {
        const char* e = getenv("DPF_EVAL_LEVEL_SHIFT");
        return e && *e ? atoi(e) : 0;
    }();
    if (L >= 4 && shift > 0 && L + (uint32_t)shift < stop && L + (uint32_t)shift <= kMaxFrontierHbm) L += shift;
    return L >= 4 ? L : 0;
}

uint64_t eval_frontier_bytes(uint64_t nkeys, uint32_t stop, uint64_t pts_per_key) {
    const uint32_t L = eval_frontier_level(stop, pts_per_key);
    if (L == 0) return 0;
    return ((nkeys << L) * 16 + (nkeys << L) + 255) & ~255ull;
}

#if DPF_EVAL_TRIE_KERNEL
// The trie kernel's limits: one key per workgroup, <= 1024 points (2 per
// thread), every level's bitmap in LDS.
static bool trie_ok(uint32_t stop, uint32_t logN, uint64_t ppk, uint32_t L) {
    if (L < 1 || L >= stop || stop > kTrieMaxStop || stop - L > kTrieMaxLevels || logN != stop + 7 || ppk == 0 ||
        ppk > kTrieCap)
        return false;
    uint32_t w = 0;
    for (uint32_t l = L + 1; l <= stop; ++l) w += trie_words(l);
    return w <= kTrieWords;
}
// The trie kernel's scratch slots (kTrieSlots x 16 KiB = 512 MiB per
// device, allocated on first use): one slot per hardware workgroup id, so
// one buffer serves every stream and concurrent launch on the device.
static void* trie_scratch() {
    static std::mutex mu;
    static void* bufs[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!bufs[dev] && hipMalloc(&bufs[dev], kTrieSlots * kTrieCap * 16) != hipSuccess) bufs[dev] = nullptr;
    return bufs[dev];
}

#endif
// Batched Eval kernel (dpf_set_eval_kernel): 0 = frontier + per-query walks,
// 1 = the trie kernel where trie_ok holds.  Env DPF_EVAL_TRIE=0|1 sets the
// initial value.
static std::atomic<int> g_eval_trie{[] {
    const char* e = getenv("DPF_EVAL_TRIE");
    return DPF_EVAL_TRIE_KERNEL && e && e[0] == '1' ? 1 : 0;
}()};
[[maybe_unused]] static bool trie_on() { return g_eval_trie.load(std::memory_order_relaxed) != 0; }
int set_eval_trie(int on) { return g_eval_trie.exchange(on ? 1 : 0); }
bool eval_trie_built() { return DPF_EVAL_TRIE_KERNEL != 0; }
int get_eval_trie() { return g_eval_trie.load(); }

hipError_t launch_eval(const uint32_t* ek, uint32_t stop, uint32_t logN, const uint64_t* xs, uint64_t nq,
                       uint64_t pts_per_key, uint8_t* out, void* frontier, uint64_t frontier_bytes,
                       hipStream_t st) {
    if (nq == 0) return hipSuccess;
    // DPF_EVAL_MODE=plain forces root walks (measurement only).
    static const bool plain = [] {
        const char* e = getenv("DPF_EVAL_MODE");
        return e && e[0] == 'p';
    }();
    const uint64_t nkeys = nq / pts_per_key;
    uint32_t L = eval_frontier_level(stop, pts_per_key);
    if (logN > 63 || plain || frontier == nullptr || frontier_bytes < eval_frontier_bytes(nkeys, stop, pts_per_key)) L = 0;
    const uint4* fseed = nullptr;
    const uint8_t* ft = nullptr;
    if (L > 0) {
        uint8_t* fs = static_cast<uint8_t*>(frontier);
        uint8_t* fts = fs + (nkeys << L) * 16;
        hipError_t e = launch_tree<true>(ek, nkeys, stop, L, 0, 0, fs, fts, 1ull << L, st);
        if (e != hipSuccess) return e;
        fseed = reinterpret_cast<const uint4*>(fs);
        ft = fts;
    }
#if DPF_EVAL_TRIE_KERNEL
    if (L > 0 && trie_on() && trie_ok(stop, logN, pts_per_key, L) && nq == nkeys * pts_per_key) {
        uint4* scr = static_cast<uint4*>(trie_scratch());
        if (scr == nullptr) return hipErrorOutOfMemory;
        hipLaunchKernelGGL(k_eval_trie, dim3((uint32_t)nkeys), dim3(kTrieBlock), 0, st, ek, stop, logN, xs,
                           (uint32_t)pts_per_key, fseed, ft, L, scr, out);
        return hipGetLastError();
    }
#endif
    // Persistent form (k_eval_persist): needs the frontier and wave-uniform keys.
    static const int persist = [] {
        const char* e = getenv("DPF_EVAL_PERSIST");
        return e && *e ? atoi(e) : DPF_EVAL_PERSIST;
    }();
    // Its LDS-DMA stages a pair's two points with one 16-byte load from xs + 2*pair,
    // so it needs a 16-byte-aligned xs; an 8-byte-aligned one (a torch slice
    // xs[1:]) takes k_eval2, whose loads are 8 bytes wide.
    const bool xs16 = (reinterpret_cast<uintptr_t>(xs) & 15u) == 0;
    if (persist && xs16 && L > 0 && pts_per_key % 128 == 0 && nq == nkeys * pts_per_key &&
        nq >= 2 * (uint64_t)kEvalPBlock) {
        const uint64_t want = (nq / 2 + kEvalPBlock - 1) / kEvalPBlock;
        const uint64_t cus = (uint64_t)cu_count();
        hipLaunchKernelGGL(k_eval_persist, dim3((uint32_t)(want < cus ? want : cus)), dim3(kEvalPBlock), 0, st, ek, stop,
                           logN, xs, nq, pts_per_key, fseed, ft, L, out);
        return hipGetLastError();
    }
#if DPF_EVAL_PAIRS
    const uint64_t nthreads = (nq + 1) / 2;
    const uint32_t block = pick_block(nthreads, kBlock);
    uint64_t blocks = (nthreads + block - 1) / block;
    // Resident workgroups only (64 KiB of table each: 2 per CU); k_eval2
    // strides over the rest.
    const uint64_t resident = 2 * (uint64_t)cu_count();
    if (DPF_EVAL_STRIDE && blocks > resident) blocks = resident;
    // Wave-uniform keys when every wave's 128 queries share one key.
    static const bool uni_on = [] {
        const char* e = getenv("DPF_EVAL_UNIFORM");
        return !(e && e[0] == '0');
    }();
    if (uni_on && pts_per_key % 128 == 0 && block % 64 == 0)
        hipLaunchKernelGGL(k_eval2<true>, dim3((uint32_t)blocks), dim3(block), 0, st, ek, stop, logN, xs, nq,
                           pts_per_key, fseed, ft, L, out);
    else
        hipLaunchKernelGGL(k_eval2<false>, dim3((uint32_t)blocks), dim3(block), 0, st, ek, stop, logN, xs, nq,
                           pts_per_key, fseed, ft, L, out);
#else
    const uint32_t block = pick_block(nq, kBlock);
    const uint64_t blocks = (nq + block - 1) / block;
    hipLaunchKernelGGL(k_eval, dim3((uint32_t)blocks), dim3(block), 0, st, ek, stop, logN, xs, nq, pts_per_key,
                       fseed, ft, L, out);
#endif
    return hipGetLastError();
}

}  // namespace dpfk
