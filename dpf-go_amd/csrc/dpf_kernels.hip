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
#include "aes_consts.hpp"
#include "aes_ttable.hpp"
#include "dpf_kernels.hpp"

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

// prg (dpf.go:59-69) plus the parent's CW correction (dpf.go:230-238).
__device__ __forceinline__ void expand(const uint8_t* tab, uint32_t lo, const Node& n, const CW& cw, Node& L,
                                       Node& R) {
    mmo2(tab, lo, KeyFixed<false>{}, n.s, L.s, KeyFixed<true>{}, n.s, R.s);
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
__device__ __forceinline__ void walk_step(const uint8_t* tab, uint32_t lo, Node& n, const CW& cw, uint32_t bit) {
    uint32_t kb = bit ? 0xffffffffu : 0u;
    Blk c = mmo1(tab, lo, KeySel{kb}, n.s);
    uint32_t tc = c.c0 & 1u;
    c.c0 &= ~1u;
    uint32_t m = tmask(n.t);
    c.c0 ^= m & cw.s.c0; c.c1 ^= m & cw.s.c1; c.c2 ^= m & cw.s.c2; c.c3 ^= m & cw.s.c3;
    n.s = c;
    n.t = tc ^ (m & (bit ? cw.tr : cw.tl));
}

__device__ __forceinline__ void store16(uint8_t* p, Blk v) {
    *reinterpret_cast<uint4*>(p) = make_uint4(v.c0, v.c1, v.c2, v.c3);
}

// Leaf conversion (dpf.go:214-224): MMO_L(s) ^ (t != 0 ? finalCW : 0).
__device__ __forceinline__ Blk leaf_fix(Blk o, uint32_t t, Blk fcw) {
    uint32_t m = tmask(t);
    return {o.c0 ^ (m & fcw.c0), o.c1 ^ (m & fcw.c1), o.c2 ^ (m & fcw.c2), o.c3 ^ (m & fcw.c3)};
}

struct Ctx {
    const uint8_t* tab;
    uint32_t lo;
    const uint32_t* ek;
    Blk fcw;
    uint8_t* outp;
};

// Depth-first expansion of D more levels below node n at tree level `lvl0 +
// (DMAX - D)`; the right child of every internal node stays live in
// registers while the left subtree is expanded.
template <int DMAX, int D>
__device__ __forceinline__ void dfs(Ctx& c, uint32_t lvl0, const Node& n) {
    if constexpr (D == 0) {
        Blk o = mmo1(c.tab, c.lo, KeyFixed<false>{}, n.s);
        store16(c.outp, leaf_fix(o, n.t, c.fcw));
        c.outp += 16;
    } else if constexpr (D == 1) {
        CW cw = load_cw(c.ek, lvl0 + DMAX - 1);
        Node L, R;
        expand(c.tab, c.lo, n, cw, L, R);
        Blk oL, oR;
        mmo2(c.tab, c.lo, KeyFixed<false>{}, L.s, oL, KeyFixed<false>{}, R.s, oR);
        store16(c.outp, leaf_fix(oL, L.t, c.fcw));
        store16(c.outp + 16, leaf_fix(oR, R.t, c.fcw));
        c.outp += 32;
    } else {
        CW cw = load_cw(c.ek, lvl0 + DMAX - D);
        Node L, R;
        expand(c.tab, c.lo, n, cw, L, R);
#pragma nounroll
        for (int side = 0; side < 2; ++side) {
            Node ch;
            ch.s.c0 = side ? R.s.c0 : L.s.c0;
            ch.s.c1 = side ? R.s.c1 : L.s.c1;
            ch.s.c2 = side ? R.s.c2 : L.s.c2;
            ch.s.c3 = side ? R.s.c3 : L.s.c3;
            ch.t = side ? R.t : L.t;
            dfs<DMAX, D - 1>(c, lvl0, ch);
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
template <int D, bool UNIFORM>
__global__ __launch_bounds__(kBlock, 4) void k_evalfull(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                        uint64_t nunits, uint32_t units_log, uint32_t ltop,
                                                        uint64_t sub_base, uint8_t* __restrict__ out,
                                                        uint64_t out_stride) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint64_t u = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (u >= nunits) return;
    uint64_t key = u >> units_log;
    if constexpr (UNIFORM) key = __builtin_amdgcn_readfirstlane((uint32_t)key);
    const uint64_t local = u & ((1ull << units_log) - 1);
    const uint64_t sub = sub_base + local;
    const uint32_t* ek = ekeys + key * ((uint64_t)(stop + 2) * 8);

    Ctx c;
    c.tab = reinterpret_cast<const uint8_t*>(s_tab);
    c.lo = (threadIdx.x & 31u) * 4u;
    c.ek = ek;
    c.fcw = load_blk(ek + 8 + 8 * stop);
    c.outp = out + key * out_stride + local * (16ull << D);

    Node n;
    n.s = load_blk(ek);
    n.t = ek[4];
    for (uint32_t i = 0; i < ltop; ++i) {
        CW cw = load_cw(ek, i);
        walk_step(c.tab, c.lo, n, cw, (uint32_t)(sub >> (ltop - 1 - i)) & 1u);
    }
    dfs<D, D>(c, ltop, n);
}

// Batched Eval: one thread per query, independent root-to-leaf walks that
// compute only the child on the path (stop+1 AES; the reference does
// 2*stop+1, dpf.go:183-204).  Output: one 0/1 byte per query, like Eval.
__global__ __launch_bounds__(kBlock, 4) void k_eval(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                    uint32_t logN, const uint64_t* __restrict__ xs, uint64_t nq,
                                                    uint64_t pts_per_key, uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= nq) return;
    const uint64_t key = q / pts_per_key;
    const uint32_t* ek = ekeys + key * ((uint64_t)(stop + 2) * 8);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint64_t x = xs[q];
    Node n;
    n.s = load_blk(ek);
    n.t = ek[4];
    for (uint32_t i = 0; i < stop; ++i) {
        CW cw = load_cw(ek, i);
        walk_step(tab, lo, n, cw, (uint32_t)(x >> (logN - 1 - i)) & 1u);
    }
    Blk o = mmo1(tab, lo, KeyFixed<false>{}, n.s);
    o = leaf_fix(o, n.t, load_blk(ek + 8 + 8 * stop));
    const uint32_t b = (uint32_t)(x & 127);
    const uint32_t w = (b >> 5) == 0 ? o.c0 : (b >> 5) == 1 ? o.c1 : (b >> 5) == 2 ? o.c2 : o.c3;
    out[q] = (uint8_t)((w >> (b & 31)) & 1u);
}

// Batched Eval with a shared frontier: many random points of
// one key share the top of the tree, so a workgroup first expands its key
// breadth-first to level L (2^L nodes in LDS, 2^L - 2 AES in all instead of
// L per query), then every query continues from its level-L node: stop - L
// path AES + the leaf MMO.  At configs[2] (1024 points, logN=20, L=9) that
// is 1022 + 1024*5 AES per key instead of 1024*14.  Each workgroup loops
// over keys so the LDS table is filled once.
template <int L>
__global__ __launch_bounds__(kBlock, 4) void k_eval_frontier(const uint32_t* __restrict__ ekeys, uint32_t stop,
                                                             uint32_t logN, const uint64_t* __restrict__ xs,
                                                             uint64_t nkeys, uint64_t pts_per_key,
                                                             uint8_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    // Levels alternate between two node buffers, level L always in A.
    __shared__ uint4 s_a[1 << L];
    __shared__ uint32_t s_at[1 << L];
    __shared__ uint4 s_b[(1 << L) / 2 > 0 ? (1 << L) / 2 : 1];
    __shared__ uint32_t s_bt[(1 << L) / 2 > 0 ? (1 << L) / 2 : 1];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    for (uint64_t key = blockIdx.x; key < nkeys; key += gridDim.x) {
        const uint32_t* ek = ekeys + key * ((uint64_t)(stop + 2) * 8);
        __syncthreads();   // previous key's queries are done with s_a
        if (threadIdx.x == 0) {
            Blk r = load_blk(ek);
            ((L & 1) ? s_b : s_a)[0] = make_uint4(r.c0, r.c1, r.c2, r.c3);
            ((L & 1) ? s_bt : s_at)[0] = ek[4];
        }
        // breadth-first: level d from level d-1 (d = 1..L)
        for (int d = 1; d <= L; ++d) {
            __syncthreads();
            const bool to_a = ((L - d) & 1) == 0;
            const uint4* src = to_a ? s_b : s_a;
            const uint32_t* srct = to_a ? s_bt : s_at;
            uint4* dst = to_a ? s_a : s_b;
            uint32_t* dstt = to_a ? s_at : s_bt;
            const CW cw = load_cw(ek, d - 1);
            for (uint32_t i = threadIdx.x; i < (1u << (d - 1)); i += blockDim.x) {
                Node n;
                const uint4 v = src[i];
                n.s = {v.x, v.y, v.z, v.w};
                n.t = srct[i];
                Node Lc, Rc;
                expand(tab, lo, n, cw, Lc, Rc);
                dst[2 * i] = make_uint4(Lc.s.c0, Lc.s.c1, Lc.s.c2, Lc.s.c3);
                dst[2 * i + 1] = make_uint4(Rc.s.c0, Rc.s.c1, Rc.s.c2, Rc.s.c3);
                dstt[2 * i] = Lc.t;
                dstt[2 * i + 1] = Rc.t;
            }
        }
        __syncthreads();
        const Blk fcw = load_blk(ek + 8 + 8 * stop);
        for (uint64_t q = threadIdx.x; q < pts_per_key; q += blockDim.x) {
            const uint64_t gq = key * pts_per_key + q;
            const uint64_t x = xs[gq];
            const uint32_t top = (uint32_t)(x >> (logN - L)) & ((1u << L) - 1);
            Node n;
            const uint4 v = s_a[top];
            n.s = {v.x, v.y, v.z, v.w};
            n.t = s_at[top];
            for (uint32_t i = L; i < stop; ++i) {
                CW cw = load_cw(ek, i);
                walk_step(tab, lo, n, cw, (uint32_t)(x >> (logN - 1 - i)) & 1u);
            }
            Blk o = mmo1(tab, lo, KeyFixed<false>{}, n.s);
            o = leaf_fix(o, n.t, fcw);
            const uint32_t b = (uint32_t)(x & 127);
            const uint32_t w = (b >> 5) == 0 ? o.c0 : (b >> 5) == 1 ? o.c1 : (b >> 5) == 2 ? o.c2 : o.c3;
            out[gq] = (uint8_t)((w >> (b & 31)) & 1u);
        }
    }
}

// ------------------------------------------------------------ launchers ---

hipError_t launch_unpack(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ek,
                         hipStream_t st) {
    const uint64_t n = nkeys * ((uint64_t)stop + 2);
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_unpack, dim3(blocks), dim3(256), 0, st, keys, key_len, nkeys, stop, ek);
    return hipGetLastError();
}

template <int D>
static hipError_t launch_full_d(const uint32_t* ek, uint32_t stop, uint64_t nunits, uint32_t units_log,
                                uint32_t ltop, uint64_t sub_base, uint8_t* out, uint64_t out_stride,
                                hipStream_t st) {
    const uint64_t blocks = (nunits + kBlock - 1) / kBlock;
    if (units_log >= 6)
        hipLaunchKernelGGL((k_evalfull<D, true>), dim3((uint32_t)blocks), dim3(kBlock), 0, st, ek, stop, nunits,
                           units_log, ltop, sub_base, out, out_stride);
    else
        hipLaunchKernelGGL((k_evalfull<D, false>), dim3((uint32_t)blocks), dim3(kBlock), 0, st, ek, stop, nunits,
                           units_log, ltop, sub_base, out, out_stride);
    return hipGetLastError();
}

// Per-thread subtree depth.  Deeper subtrees amortise the root-to-subtree
// walk (ltop AES per thread against 3*2^D - 2), but a small batch of keys
// then launches too few threads to fill the GPU; shrink D (not below kMinD)
// until the grid reaches two 512-thread workgroups per CU.
// DPF_SUBTREE_DEPTH overrides the choice (measurement only).
static uint32_t pick_depth(uint32_t span, uint64_t nkeys) {
    static const int forced = [] {
        const char* e = getenv("DPF_SUBTREE_DEPTH");
        return e ? atoi(e) : -1;
    }();
    uint32_t d = span < kMaxD ? span : kMaxD;
    if (forced >= 0) return span < (uint32_t)forced ? span : (uint32_t)forced;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const uint64_t fill = (uint64_t)cus * 2 * kBlock;
    auto threads = [&](uint32_t dd) { return span - dd >= 40 ? ~0ull : nkeys << (span - dd); };
    while (d > kMinD && threads(d) < fill) --d;
    return d;
}

hipError_t launch_evalfull(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t prefix_bits,
                           uint64_t prefix, uint8_t* out, uint64_t out_stride, hipStream_t st) {
    const uint32_t span = stop - prefix_bits;          // levels below the prefix node
    const uint32_t d = pick_depth(span, nkeys);         // per-thread subtree depth
    const uint32_t ltop = stop - d;                     // levels walked per thread
    const uint32_t units_log = ltop - prefix_bits;      // threads per key = 2^units_log
    const uint64_t nunits = nkeys << units_log;
    const uint64_t sub_base = prefix << units_log;
    if (nunits == 0) return hipSuccess;
    switch (d) {
        case 0: return launch_full_d<0>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        case 1: return launch_full_d<1>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        case 2: return launch_full_d<2>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        case 3: return launch_full_d<3>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        case 4: return launch_full_d<4>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        case 5: return launch_full_d<5>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        case 6: return launch_full_d<6>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
        default: return launch_full_d<7>(ek, stop, nunits, units_log, ltop, sub_base, out, out_stride, st);
    }
}

template <int L>
static hipError_t launch_frontier(const uint32_t* ek, uint32_t stop, uint32_t logN, const uint64_t* xs,
                                  uint64_t nkeys, uint64_t ppk, uint8_t* out, hipStream_t st) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const uint64_t grid = nkeys < (uint64_t)cus * 2 ? nkeys : (uint64_t)cus * 2;
    hipLaunchKernelGGL((k_eval_frontier<L>), dim3((uint32_t)grid), dim3(kBlock), 0, st, ek, stop, logN, xs, nkeys,
                       ppk, out);
    return hipGetLastError();
}

hipError_t launch_eval(const uint32_t* ek, uint32_t stop, uint32_t logN, const uint64_t* xs, uint64_t nq,
                       uint64_t pts_per_key, uint8_t* out, hipStream_t st) {
    if (nq == 0) return hipSuccess;
    // Shared frontier at level L when a key's points cover it: 2^L <= ppk / 2.
    static const bool no_frontier = getenv("DPF_EVAL_NO_FRONTIER") != nullptr;
    uint32_t L = 0;
    while (L < kMaxFrontier && L < stop && (2ull << (L + 1)) <= pts_per_key) ++L;
    if (!no_frontier && L >= 6) {
        const uint64_t nkeys = nq / pts_per_key;
        switch (L) {
            case 6: return launch_frontier<6>(ek, stop, logN, xs, nkeys, pts_per_key, out, st);
            case 7: return launch_frontier<7>(ek, stop, logN, xs, nkeys, pts_per_key, out, st);
            case 8: return launch_frontier<8>(ek, stop, logN, xs, nkeys, pts_per_key, out, st);
            default: return launch_frontier<9>(ek, stop, logN, xs, nkeys, pts_per_key, out, st);
        }
    }
    const uint64_t blocks = (nq + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_eval, dim3((uint32_t)blocks), dim3(kBlock), 0, st, ek, stop, logN, xs, nq, pts_per_key,
                       out);
    return hipGetLastError();
}

}  // namespace dpfk
