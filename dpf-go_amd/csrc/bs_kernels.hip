// bs_kernels.hip — EvalFull with the byte-sliced (table-free) AES back end.
//
// Reference: evalFullRecursive / EvalFull (dpf/dpf.go:213-262) over prg
// (dpf.go:59-69) and aes128MMO (dpf/aes_amd64.s:51-82).  Same outputs as the
// T-table tree kernel (dpf_kernels.hip), bit for bit.
//
// Work split (one launch of each):
//   1. k_evalfull<NODES> (T-table, dpf_kernels.hip) writes the frontier: the
//      2^f nodes of every key at level f = stop - D (seed + t byte);
//   2. k_evalfull_bs<D>: a lane takes 8 consecutive frontier nodes as one
//      byte-sliced set (aes_bytesliced.hpp) and expands them D levels
//      depth-first.  An expansion is two AES-MMO sets (all 8 nodes under the
//      left key, then the right key); the 16 children are repacked into the
//      next two sets of 8 consecutive nodes with one shift + one v_bitop3 per
//      word (the block order inside a set follows a fixed 3-cycle pattern,
//      sigma below), so the leaf sets are 8 consecutive leaves = one 128-byte
//      line per lane, written with 8 back-to-back 16-byte stores.
// All lanes of a wave run the same DFS (uniform control flow); with >= 64
// lanes per key (logN >= 20) the wave is one key and the correction words
// come through scalar loads.  One AES body serves every step (a loop over
// steps), so the code stays ~1 AES round of instructions.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aes_bytesliced.hpp"
#include "bs_kernels.hpp"
#include "dpf_kernels.hpp"
#include "wave_prio.hpp"

#ifndef DPF_BS_PRIO
#define DPF_BS_PRIO 1   // issue priority by progress in k_evalfull_bs
#endif
#ifndef DPF_BS_FEEDBACK
#define DPF_BS_FEEDBACK 0   // >0: 512-thread workgroups (every wave of a CU) and progress-feedback priority (A/B)
#endif

namespace dpfk {

using bs::aes_mmo8;
using bs::transpose32;

// Byte-sliced correction words: per key, `stop` level records of 36 words
// (32 sCW planes, then XL, YL, XR, YR) and the final CW (32 planes).
// Plane word (8*row + plane), byte c = 0xFF iff bit `plane` of CW byte
// (c, row) is set.  t classes (tCW byte v): X = v == 1, Y = v > 1 (as masks),
// so that a child's "t != 0" is  tp ? ((b ^ X) | Y) : b  for its raw bit b
// (dpf.go:185-193,230-238: t bytes XOR as bytes, tested != 0).
constexpr uint32_t kBsRec = 36;

__host__ __device__ uint64_t bs_key_words(uint32_t stop) { return (uint64_t)stop * kBsRec + 32; }

__device__ __forceinline__ uint32_t planes_word(const uint8_t* p, uint32_t row, uint32_t plane) {
    uint32_t v = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        if ((p[4 * c + row] >> plane) & 1u) v |= 0xFFu << (8 * c);
    return v;
}

// One thread per (key, record): record r < stop = level r, r == stop = final CW.
__global__ void k_unpack_bs(const uint8_t* __restrict__ keys, uint64_t key_len, uint64_t nkeys, uint32_t stop,
                            uint32_t* __restrict__ ekb) {
    const uint64_t recs = (uint64_t)stop + 1;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys * recs) return;
    const uint64_t k = i / recs, r = i % recs;
    const uint8_t* kp = keys + k * key_len;
    uint32_t* o = ekb + k * bs_key_words(stop) + r * kBsRec;
    const uint8_t* p = r < stop ? kp + 17 + 18 * r : kp + key_len - 16;   // dpf.go:231-233 / :206,219
    for (uint32_t w = 0; w < 32; ++w) o[w] = planes_word(p, w >> 3, w & 7);
    if (r < stop) {
        const uint8_t tl = p[16], tr = p[17];
        o[32] = tl == 1 ? ~0u : 0u;
        o[33] = tl > 1 ? ~0u : 0u;
        o[34] = tr == 1 ? ~0u : 0u;
        o[35] = tr > 1 ? ~0u : 0u;
    }
}

// Both back ends' key records in one launch, one thread per output word
// (the tree workspace holds both, so either back end can run from one
// expansion): record r of a key has 8 T-table words (k_unpack's layout,
// dpf_kernels.hip) and, for r >= 1, the byte-sliced record r-1 (36 words;
// 32 for the final CW).  Replaces k_unpack + k_unpack_bs (2 launches, one
// thread per record) on the tree paths.
constexpr uint32_t kUnpackWords = 8 + kBsRec;
__global__ void k_unpack_both(const uint8_t* __restrict__ keys, uint64_t key_len, uint64_t nkeys, uint32_t stop,
                              uint32_t* __restrict__ ek, uint32_t* __restrict__ ekb) {
    const uint64_t recs = (uint64_t)stop + 2;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys * recs * kUnpackWords) return;
    const uint64_t k = i / (recs * kUnpackWords), rem = i % (recs * kUnpackWords);
    const uint32_t r = (uint32_t)(rem / kUnpackWords), w = (uint32_t)(rem % kUnpackWords);
    const uint8_t* kp = keys + k * key_len;
    // byte source of record r: root (dpf.go:244-246), level r-1 CW (:231-233), final CW at len-16 (:206,219)
    const uint8_t* p = r == 0 ? kp : r <= stop ? kp + 17 + 18 * (r - 1) : kp + key_len - 16;
    if (w < 8) {
        uint32_t v = 0;
        if (w < 4) {
            v = (uint32_t)p[4 * w] | ((uint32_t)p[4 * w + 1] << 8) | ((uint32_t)p[4 * w + 2] << 16) |
                ((uint32_t)p[4 * w + 3] << 24);
        } else if (w == 4 && r <= stop) {
            v = p[16];                                   // root t / tLCW
        } else if (w == 5 && r >= 1 && r <= stop) {
            v = p[17];                                   // tRCW
        }
        ek[k * (recs * 8) + r * 8 + w] = v;
        return;
    }
    if (r == 0) return;                                  // the root has no byte-sliced record
    const uint32_t rb = r - 1, j = w - 8;                // rb == stop: the final CW
    if (rb == stop && j >= 32) return;
    uint32_t v;
    if (j < 32) {
        v = planes_word(p, j >> 3, j & 7);
    } else {
        const uint8_t t = p[16 + ((j - 32) >> 1)];      // tLCW for 32/33, tRCW for 34/35
        v = (j & 1) ? (t > 1 ? ~0u : 0u) : (t == 1 ? ~0u : 0u);
    }
    ekb[k * bs_key_words(stop) + (uint64_t)rb * kBsRec + j] = v;
}

hipError_t launch_unpack_both(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ek,
                              uint32_t* ekb, hipStream_t st) {
    const uint64_t n = nkeys * ((uint64_t)stop + 2) * kUnpackWords;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_both, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, keys, key_len, nkeys, stop,
                       ek, ekb);
    return hipGetLastError();
}

// The byte-sliced records from the T-table records already in the
// workspace (ek, k_unpack's layout: 16 CW bytes as 4 little-endian words,
// then tLCW, tRCW as words 4, 5), one thread per output word.  Lets the
// T-table paths unpack only their own 8-word records and build these only
// when the byte-sliced back end runs.
__global__ void k_bs_from_ek(const uint32_t* __restrict__ ek, uint64_t nkeys, uint32_t stop,
                             uint32_t* __restrict__ ekb) {
    const uint64_t per = bs_key_words(stop);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkeys * per) return;
    const uint64_t k = i / per, rem = i % per;
    const uint32_t rb = (uint32_t)(rem / kBsRec), j = (uint32_t)(rem % kBsRec);   // rb == stop: the final CW
    const uint32_t* rec = ek + k * ((uint64_t)(stop + 2) * 8) + (uint64_t)(rb + 1) * 8;
    uint32_t v;
    if (j < 32) {
        v = planes_word(reinterpret_cast<const uint8_t*>(rec), j >> 3, j & 7);
    } else {
        const uint8_t t = (uint8_t)rec[4 + ((j - 32) >> 1)];   // tLCW for 32/33, tRCW for 34/35
        v = (j & 1) ? (t > 1 ? ~0u : 0u) : (t == 1 ? ~0u : 0u);
    }
    ekb[i] = v;
}

hipError_t launch_bs_from_ek(const uint32_t* ek, uint64_t nkeys, uint32_t stop, uint32_t* ekb, hipStream_t st) {
    const uint64_t n = nkeys * bs_key_words(stop);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_bs_from_ek, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, ek, nkeys, stop, ekb);
    return hipGetLastError();
}

// Child set after aes_mmo8 (o = MMO(x)): split the control bits off (byte 0
// of row 0 / plane 0), clear them, apply the parent's correction (dpf.go:
// 61-68,230-238).  tp: parent "t != 0" mask (bit i of every byte = block i).
__device__ __forceinline__ uint32_t child_fix(uint32_t (&o)[32], uint32_t tp, const uint32_t* __restrict__ cw,
                                              uint32_t side) {
    const uint32_t b = __builtin_amdgcn_perm(o[0], o[0], 0u);   // raw t bits, broadcast to 4 bytes
    o[0] &= 0xFFFFFF00u;
#pragma unroll
    for (int w = 0; w < 32; ++w) o[w] = __builtin_amdgcn_bitop3_b32(o[w], tp, cw[w], 0x78);   // o ^ (tp & cw)
    const uint32_t X = cw[32 + 2 * side], Y = cw[33 + 2 * side];
    return (tp & ((b ^ X) | Y)) | (~tp & b);
}

// Repack children of 8 consecutive nodes: L/R sets (same block order) ->
// A = first 8 children, B = last 8.  Shift s and mask m by depth (see sigma).
__device__ __forceinline__ uint32_t rp_a(uint32_t l, uint32_t r, uint32_t s, uint32_t m) {
    return __builtin_amdgcn_bitop3_b32(l, r << s, m, 0xe4);   // m ? l : r << s
}
__device__ __forceinline__ uint32_t rp_b(uint32_t l, uint32_t r, uint32_t s, uint32_t m) {
    return __builtin_amdgcn_bitop3_b32(l >> s, r, m, 0xe4);   // m ? l >> s : r
}

// Leaf conversion of a set (MMO_L output o, leaf t mask tl): ^ (t ? finalCW :
// 0), back to 8 blocks, 8 consecutive 16-byte stores (one 128-byte line).
__device__ __forceinline__ void leaf_store(uint32_t (&o)[32], uint32_t tl, const uint32_t* __restrict__ fcw,
                                           uint8_t* p, const Sigma& sig) {
#pragma unroll
    for (int w = 0; w < 32; ++w) o[w] = __builtin_amdgcn_bitop3_b32(o[w], tl, fcw[w], 0x78);
    transpose32(o);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        *reinterpret_cast<uint4*>(p + 16 * sig.v[i]) = make_uint4(o[i], o[8 + i], o[16 + i], o[24 + i]);
}

#define DPF_BS_COPY(DST, SRC) _Pragma("unroll") for (int w_ = 0; w_ < 32; ++w_) DST[w_] = SRC[w_];
#define DPF_BS_PUSH_LDS(SLOT, SRC) \
    _Pragma("unroll") for (int q_ = 0; q_ < 8; ++q_) \
        lds[SLOT][q_][lane] = make_uint4(SRC[4 * q_], SRC[4 * q_ + 1], SRC[4 * q_ + 2], SRC[4 * q_ + 3]);
#define DPF_BS_POP_LDS(SLOT, DST) \
    _Pragma("unroll") for (int q_ = 0; q_ < 8; ++q_) { \
        const uint4 v_ = lds[SLOT][q_][lane]; \
        DST[4 * q_] = v_.x; DST[4 * q_ + 1] = v_.y; DST[4 * q_ + 2] = v_.z; DST[4 * q_ + 3] = v_.w; \
    }

constexpr int kBsBlock = DPF_BS_FEEDBACK ? 512 : 256;

// Thread u: key u >> (flog - 3), frontier nodes 8*(u mod 2^(flog-3)) .. +7
// of that key (level lvl0; 2^flog frontier nodes per key).  Output: 2^D
// leaves of 16 B below each node, at out + key * out_stride.
template <int D, bool UNIFORM>
__global__ __launch_bounds__(kBsBlock, 2) void k_evalfull_bs(const uint4* __restrict__ fseed,
                                                        const uint8_t* __restrict__ ft, uint32_t flog,
                                                        const uint32_t* __restrict__ ekb, uint32_t stop,
                                                        uint32_t lvl0, uint64_t nthreads, uint8_t* __restrict__ out,
                                                        uint64_t out_stride) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
#if DPF_BS_FEEDBACK
    __shared__ __attribute__((aligned(16))) uint32_t s_prog[64];
    if (threadIdx.x < 64) s_prog[threadIdx.x] = 0xffffffffu;
    __syncthreads();                               // before any wave returns or reads the slots
    uint32_t pslot = 0;
    uint32_t* prog = blockDim.x == 512u ? prog_slots(s_prog, pslot) : nullptr;
#endif
    if (u >= nthreads) return;
#if DPF_BS_FEEDBACK
    if (prog) prog[pslot] = 0;
#endif
    const uint32_t glog = flog - 3;
    uint64_t key = u >> glog;
    if constexpr (UNIFORM) key = __builtin_amdgcn_readfirstlane((uint32_t)key);
    const uint64_t g = u & ((1ull << glog) - 1);
    const uint64_t node0 = (key << flog) + 8 * g;
    const uint32_t* ek = ekb + key * bs_key_words(stop);
    const uint32_t* fcw = ek + (uint64_t)stop * kBsRec;
    uint8_t* obase = out + key * out_stride + ((g * 8) << D) * 16;
    constexpr Sigma sig = sigma_at(D);

    uint32_t X[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {                 // M[8c + i] = word c of block i
        const uint4 v = fseed[node0 + i];
        X[i] = v.x; X[8 + i] = v.y; X[16 + i] = v.z; X[24 + i] = v.w;
    }
    transpose32(X);
    uint32_t tX = 0;
    {
        const uint2 tw = *reinterpret_cast<const uint2*>(ft + node0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t byte = ((i < 4 ? tw.x : tw.y) >> (8 * (i & 3))) & 0xFFu;
            tX |= (byte != 0 ? 1u : 0u) << i;
        }
        tX *= 0x01010101u;
    }

    // Depth-first over sets.  An iteration expands X (depth d < D, set
    // index `path` among the 2^d sets of the lane at that depth): left and
    // right AES-MMO sets, repack into A (first 8 children) and B (last 8).
    // Above the leaves A is expanded next and B waits in a stack slot; at
    // the bottom A and B are leaf sets.  Four AES call sites, no per-step
    // register copies besides the stack.
    // Stack of pending right sets: depth 2 in VGPRs; depths 0 and 1 (pushed
    // once / twice per lane) in this wave's LDS rows, which leaves the AES
    // rounds ~180 VGPRs to schedule in at 2 waves/SIMD.
    __shared__ uint4 s_stack[kBsBlock / 64][2][8][64];
    uint4 (*lds)[8][64] = s_stack[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    uint32_t S2[32];
    uint32_t tS0 = 0, tS1 = 0, tS2 = 0;
    uint32_t d = 0, path = 0;
#if DPF_BS_PRIO
    // Issue priority by progress, as the T-table tree kernel's prio_step:
    // 3 until 3/4 of the lane's leaf-set pairs, 2, then 1 at 7/8.
    uint32_t pairs = 0;
    constexpr uint32_t kPairs = 1u << (D - 1);
    __builtin_amdgcn_s_setprio(3);
#endif
    for (;;) {
        const uint32_t* cw = ek + (uint64_t)(lvl0 + d) * kBsRec;
        uint32_t L[32], R[32], B[32];
        aes_mmo8(X, L, 0);
        const uint32_t tL = child_fix(L, tX, cw, 0);
        aes_mmo8(X, R, 1);
        const uint32_t tR = child_fix(R, tX, cw, 1);
        // shift / mask cycle by depth: 4 / 0x0F, 2 / 0x33, 1 / 0x55
        const uint32_t dm = d % 3;
        const uint32_t sh = dm == 0 ? 4u : dm == 1 ? 2u : 1u;
        const uint32_t m = dm == 0 ? 0x0F0F0F0Fu : dm == 1 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int w = 0; w < 32; ++w) {
            X[w] = rp_a(L[w], R[w], sh, m);
            B[w] = rp_b(L[w], R[w], sh, m);
        }
        const uint32_t tB = rp_b(tL, tR, sh, m);
        tX = rp_a(tL, tR, sh, m);
        path <<= 1;
        if (d + 1 < D) {
            switch (d) {                            // push B (static register slots)
                case 0: DPF_BS_PUSH_LDS(0, B) tS0 = tB; break;
                case 1: DPF_BS_PUSH_LDS(1, B) tS1 = tB; break;
                default: DPF_BS_COPY(S2, B) tS2 = tB; break;
            }
            ++d;
            continue;
        }
        // Leaf sets A (X) and B: 8 consecutive leaves 8*path + sigma(i) each (dpf.go:214-224).
        {
            uint32_t O[32];
            aes_mmo8(X, O, 0);
            leaf_store(O, tX, fcw, obase + (uint64_t)path * 128, sig);
        }
        {
            uint32_t O[32];
            aes_mmo8(B, O, 0);
            leaf_store(O, tB, fcw, obase + (uint64_t)(path + 1) * 128, sig);
        }
#if DPF_BS_PRIO
        ++pairs;
#if DPF_BS_FEEDBACK
        if (prog) prio_by_lead(prog, pslot, pairs, 1, DPF_BS_FEEDBACK);
        else
#endif
        if (pairs * 8 >= 7 * kPairs) __builtin_amdgcn_s_setprio(1);
        else if (pairs * 4 >= 3 * kPairs) __builtin_amdgcn_s_setprio(2);
#endif
        path >>= 1;                               // back to X's own index at depth d
        while (d > 0 && (path & 1u)) {            // climb over finished right branches
            path >>= 1;
            --d;
        }
        if (d == 0) break;
        switch (d - 1) {                        // pop the pending right set of depth d
            case 0: DPF_BS_POP_LDS(0, X) tX = tS0; break;
            case 1: DPF_BS_POP_LDS(1, X) tX = tS1; break;
            default: DPF_BS_COPY(X, S2) tX = tS2; break;
        }
        path |= 1u;
    }
#if DPF_BS_FEEDBACK
    if (prog) prog[pslot] = 0xffffffffu;   // done: no longer the slowest
#endif
}

hipError_t launch_unpack_bs(const uint8_t* keys, uint64_t key_len, uint64_t nkeys, uint32_t stop, uint32_t* ekb,
                            hipStream_t st) {
    const uint64_t n = nkeys * ((uint64_t)stop + 1);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_bs, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, keys, key_len, nkeys, stop,
                       ekb);
    return hipGetLastError();
}

bool bs_applicable(uint32_t stop, uint32_t prefix_bits) {
    return stop >= prefix_bits + kBsDMin + 3;   // >= 8 frontier nodes per key below the prefix
}

// Lanes of depth 4 when that fills 2 waves/SIMD on every CU, else depth 3
// (twice the lanes, a frontier one level deeper).
uint32_t bs_depth(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits) {
    if (stop < prefix_bits + kBsDMax + 3) return kBsDMin;
    const uint64_t lanes4 = nkeys << (stop - prefix_bits - kBsDMax - 3);
    return lanes4 >= 131072 ? kBsDMax : kBsDMin;
}

// Sized for the shallower depth (the larger frontier) whatever is picked per launch.
uint64_t bs_frontier_bytes(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits) {
    if (!bs_applicable(stop, prefix_bits)) return 0;
    const uint64_t n = nkeys << (stop - kBsDMin - prefix_bits);
    return (n * 16 + n + 255) & ~255ull;
}

template <int D>
static hipError_t launch_bs_d(const uint4* fs, const uint8_t* fts, uint32_t flog, const uint32_t* ekb, uint32_t stop,
                              uint32_t f, uint64_t nkeys, uint8_t* out, uint64_t out_stride, hipStream_t st) {
    const uint64_t threads = nkeys << (flog - 3);
    const dim3 grid((uint32_t)((threads + kBsBlock - 1) / kBsBlock));
    if (flog - 3 >= 6)
        hipLaunchKernelGGL((k_evalfull_bs<D, true>), grid, dim3(kBsBlock), 0, st, fs, fts, flog, ekb, stop, f, threads,
                           out, out_stride);
    else
        hipLaunchKernelGGL((k_evalfull_bs<D, false>), grid, dim3(kBsBlock), 0, st, fs, fts, flog, ekb, stop, f,
                           threads, out, out_stride);
    return hipGetLastError();
}

hipError_t launch_evalfull_bs(const uint32_t* ek, const uint32_t* ekb, uint64_t nkeys, uint32_t stop,
                              uint32_t prefix_bits, uint64_t prefix, uint8_t* out, uint64_t out_stride, void* frontier,
                              hipStream_t st) {
    if (nkeys == 0) return hipSuccess;
    if (!bs_applicable(stop, prefix_bits)) return hipErrorInvalidValue;
    const uint32_t dd = bs_depth(nkeys, stop, prefix_bits);
    const uint32_t f = stop - dd;                   // frontier level
    const uint32_t flog = f - prefix_bits;          // frontier nodes per key below the prefix
    uint8_t* fs = static_cast<uint8_t*>(frontier);
    uint8_t* fts = fs + (nkeys << flog) * 16;
    hipError_t e = launch_nodes(ek, nkeys, stop, f, prefix_bits, prefix, fs, fts, 1ull << flog, st);
    if (e != hipSuccess) return e;
    const uint4* fsv = reinterpret_cast<const uint4*>(fs);
    return dd == kBsDMax ? launch_bs_d<kBsDMax>(fsv, fts, flog, ekb, stop, f, nkeys, out, out_stride, st)
                         : launch_bs_d<kBsDMin>(fsv, fts, flog, ekb, stop, f, nkeys, out, out_stride, st);
}

// 8 independent blocks per lane through the byte-sliced MMO (AES
// microbenchmark / self-test entry): in/out [n][16] bytes, n % 8 == 0.
__global__ __launch_bounds__(256) void k_mmo_bs(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t nsets,
                                                uint32_t key, uint32_t reps) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nsets) return;
    uint32_t X[32], O[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint4 v = in[u * 8 + i];
        X[i] = v.x; X[8 + i] = v.y; X[16 + i] = v.z; X[24 + i] = v.w;
    }
    transpose32(X);
    for (uint32_t r = 0; r < reps; ++r) {
        aes_mmo8(X, O, key);
        DPF_BS_COPY(X, O)
    }
    transpose32(X);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[u * 8 + i] = make_uint4(X[i], X[8 + i], X[16 + i], X[24 + i]);
}

hipError_t launch_mmo_bs(const uint8_t* in, uint8_t* out, uint64_t nblocks, uint32_t key, uint32_t reps,
                         hipStream_t st) {
    const uint64_t sets = nblocks / 8;
    if (sets == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mmo_bs, dim3((uint32_t)((sets + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), sets, key, reps);
    return hipGetLastError();
}

}  // namespace dpfk
