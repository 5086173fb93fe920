// pir_kernels.hip — XOR-fold of records selected by EvalFull bits on gfx950:
// the 2-server PIR answer (last row: a build-only operator with
// no reference counterpart) and its general-payload form.
//
//   ans_k = XOR over records i with bit_i(EvalFull(key_k)) = 1 of DB[i]
//
// Phase 1 (dpf_kernels.hip, subtree EvalFull) writes each key's selection
// bits into HBM: bits[k][i/32] bit (i%32), which is exactly EvalFull's packed
// LSB-first byte layout (dpf/dpf.go:248-261) read as little-endian u32.
// Phase 2 (here) reads every record once from HBM per launch and folds it
// into all of the launch's answers.  The fold is a GF(2) product and stays
// bitwise (VALU XOR + LDS table lookups); it is not reshaped into an int8
// MFMA GEMM (8x data expansion for the same HBM-bound stream).
//
// Work unit.  A "chunk" is 64 records (one 64-bit word pair of every key's
// selection bits); a record is C 32-byte columns (C = rec_bytes / 32).  A
// chunk is processed as C "sub-steps" of 2 KiB of contiguous DB bytes (64/C
// records x all C columns), loaded by one wave as two coalesced 1 KiB loads:
// lane l holds 16-byte pieces p = l and p = 64 + l.  Records of any other
// multiple of 32 B run as C = 1 over one 32-byte column at a time (rec_u4 /
// col below), one launch per column.
//
// Two kernels, chosen by batch size (launch_pir_fold):
//   k_fold_direct  B <= 16 keys: each lane XORs its pieces into per-key
//                  accumulators under the key's selection bit (selection
//                  words come through scalar loads, uniform per wave).
//                  ~10 VALU per key per 2 KiB: HBM-bound up to 16 keys.
//   k_fold4r       B > 16: Four-Russians.  Per 4-record group and 32-byte
//                  column a 16-entry table (entry e = XOR of the records
//                  whose bit is set in e) is built in LDS once per wave and
//                  looked up by up to 4 x 64 keys (lane = key): 2
//                  ds_read_b128 per key per group instead of 32 masked XORs.
#include <hip/hip_runtime.h>
#include <atomic>
#include <stdint.h>
#include <stdlib.h>

#include "dpf_kernels.hpp"
#include "pir_kernels.hpp"
#include "tree_ops.hpp"

namespace dpfk {

#ifdef DPF_FOLD_TIMES
constexpr uint64_t kFoldTimesMax = 1u << 14;
__device__ uint64_t g_fold_times[4 * kFoldTimesMax];
#endif

// v_bitop3_b32 truth tables: src0 = 0xF0, src1 = 0xCC, src2 = 0xAA.
constexpr uint8_t kTT0 = 0xF0, kTT1 = 0xCC, kTT2 = 0xAA;
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, kTT0 ^ kTT1 ^ kTT2);
}
// a ^ (b & m)
__device__ __forceinline__ uint32_t xam(uint32_t a, uint32_t b, uint32_t m) {
    return __builtin_amdgcn_bitop3_b32(a, b, m, kTT0 ^ (kTT1 & kTT2));
}
__device__ __forceinline__ uint4 x4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }
__device__ __forceinline__ uint4 x4am(uint4 a, uint4 b, uint32_t m) {
    return make_uint4(xam(a.x, b.x, m), xam(a.y, b.y, m), xam(a.z, b.z, m), xam(a.w, b.w, m));
}
// The first fold launch of a call clears the answers (instead of a separate
// memset launch); k_xor_parts runs after it in stream order.
__device__ __forceinline__ void zero_answers(uint32_t* zero, uint64_t words) {
    if (zero == nullptr) return;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < words; t += (uint64_t)gridDim.x * blockDim.x)
        zero[t] = 0;
}
// Issue priority by progress (as the tree kernels' prio_step): a SIMD's
// waves issue oldest-first, so without it the oldest workgroup on a CU
// finishes first and the youngest runs alone at the end.  Priority 3 until
// 3/4 of the wave's range, then 2, 1 at 7/8, 0 at 15/16.
__device__ __forceinline__ void fold_prio(uint64_t done, uint64_t all) {
#if DPF_FOLD_PRIO
    const uint64_t x = done * 16;
    if (x >= 15 * all) __builtin_amdgcn_s_setprio(0);
    else if (x >= 14 * all) __builtin_amdgcn_s_setprio(1);
    else if (x >= 12 * all) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
#else
    (void)done;
    (void)all;
#endif
}
// Workgroup barrier of the folds' LDS staging.  DPF_FOLD_RAW_BARRIER=1 fences
// the local address space only (lgkmcnt) around s_barrier, so a global
// prefetch issued before the barrier cannot be forced to land by it.  r05
// measured it against __syncthreads(): identical (fold B=64 134.3 vs 134.3 us,
// B=256 417 vs 416 us, PIR W=8 step 0.0765 vs 0.0765 ms;
// profiles/r05/fold_barrier) -- the compiler already keeps the prefetch in
// flight across __syncthreads -- so the default is the plain barrier.
#ifndef DPF_FOLD_RAW_BARRIER
#define DPF_FOLD_RAW_BARRIER 0
#endif
__device__ __forceinline__ void lds_barrier() {
#if DPF_FOLD_RAW_BARRIER
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#else
    __syncthreads();
#endif
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Piece p (0..127) of sub-step q of chunk cc, as a 16-byte index into the DB.
// C > 1: contiguous records; C == 1: record stride rec_u4, column col (any
// record width that is a multiple of 32 B).  Indices past the end are
// clamped to the last record (its selection bit is masked off).
template <int C>
__device__ __forceinline__ uint64_t piece_index(uint64_t cc, uint32_t q, uint32_t p, uint64_t nrec, uint64_t rec_u4,
                                                uint32_t col) {
    if constexpr (C == 1) {
        uint64_t r = cc * 64 + (p >> 1);
        if (r >= nrec) r = nrec - 1;
        return r * rec_u4 + 2 * col + (p & 1);
    } else {
        const uint64_t last = nrec * 2 * C - 1;
        const uint64_t i = (cc * C + q) * 128 + p;
        return i < last ? i : last;
    }
}

// Bits of chunk cc's records below nrec, for word 0 (records 0..31) and 1;
// none when the chunk is not the caller's (live = false).  Arithmetic, not
// branches: a branch here splits the lookup block and the register
// allocator then spills the table reads around it.
__device__ __forceinline__ uint2 valid_mask(uint64_t cc, uint64_t nrec, bool live = true) {
    uint64_t v = nrec > cc * 64 ? nrec - cc * 64 : 0;
    v = live ? (v < 64 ? v : 64) : 0;
    const uint32_t lo = v < 32 ? (uint32_t)v : 32u, hi = v > 32 ? (uint32_t)v - 32u : 0u;
    return make_uint2((uint32_t)((1ull << lo) - 1), (uint32_t)((1ull << hi) - 1));
}

// ---------------------------------------------------------------------------
// k_fold_direct<C, KB>: up to KB keys per launch, 4 waves per workgroup, each
// wave takes every 4th chunk of the workgroup's contiguous range.  Lane l
// always holds the same 16-byte position u = l mod 2C of its records, so its
// accumulators are 4 words per key, XOR-reduced across lanes at the end.
#ifndef DPF_WALK_BATCH_FZ
#define DPF_WALK_BATCH_FZ 1   // k_pir_fused block-root walk: batched single-block rounds
#endif
#ifndef DPF_FZ_BATCH
#define DPF_FZ_BATCH 0        // k_pir_fused producers: batched AES rounds (aes2_rounds<BATCH>)
#endif
#ifndef DPF_FZ_NOFOLD
#define DPF_FZ_NOFOLD 0       // measurement only: folders take the ring entries without folding them
#endif
#ifndef DPF_FZ_TOUCH
#define DPF_FZ_TOUCH 1        // k_pir_fused producers touch the next super-group into L2
#endif
#ifndef DPF_FOLD_ABLATE
#define DPF_FOLD_ABLATE 0   // measurement builds of k_fold_mfma: 1 = loads only, 2 = no HBM reads (wrong answers)
#endif
// A streamed 16-byte operand; NT: a nontemporal load (the `nt` cache policy),
// for DB slices too large to stay in the caches between batches (launch_mfma_mt).
typedef uint32_t fold_nt4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 fold_ld(const uint4* p) {
    if constexpr (NT) {
        const fold_nt4 v = __builtin_nontemporal_load(reinterpret_cast<const fold_nt4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
#ifndef DPF_FOLD_GLDS_DEFAULT
#define DPF_FOLD_GLDS_DEFAULT 0   // launch_mfma_mt: LDS-DMA fold shape (fold_glds_mode)
#endif
#ifndef DPF_FOLD_PRIO
#define DPF_FOLD_PRIO 1   // issue priority by progress (fold_prio)
#endif
#ifndef DPF_FOLD_SKEW_DEFAULT
#define DPF_FOLD_SKEW_DEFAULT 62   // percent of a CU's chunk pair for its first k_fold4r workgroup (launch_4r)
#endif
#ifndef DPF_FOLD_PIPE
#define DPF_FOLD_PIPE 1   // table pairs in flight per wave in k_fold4r's lookups (2: no gain, fold_bench r03)
#endif
constexpr int kDWaves = 4;
constexpr int kDirectMaxKeys = 16;

template <int C, int KB>
__global__ __launch_bounds__(64 * kDWaves) void k_fold_direct(const uint32_t* __restrict__ bits, uint64_t wpk,
                                                             const uint4* __restrict__ db, uint64_t nrec,
                                                             uint64_t rec_u4, uint32_t col, uint32_t nkeys,
                                                             uint64_t chunks_per_block, uint32_t* __restrict__ parts,
                                                             uint32_t* __restrict__ zero, uint64_t zero_words) {
    zero_answers(zero, zero_words);
    __shared__ uint32_t s_comb[kDWaves][KB][2 * C][4];
    const uint32_t l = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunks = (nrec + 63) / 64;
    const uint64_t c0 = (uint64_t)blockIdx.x * chunks_per_block;
    const uint64_t cend = c0 + chunks_per_block < nchunks ? c0 + chunks_per_block : nchunks;
    uint32_t acc[KB][4];
#pragma unroll
    for (int k = 0; k < KB; ++k) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0;
    // Record (within the chunk) of sub-step q's pieces l (A) and 64 + l (B).
    const uint32_t rA0 = l / (2 * C);
    // Selection words travel like the pieces: lane l loads key (l mod KB)'s
    // word pair of a chunk together with the chunk's first sub-step (vector
    // loads, one chunk ahead), and v_readlane hands each key's pair to the
    // wave as scalars.  (Per-key scalar loads were each waited on where used.)
    const uint32_t skey = (l % KB) < nkeys ? (l % KB) : 0;
    auto load = [&](uint64_t cc, uint32_t q, uint4& A, uint4& B, uint2& S) __attribute__((always_inline)) {
        A = db[piece_index<C>(cc, q, l, nrec, rec_u4, col)];
        B = db[piece_index<C>(cc, q, 64 + l, nrec, rec_u4, col)];
        if (q == 0) {
            const uint64_t cs = cc < nchunks ? cc : nchunks - 1;
            S = *reinterpret_cast<const uint2*>(bits + skey * wpk + 2 * cs);
        }
    };
    // Items (chunk, sub-step) in pairs of chunks: 2C items, so the two load
    // buffers alternate by item parity and the next item's pieces are in
    // flight while this one is folded.  Every step issues its loads and XORs
    // unconditionally (indices clamped, selection bits masked): a branch
    // around a prefetch makes the compiler drain every load (s_waitcnt
    // vmcnt(0)) at the join.
    uint4 A0, B0, A1, B1;
    uint2 S0 = make_uint2(0, 0), S1 = make_uint2(0, 0);
    load(c0 + w, 0, A0, B0, S0);
    uint2 sel[KB];
    auto step = [&](uint64_t cp, int i, const uint4& A, const uint4& B, const uint2& S, uint4& NA, uint4& NB,
                    uint2& NS) __attribute__((always_inline)) {
        const uint64_t cc = cp + (uint64_t)(i / C) * kDWaves;
        const uint32_t q = (uint32_t)(i % C);
        const uint64_t nc = i + 1 < 2 * C ? cp + (uint64_t)((i + 1) / C) * kDWaves : cp + 2 * kDWaves;
        const uint32_t nq = i + 1 < 2 * C ? (uint32_t)((i + 1) % C) : 0;
        if (q == 0) {
            const uint2 vm = valid_mask(cc, nrec, cc < cend);
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const bool live = (uint32_t)k < nkeys;
                const uint32_t sx = __builtin_amdgcn_readlane(S.x, k), sy = __builtin_amdgcn_readlane(S.y, k);
                sel[k] = make_uint2(live ? sx & vm.x : 0u, live ? sy & vm.y : 0u);
            }
        }
        load(nc, nq, NA, NB, NS);
        // Records of A and B: 64q/C + rA0 and that + 32/C.  For C = 1 they are
        // in words 0 and 1; for C >= 2 both are in word 2q/C.
        const uint32_t rA = (64 * q) / C + rA0, rB = rA + 32 / C;
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            const uint32_t wA = C == 1 ? sel[k].x : ((2 * q) / C ? sel[k].y : sel[k].x);
            const uint32_t wB = C == 1 ? sel[k].y : wA;
            const uint32_t mA = 0u - ((wA >> (rA & 31)) & 1u);
            const uint32_t mB = 0u - ((wB >> (rB & 31)) & 1u);
            acc[k][0] = xam(xam(acc[k][0], A.x, mA), B.x, mB);
            acc[k][1] = xam(xam(acc[k][1], A.y, mA), B.y, mB);
            acc[k][2] = xam(xam(acc[k][2], A.z, mA), B.z, mB);
            acc[k][3] = xam(xam(acc[k][3], A.w, mA), B.w, mB);
        }
    };
    for (uint64_t cp = c0 + w; cp < cend; cp += 2 * kDWaves) {
        fold_prio(cp - c0, cend - c0);
#pragma unroll
        for (int i = 0; i < 2 * C; i += 2) {
            step(cp, i, A0, B0, S0, A1, B1, S1);
            step(cp, i + 1, A1, B1, S1, A0, B0, S0);
        }
    }
    // Lanes with the same position u = l mod 2C hold partial XORs of the same words.
#pragma unroll
    for (int k = 0; k < KB; ++k) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t v = acc[k][d];
#pragma unroll
            for (int off = 2 * C; off < 64; off *= 2) v ^= (uint32_t)__shfl_xor((int)v, off, 64);
            acc[k][d] = v;
        }
    }
    if (l < 2 * C) {
#pragma unroll
        for (int k = 0; k < KB; ++k)
#pragma unroll
            for (int d = 0; d < 4; ++d) s_comb[w][k][l][d] = acc[k][d];
    }
    __syncthreads();
    // parts[block][key][8C words]; word 4u + d of a key's answer is position u, dword d.
    constexpr uint32_t words = (uint32_t)KB * 8 * C;
    for (uint32_t t = threadIdx.x; t < words; t += blockDim.x) {
        const uint32_t k = t / (8 * C), u = (t / 4) % (2 * C), d = t % 4;
        uint32_t v = 0;
#pragma unroll
        for (int ww = 0; ww < kDWaves; ++ww) v ^= s_comb[ww][k][u][d];
        parts[(uint64_t)blockIdx.x * words + t] = v;
    }
}

// ---------------------------------------------------------------------------
// k_fold4r<C, KW, WV>: Four-Russians over 64*KW keys (lane l = keys l, 64+l,
// ...), WV waves per workgroup.  Per sub-step the wave owns 16 tables (4-record
// group gs x column cl, t = gs*C + cl), each two 256-byte rows (half h of the
// 32-byte column) of 16 slots:
//   stage : the loaded pieces go straight to their single-record slots
//           (entries 1, 2, 4, 8); entry 0 is a zero written once;
//   build : lanes 4t .. 4t+3 (h = l&1, a = (l>>1)&1) read the row's 4 records
//           and write the other 11 entries, 6 stores per lane;
//   lookup: each key-lane takes the group's 4 selection bits -- a nibble of
//           EvalFull's LSB-first layout -- as the entry index and XORs the
//           32-byte entry (2 ds_read_b128) into column cl's accumulator.
// Slot of entry e in row (t, h): f(e) ^ sw(t, h), f linear with f(8) = 11,
// sw = 2[t&1] ^ 1[t&2] ^ 4h (searched exhaustively): every staging store,
// build read and build store is conflict-free in its lane groups (8-lane
// groups over 32 banks for ds_write_b128, the 16-lane groups of ds_read_b128
// over 64 banks), lookups read one row and f is a bijection.
// The build is amortised over all 64*KW keys, so a B = 256 batch reads the DB
// once with 1/4 of the per-key table work of B = 64.

__host__ __device__ constexpr uint32_t f_slot(uint32_t e) { return e ^ (((e >> 3) & 1u) * 3u); }
__host__ __device__ constexpr uint32_t sw_row(uint32_t t, uint32_t h) {
    return ((t & 1u) ? 2u : 0u) ^ ((t & 2u) ? 1u : 0u) ^ (h ? 4u : 0u);
}

template <int WV>
struct Fold4rCfg {
    static constexpr int batch = 2 * WV;          // chunks per selection batch: 16*WV bytes of a key's bits
    static constexpr int sel_row = 4 * WV + 2;    // words per staged row (+2 pad: conflict-free ds_read_b64)
};

template <int C, int KW, int WV>
__global__ __launch_bounds__(64 * WV, WV == 8 ? 4 : 3) void k_fold4r(const uint32_t* __restrict__ bits, uint64_t wpk,
                                                                    const uint4* __restrict__ db, uint64_t nrec,
                                                                    uint64_t rec_u4, uint32_t col, uint32_t nkeys,
                                                                    uint64_t chunks_per_block,
                                                                    uint32_t* __restrict__ parts,
                                                                    uint32_t* __restrict__ zero, uint64_t zero_words,
                                                                    uint32_t nfirst, uint64_t cpb_first) {
    zero_answers(zero, zero_words);
    using Cfg = Fold4rCfg<WV>;
    __shared__ uint4 s_tab[WV][32 * 16];                                   // 8 KiB per wave
    __shared__ __attribute__((aligned(16))) uint32_t s_sel[KW * 64 * Cfg::sel_row];
    const uint32_t l = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunks = (nrec + 63) / 64;
    // The first nfirst workgroups (dispatched first: one per CU) take
    // cpb_first chunks, the rest chunks_per_block (fold_split below).
    const uint64_t b = blockIdx.x;
    const uint64_t c0 = b < nfirst ? b * cpb_first : nfirst * cpb_first + (b - nfirst) * chunks_per_block;
    const uint64_t my = b < nfirst ? cpb_first : chunks_per_block;
    const uint64_t cend = c0 + my < nchunks ? c0 + my : nchunks;
    uint4* tab = s_tab[w];
#ifdef DPF_FOLD_TIMES
    const uint64_t t_start = wall_clock64();
#endif

    // Entry 0 of every row: a zero slot, written once.
    if (l < 32) tab[l * 16 + sw_row(l >> 1, l & 1)] = make_uint4(0, 0, 0, 0);
    // Staging slots of this lane's pieces p = l (A) and 64 + l (B, table + 8).
    const uint32_t pr = l / (2 * C), pcl = (l / 2) % C, ph = l & 1;
    const uint32_t pt = (pr >> 2) * C + pcl, pi = pr & 3;
    const uint32_t stA = (2 * pt + ph) * 16 + (f_slot(1u << pi) ^ sw_row(pt, ph));
    const uint32_t stB = stA + 16 * 16;
    // Build role: row (bt, bh), lane pair a.
    const uint32_t bt = l >> 2, bh = l & 1, ba = (l >> 1) & 1;
    uint4* brow = tab + (2 * bt + bh) * 16;
    const uint32_t bsw = sw_row(bt, bh);
    const uint32_t m0 = ba ? 0u : ~0u;

    // Selection staging: thread t copies 16 B of key (kg*64 + t/WV)'s line.
    const uint32_t sk = threadIdx.x / WV, sp = threadIdx.x % WV;
    auto load_sel = [&](int kg, uint64_t cb) __attribute__((always_inline)) {
        const uint32_t key = (uint32_t)kg * 64 + sk;
        const uint32_t* srow = bits + (uint64_t)(key < nkeys ? key : 0) * wpk;
        const uint64_t wo = cb * 2 + 4 * sp;                         // clamped, then zeroed: no branch
        const uint4 v = *reinterpret_cast<const uint4*>(srow + (wo + 4 <= wpk ? wo : wpk - 4));
        return wo + 4 <= wpk ? v : make_uint4(0, 0, 0, 0);
    };
    uint32_t keymask[KW];
#pragma unroll
    for (int kg = 0; kg < KW; ++kg) keymask[kg] = (uint32_t)kg * 64 + l < nkeys ? ~0u : 0u;

    uint32_t acc[KW][C][8];
#pragma unroll
    for (int kg = 0; kg < KW; ++kg)
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[kg][c][i] = 0;

    auto fold = [&](uint64_t cc, uint32_t q, uint64_t cb, const uint4& A, const uint4& B) __attribute__((always_inline)) {
        // stage
        tab[stA] = A;
        tab[stB] = B;
        wave_sync();
        // build: R_i = record i of this row's group
        const uint4 R0 = brow[f_slot(1) ^ bsw], R1 = brow[f_slot(2) ^ bsw];
        const uint4 R2 = brow[f_slot(4) ^ bsw], R3 = brow[f_slot(8) ^ bsw];
        const uint4 R12 = x4(R1, R2), R13 = x4(R1, R3), R23 = x4(R2, R3), R123 = x4(R12, R3);
        // a = 0 writes 7, 11, 13, 15, 3, 5; a = 1 writes 6, 10, 12, 14, 9.
        brow[f_slot(7 ^ ba) ^ bsw] = x4am(R12, R0, m0);
        brow[f_slot(11 ^ ba) ^ bsw] = x4am(R13, R0, m0);
        brow[f_slot(13 ^ ba) ^ bsw] = x4am(R23, R0, m0);
        brow[f_slot(15 ^ ba) ^ bsw] = x4am(R123, R0, m0);
        const uint4 S = ba ? R3 : R1;
        brow[f_slot(ba ? 9 : 3) ^ bsw] = x4(R0, S);
        if (!ba) brow[f_slot(5) ^ bsw] = x4(R0, R2);
        wave_sync();
        // lookups
        const uint32_t j = (uint32_t)(cc - cb);
        const uint2 vm = valid_mask(cc, nrec);
#pragma unroll
        for (int kg = 0; kg < KW; ++kg) {
            // One lane group at a time: interleaving their reads only spills.
            if (kg) __builtin_amdgcn_sched_barrier(0);
            uint2 sel = *reinterpret_cast<const uint2*>(&s_sel[(kg * 64 + l) * Cfg::sel_row + 2 * j]);
            sel.x &= vm.x & keymask[kg];
            sel.y &= vm.y & keymask[kg];
            // Nibbles n of this sub-step: n = q*16/C + gs, gs < 16/C (word n >> 3).
            // Pre-swizzle: f applied to every nibble.
            auto fz = [](uint32_t z) __attribute__((always_inline)) {
                const uint32_t m = (z >> 3) & 0x11111111u;
                return z ^ m ^ (m << 1);
            };
            const uint32_t z0 = fz(sel.x), z1 = fz(sel.y);
            // Tables t and t + C share column cl: one 3-input XOR per word for
            // both (the bitop3 builtin also keeps the compiler from
            // re-associating the chain).  The 8 pairs are software-pipelined:
            // pair p + kPipe's 4 reads are issued before pair p's XORs, with
            // scheduling fences so the compiler keeps that order (left alone,
            // it reads one pair, waits, XORs: 4 reads in flight per wave).
            auto slot = [&](uint32_t t) __attribute__((always_inline)) {
                const uint32_t n = q * (16 / C) + t / C;
                const uint32_t z = (n >> 3) ? z1 : z0;
                return (z >> (4 * (n & 7))) & 15u;
            };
            // Two pairs in flight where the registers allow (measured: no spills).
            constexpr int kPairs = 8;
            constexpr int kPipe = (KW * C >= 8 && C < 8) || (WV == 8 && C >= 4) ? 1 : DPF_FOLD_PIPE;
            uint4 rd[kPairs][4];
            auto pair_t0 = [](int pi) { return (pi / C) * 2 * C + pi % C; };   // pair pi = tables (t0, t0 + C)
            auto issue = [&](int pi) __attribute__((always_inline)) {
                const uint32_t t0 = pair_t0(pi), t1 = t0 + C;
                const uint32_t e0 = slot(t0), e1 = slot(t1);
                rd[pi][0] = tab[(2 * t0) * 16 + (e0 ^ sw_row(t0, 0))];
                rd[pi][1] = tab[(2 * t0 + 1) * 16 + (e0 ^ sw_row(t0, 1))];
                rd[pi][2] = tab[(2 * t1) * 16 + (e1 ^ sw_row(t1, 0))];
                rd[pi][3] = tab[(2 * t1 + 1) * 16 + (e1 ^ sw_row(t1, 1))];
            };
#pragma unroll
            for (int pi = 0; pi < kPipe; ++pi) issue(pi);
#pragma unroll
            for (int pi = 0; pi < kPairs; ++pi) {
                if (pi + kPipe < kPairs) issue(pi + kPipe);
                __builtin_amdgcn_sched_barrier(0);
                const uint4 lo0 = rd[pi][0], hi0 = rd[pi][1], lo1 = rd[pi][2], hi1 = rd[pi][3];
                uint32_t* a = acc[kg][pair_t0(pi) % C];
                a[0] = x3(a[0], lo0.x, lo1.x); a[1] = x3(a[1], lo0.y, lo1.y);
                a[2] = x3(a[2], lo0.z, lo1.z); a[3] = x3(a[3], lo0.w, lo1.w);
                a[4] = x3(a[4], hi0.x, hi1.x); a[5] = x3(a[5], hi0.y, hi1.y);
                a[6] = x3(a[6], hi0.z, hi1.z); a[7] = x3(a[7], hi0.w, hi1.w);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        wave_sync();
    };

    // Batches of Cfg::batch chunks (one 16*WV-byte piece of every key's bits);
    // each wave takes chunks cb + w and cb + WV + w of a batch, C sub-steps
    // each.  Loads ping-pong between two buffers (2C items per batch, even),
    // so the next sub-step's records are in flight during a fold.
    auto load = [&](uint64_t cc, uint32_t q, uint4& A, uint4& B) __attribute__((always_inline)) {
        A = db[piece_index<C>(cc, q, l, nrec, rec_u4, col)];
        B = db[piece_index<C>(cc, q, 64 + l, nrec, rec_u4, col)];
    };
    uint4 A0, B0, A1, B1;
    load(c0 + w, 0, A0, B0);
    uint4 snext[KW];
#pragma unroll
    for (int kg = 0; kg < KW; ++kg) snext[kg] = load_sel(kg, c0);
    auto step = [&](uint64_t cb, int i, const uint4& A, const uint4& B, uint4& NA, uint4& NB) __attribute__((always_inline)) {
        const uint64_t cc = cb + w + (uint64_t)(i / C) * WV;
        const uint32_t q = (uint32_t)(i % C);
        const uint64_t nc = i + 1 < 2 * C ? cb + w + (uint64_t)((i + 1) / C) * WV : cb + Cfg::batch + w;
        const uint32_t nq = i + 1 < 2 * C ? (uint32_t)((i + 1) % C) : 0;
        load(nc, nq, NA, NB);            // unconditional (clamped): see k_fold_direct
        if (cc < cend) fold(cc, q, cb, A, B);
    };
    for (uint64_t cb = c0; cb < cend; cb += Cfg::batch) {
        fold_prio(cb - c0, cend - c0);
        lds_barrier();                                     // previous batch's selection reads are done
#pragma unroll
        for (int kg = 0; kg < KW; ++kg) {
            uint32_t* row = &s_sel[(kg * 64 + sk) * Cfg::sel_row + 4 * sp];
            *reinterpret_cast<uint2*>(row) = make_uint2(snext[kg].x, snext[kg].y);
            *reinterpret_cast<uint2*>(row + 2) = make_uint2(snext[kg].z, snext[kg].w);
        }
        lds_barrier();
#pragma unroll
        for (int kg = 0; kg < KW; ++kg) snext[kg] = load_sel(kg, cb + Cfg::batch);
#pragma unroll
        for (int i = 0; i < 2 * C; i += 2) {
            step(cb, i, A0, B0, A1, B1);
            step(cb, i + 1, A1, B1, A0, B0);
        }
    }
#ifdef DPF_FOLD_TIMES
    // Measurement build only (tools/fold_bench.hip -DDPF_FOLD_TIMES): per
    // wave, start / end of its chunk loop and the CU it ran on.
    if (l == 0) {
        const uint64_t wv = (uint64_t)blockIdx.x * WV + w;
        if (wv < kFoldTimesMax) {
            g_fold_times[4 * wv] = t_start;
            g_fold_times[4 * wv + 1] = wall_clock64();
            g_fold_times[4 * wv + 2] = __builtin_amdgcn_s_getreg(0xF804);   // HW_ID
            g_fold_times[4 * wv + 3] = __builtin_amdgcn_s_getreg(0xF814);   // XCC_ID
        }
    }
#endif
    // Combine the workgroup's waves in LDS (reusing the tables), one
    // 8-word slice (key group, column) at a time: parts[block][key][8C words].
    constexpr uint32_t pkeys = 64 * KW, pwords = 8 * C;
    uint32_t* comb = reinterpret_cast<uint32_t*>(&s_tab[0][0]);     // [wave][lane][8]
#pragma unroll
    for (int kg = 0; kg < KW; ++kg)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 8; ++i) comb[(w * 64 + l) * 8 + i] = acc[kg][c][i];
            __syncthreads();
            for (uint32_t t = threadIdx.x; t < 64 * 8; t += blockDim.x) {
                uint32_t v = 0;
#pragma unroll
                for (int ww = 0; ww < WV; ++ww) v ^= comb[ww * 64 * 8 + t];
                const uint32_t key = kg * 64 + t / 8;
                parts[((uint64_t)blockIdx.x * pkeys + key) * pwords + c * 8 + (t % 8)] = v;
            }
        }
}

// ans[k * ans_words + off + i] ^= XOR over workgroups p of parts[p][k][i]
// (k < nkeys, i < pwords; pkeys keys per part).  Block (x, y): 256 words x
// parts y, y + gridDim.y, ...; one atomicXor each.
__global__ __launch_bounds__(256) void k_xor_parts(const uint32_t* __restrict__ parts, uint64_t nparts, uint32_t nkeys,
                                                   uint32_t pkeys, uint32_t pwords, uint32_t* __restrict__ ans,
                                                   uint64_t ans_words, uint32_t off) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nkeys * pwords) return;
    const uint32_t k = t / pwords, i = t % pwords;
    uint32_t v = 0;
    // Eight independent loads in flight per step (a strided loop of single
    // loads left the kernel at ~5 us, mostly dependent L2 round trips).
    const uint64_t g = gridDim.y;
    uint64_t p = blockIdx.y;
    for (; p + 7 * g < nparts; p += 8 * g) {
        uint32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = parts[((p + u * g) * pkeys + k) * pwords + i];
#pragma unroll
        for (int u = 0; u < 8; ++u) v ^= x[u];
    }
    for (; p < nparts; p += g) v ^= parts[(p * pkeys + k) * pwords + i];
    if (v) atomicXor(ans + (uint64_t)k * ans_words + off + i, v);
}

// XOR nparts workgroup partials into the answers (stream-ordered after the fold).
static hipError_t launch_xor_parts(const uint32_t* parts, uint64_t nparts, uint32_t nkeys, uint32_t pkeys,
                                   uint32_t pwords, uint32_t* ans, uint64_t ans_words, uint32_t off, hipStream_t st) {
    // Part slices per answer word, one atomic each: 16 for <= 256 partials
    // (the PIR rank at N = 8: step 0.0733-0.0737 vs 0.0740-0.0745 ms with 64,
    // 8 in between), 64 above (one GPU, 768 partials: 0.3799-0.3802 vs
    // 0.3811-0.3817 with 16); tools/archive/r05_xys.sh, profiles/r05/xor_parts/.
    // DPF_XOR_PARTS_YS=<n> (measurement only) fixes it.
    static const uint64_t yenv = [] {
        const char* e = getenv("DPF_XOR_PARTS_YS");
        return e && atoi(e) > 0 ? (uint64_t)atoi(e) : 0ull;
    }();
    const uint64_t ymax = yenv ? yenv : nparts <= 256 ? 16 : 64;
    const uint32_t ys = (uint32_t)(nparts < ymax ? nparts : ymax);
    hipLaunchKernelGGL(k_xor_parts, dim3((nkeys * pwords + 255) / 256, ys), dim3(256), 0, st, parts, nparts, nkeys,
                       pkeys, pwords, ans, ans_words, off);
    return hipGetLastError();
}

static int cu_count_fold() { return cu_count(); }   // the calling thread's CU budget (dpf_kernels.hip)

constexpr uint64_t kFoldMaxBlocks = 1024;          // workgroups per launch (partials area)
constexpr uint64_t kFoldPartBytes = 64 * 4 * 32 * 2;   // largest part: 64*KW keys x 32C bytes, KW*C <= 8
constexpr uint32_t kFoldMaxSgPerBlock = 1u << 15; // k_fold_mfma: super-groups per workgroup (fp32-exact counts)

uint64_t pir_fold_parts_bytes() { return kFoldMaxBlocks * kFoldPartBytes; }

// Tuning / test limits (set_fold_limits): workgroups per fold launch and
// super-groups per matrix-core fold workgroup.
static std::atomic<uint32_t> g_fold_blocks{(uint32_t)kFoldMaxBlocks};
static std::atomic<uint32_t> g_fold_max_sg{kFoldMaxSgPerBlock};
static uint32_t fold_max_sg() { return g_fold_max_sg.load(std::memory_order_relaxed); }
void set_fold_limits(uint32_t max_blocks, uint32_t max_sg) {
    g_fold_blocks.store(max_blocks == 0 || max_blocks > kFoldMaxBlocks ? (uint32_t)kFoldMaxBlocks : max_blocks);
    g_fold_max_sg.store(max_sg == 0 || max_sg > kFoldMaxSgPerBlock ? kFoldMaxSgPerBlock : max_sg);
}

namespace {

// Split nchunks into `blocks` contiguous ranges of whole `gran`-chunk batches.
// cap_in: the workgroup cap the caller sized its passes with (0: read it
// here); a launcher that derives a per-workgroup bound from the cap must pass
// the value it read, so a concurrent dpf_set_fold_limits cannot change it
// between the two reads.
void split_chunks(uint64_t nchunks, uint64_t want_blocks, uint64_t gran, uint64_t& blocks, uint64_t& cpb,
                  uint64_t cap_in = 0) {
    const uint64_t cap = cap_in ? cap_in : g_fold_blocks.load(std::memory_order_relaxed);
    if (want_blocks > cap) want_blocks = cap;
    cpb = (nchunks + want_blocks - 1) / want_blocks;
    cpb = (cpb + gran - 1) / gran * gran;
    blocks = (nchunks + cpb - 1) / cpb;
}

struct FoldArgs {
    const uint32_t* bits;
    uint64_t wpk;
    const uint4* db;
    uint64_t nrec, rec_u4;
    uint32_t col, nkeys;
    uint32_t* parts;
    uint32_t* zero;          // first pass: the answers, cleared before k_xor_parts XORs into them
    uint64_t zero_words;
};

template <int C, int KB>
hipError_t launch_direct_kb(const FoldArgs& a, uint64_t nchunks, uint64_t& blocks, hipStream_t st) {
    uint64_t cpb;
    split_chunks(nchunks, (uint64_t)cu_count_fold() * 4, 2 * kDWaves, blocks, cpb);
    hipLaunchKernelGGL((k_fold_direct<C, KB>), dim3((uint32_t)blocks), dim3(64 * kDWaves), 0, st, a.bits, a.wpk, a.db,
                       a.nrec, a.rec_u4, a.col, a.nkeys, cpb, a.parts, a.zero, a.zero_words);
    return hipGetLastError();
}

// The direct kernel's work is linear in its key slots: 1, 4 or 16 by batch.
template <int C>
hipError_t launch_direct(const FoldArgs& a, uint64_t nchunks, uint64_t& blocks, uint32_t& pkeys, hipStream_t st) {
    if (a.nkeys <= 1) return pkeys = 1, launch_direct_kb<C, 1>(a, nchunks, blocks, st);
    if (a.nkeys <= 4) return pkeys = 4, launch_direct_kb<C, 4>(a, nchunks, blocks, st);
    return pkeys = kDirectMaxKeys, launch_direct_kb<C, kDirectMaxKeys>(a, nchunks, blocks, st);
}

template <int C, int KW>
hipError_t launch_4r(const FoldArgs& a, uint64_t nchunks, uint64_t& blocks, hipStream_t st) {
    // KW = 1, C < 8: 8 waves, 72 KiB of LDS -> 2 workgroups (16 waves, 128
    // VGPRs) per CU.  Otherwise 4 waves, 41-50 KiB -> 3 per CU (168 VGPRs:
    // 64 accumulators per lane).
    constexpr int WV = KW == 1 && C < 8 ? 8 : 4;
    const uint64_t cus = (uint64_t)cu_count_fold();
    const uint64_t per_cu = WV == 8 ? 2 : 3;
    uint64_t cpb;
    split_chunks(nchunks, cus * per_cu, 2 * WV, blocks, cpb);
    // Two workgroups per CU: a SIMD's waves issue oldest-first, so the CU's
    // first workgroup runs ahead of its second (fold per-wave times: 100 vs
    // 143 us at configs[4]).  DPF_FOLD_SKEW (percent of a CU pair's chunks
    // for the first workgroup) shifts work to it.
    static const int skew = [] {
        const char* e = getenv("DPF_FOLD_SKEW");
        return e ? atoi(e) : DPF_FOLD_SKEW_DEFAULT;
    }();
    uint32_t nfirst = 0;
    uint64_t cpb_first = cpb;
    const uint64_t gran = 2 * WV;
    if (per_cu == 2 && skew > 50 && skew < 100 && blocks == 2 * cus) {
        const uint64_t pair = 2 * cpb;
        cpb_first = (pair * (uint64_t)skew / 100 + gran / 2) / gran * gran;
        const uint64_t rest = pair - cpb_first;
        if (rest >= gran && nchunks <= cus * pair) {
            nfirst = (uint32_t)cus;
            cpb = rest;
        } else {
            cpb_first = cpb;
        }
    }
    hipLaunchKernelGGL((k_fold4r<C, KW, WV>), dim3((uint32_t)blocks), dim3(64 * WV), 0, st, a.bits, a.wpk, a.db,
                       a.nrec, a.rec_u4, a.col, a.nkeys, cpb, a.parts, a.zero, a.zero_words, nfirst, cpb_first);
    return hipGetLastError();
}

// One pass over the DB for `a.nkeys` keys (<= 64*KW or <= 16 direct) with C
// columns per record: fold kernel, then k_xor_parts into ans.
template <int C>
hipError_t fold_pass(const FoldArgs& a, bool direct, int kw, uint32_t* ans, uint64_t ans_words, uint32_t off,
                     hipStream_t st) {
    const uint64_t nchunks = (a.nrec + 63) / 64;
    uint64_t blocks = 0;
    uint32_t pkeys;
    hipError_t e;
    if (direct) {
        e = launch_direct<C>(a, nchunks, blocks, pkeys, st);
    } else if (kw >= 4) {
        if constexpr (C <= 2) e = launch_4r<C, 4>(a, nchunks, blocks, st);
        else return hipErrorInvalidValue;
        pkeys = 256;
    } else if (kw == 2) {
        if constexpr (C <= 4) e = launch_4r<C, 2>(a, nchunks, blocks, st);
        else return hipErrorInvalidValue;
        pkeys = 128;
    } else {
        e = launch_4r<C, 1>(a, nchunks, blocks, st);
        pkeys = 64;
    }
    if (e != hipSuccess) return e;
    return launch_xor_parts(a.parts, blocks, a.nkeys, pkeys, 8 * C, ans, ans_words, off, st);
}

}  // namespace

// ---------------------------------------------------------------------------
// The fold as a GF(2) matrix product on the matrix cores.
//
//   count[k][n] = sum_i sel[k][i] * dbbit[i][n],   ans bit (k, n) = count & 1
//
// is a {0,1} product of [keys x records] by [records x 256 bit positions], so
// it runs on v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 (FP4) operands: every
// product is exactly 1 or 0, the fp32 accumulators hold exact counts (far
// below 2^24 per wave), and the parity is the answer bit.  No LDS at all.
//
// Operands.  An MFMA operand lane holds 32 K-values (records) of ONE row
// (key) or column (bit position); the K order inside the lane is ours to
// pick as long as A and B agree.  The key side is EvalFull's own layout: one
// selection word = 32 consecutive records of one key.  The DB side needs the
// transposed form -- for bit position n, one word of 32 consecutive records
// -- which the PIR server builds once when the DB is loaded (the "sliced"
// layout, k_slice_db below):
//   dbs[S][n][g] (u32), S = super-group of 256 records, n < 256 bit position,
//   g < 8 record group; bit j = bit n of record 256 S + 32 g + j.
// A lane (n, h) loads dbs[S][n][4h .. 4h+3] and a key lane (k, h) loads
// selection words 8S + 4h .. +3 (one dwordx4 each, both coalesced): K-block
// t < 4 of super-group S is record groups t (h = 0) and 4 + t (h = 1).
// Word -> FP4 operand in registers, nibble i of dword d = record 4i + d:
//   one side  d0 = x & 0x1..  (0.5)  d1 = x & 0x2.. (1.0)  d2 = x & 0x4.. (2.0)
//             d3 = (x >> 1) & 0x4.. (2.0)                       5 VALU per word
//   the other d0 = (s << 2) & 0x4.. (2.0)  d1 = s & 0x2.. (1.0)
//             d2 = (s >> 2) & 0x1.. (0.5)  d3 = (s >> 3) & 0x1.. (0.5)   7 VALU
// so every nonzero product is exactly 1 with unit (E8M0 127) scales.
//
// Mapping.  A wave covers MT key tiles (32 keys) x NT bit tiles (32 bit
// positions) of a contiguous run of super-groups; the 8/NT waves of a
// workgroup split the record's 256 bits and share its selection words (L1).
// At the end each accumulator register's parities become two answer words by
// one ballot (C/D layout: lane = column n, register e = rows (e&3) +
// 8(e>>2) + 4h), written to the workgroup's partial; k_xor_parts combines.
typedef int fold_v8i __attribute__((ext_vector_type(8)));
typedef float fold_v16f __attribute__((ext_vector_type(16)));

// Which side takes the cheap 5-op expansion (ANDs + one shift; weights 0.5,
// 1, 2, 2) and which the 7-op one (weights 2, 1, 0.5, 0.5): a selection
// operand feeds NT MFMAs and a DB operand MT, so per MFMA the VALU cost is
// sel/NT + db/MT, lowest with the cheap form on the side with fewer tiles
// (kernel template below; DPF_FOLD_SEL_CHEAP=0/1 forces one for A/B runs).
#ifndef DPF_FOLD_SEL_CHEAP
#define DPF_FOLD_SEL_CHEAP -1
#endif
__device__ __forceinline__ fold_v8i fp4_w5(uint32_t x) {     // weights 0.5, 1, 2, 2
    fold_v8i r;
    r[0] = (int)(x & 0x11111111u);
    r[1] = (int)(x & 0x22222222u);
    r[2] = (int)(x & 0x44444444u);
    r[3] = (int)((x >> 1) & 0x44444444u);
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}
__device__ __forceinline__ fold_v8i fp4_w7(uint32_t s) {     // weights 2, 1, 0.5, 0.5
    fold_v8i r;
    r[0] = (int)((s << 2) & 0x44444444u);
    r[1] = (int)(s & 0x22222222u);
    r[2] = (int)((s >> 2) & 0x11111111u);
    r[3] = (int)((s >> 3) & 0x11111111u);
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}
template <bool SC>
__device__ __forceinline__ fold_v8i fp4_db(uint32_t x) { return SC ? fp4_w7(x) : fp4_w5(x); }
template <bool SC>
__device__ __forceinline__ fold_v8i fp4_sel(uint32_t s) { return SC ? fp4_w5(s) : fp4_w7(s); }
__device__ __forceinline__ uint32_t u4w(const uint4& v, int t) { return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w; }

constexpr int kFoldFp4 = 4;         // cbsz / blgp format code of e2m1
constexpr int kE8M0One = 127;       // block scale 2^0

// Selection words reach the waves through LDS: per block of SG super-groups
// the workgroup copies each key's SG*32-byte span (coalesced) into a padded
// row, and the next block's selection words and DB pieces are in flight in
// registers while this block is folded (block-level double buffering: a
// super-group of MFMA work is ~0.2-0.4 us per wave, shorter than the HBM
// latency under load).  Loaded straight into the operand lanes, 16 B per
// lane from 32 rows 2 MiB apart, the fold fetched ~1.6x its bytes and ran at
// a third of the HBM rate (profiles/r04/fold_v1).
#ifndef DPF_FOLD_PD
#define DPF_FOLD_PD 1   // staged blocks in flight ahead of the one being folded (1 or 2)
#endif
// KG key groups per workgroup: wave w takes bit slice w % (8/NT) of key
// group w / (8/NT), so a workgroup covers 32*MT*KG keys x 256 bits.
// SGM: the selection bits are super-group-major in chunks of G super-groups,
// sel[S / G][sgm_keys][G * 8 words] (G = sgm_g: 1, or 4 = one 128-byte line
// of a key per chunk, as the PIR tree kernel writes them), so a staged block
// is one contiguous region instead of EvalFull's key-major [key][wpk words].
// Exactness of the fp32 counts: an accumulator gains at most 64 per MFMA
// (one per record of a K-block), and fp32 holds every integer up to 2^24.
// A workgroup's run of super-groups would grow with the DB and shrink with
// the CU count, so launch_mfma_mt never gives one more than
// kFoldMaxSgPerBlock = 2^15 super-groups (2^23 records): it adds workgroups,
// and beyond kFoldMaxBlocks of them it folds the DB in passes, each pass's
// partials XORed into the answers.  (Reducing the counts to parities inside
// the kernel moved the large-tile accumulators out of AGPRs and spilled them:
// 2.5x slower at 256 keys, r05.)  wlim: selection words per key row from
// `bits` (the row stride stays wpk), so a pass can start mid-row.
#ifndef DPF_FOLD_MINB4
#define DPF_FOLD_MINB4 2   // min workgroups per CU the <=4-tile shapes are compiled for (A/B: 4 = <=128 VGPRs)
#endif
template <int MT, int NT, int SG, int KG, int SGM = 0, bool NTDB = false>
__global__ __launch_bounds__(64 * (8 / NT) * KG, (MT * NT <= 4) ? DPF_FOLD_MINB4 : 1) void k_fold_mfma(
    const uint32_t* __restrict__ bits, uint64_t wpk, const uint4* __restrict__ dbs, uint64_t nsg, uint32_t nkeys,
    uint64_t sg_per_block, uint32_t* __restrict__ parts, uint32_t* __restrict__ zero, uint64_t zero_words,
    uint64_t wlim, uint32_t sgm_keys = 0) {
    constexpr int NS = 8 / NT;                                 // bit slices
    constexpr int NW = NS * KG;
    constexpr bool SC = DPF_FOLD_SEL_CHEAP >= 0 ? DPF_FOLD_SEL_CHEAP == 1 : NT < MT;
    constexpr int kRows = 32 * MT * KG;
    constexpr int kRow = SG * 8 + 4;                           // words per staged row (+4: conflict-free b128 reads)
    constexpr int kPieces = kRows * (SG * 2);                  // uint4 pieces per staged block
    constexpr int kPer = (kPieces + 64 * NW - 1) / (64 * NW);  // per thread
    __shared__ __attribute__((aligned(16))) uint32_t s_sel[kRows * kRow];
    zero_answers(zero, zero_words);
    const uint32_t l = threadIdx.x & 63, h = l >> 5, r = l & 31;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t w = wv % NS, kg = wv / NS;                   // bit slice, key group
    const uint64_t s0 = (uint64_t)blockIdx.x * sg_per_block;
    const uint64_t s1 = s0 + sg_per_block < nsg ? s0 + sg_per_block : nsg;
    if (s0 >= s1) return;                                       // uniform over the workgroup
    // Staging role: piece p = threadIdx.x + i*64*NW is row p/(2SG), 16 bytes p%(2SG).
    // Piece p -> (row, q = 16-byte piece of the row's block span): key-major,
    // row = p / 2SG; super-group-major, p = (s * kRows + row) * 2 + half.
    auto piece = [&](uint32_t p, uint32_t& row, uint32_t& q) __attribute__((always_inline)) {
        if constexpr (SGM == 1) {
            row = (p >> 1) % kRows;
            q = 2 * ((p >> 1) / kRows) + (p & 1);
        } else {
            row = p / (2 * SG);
            q = p % (2 * SG);
        }
    };
    auto load_sel = [&](uint64_t sb, uint4 (&v)[kPer]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const uint32_t p = threadIdx.x + (uint32_t)i * 64 * NW;
            uint32_t row, q;
            piece(p, row, q);
            const uint64_t word = sb * 8 + 4 * q;
            const bool ok = p < (uint32_t)kPieces && row < nkeys && word + 4 <= wlim;
            const uint64_t S = sb + q / 2;
            const uint64_t at = SGM ? ((S / SGM * sgm_keys + row) * SGM + S % SGM) * 8 + 4 * (q & 1)
                                    : (uint64_t)row * wpk + word;
#if DPF_FOLD_ABLATE == 2
            const uint32_t z = (uint32_t)at * 2654435761u;      // no HBM read (measurement build)
            const uint4 x = make_uint4(z, z ^ 0x5555u, z + 7u, ~z);
#else
            const uint4 x = *reinterpret_cast<const uint4*>(bits + (ok ? at : 0));
#endif
            v[i] = ok ? x : make_uint4(0, 0, 0, 0);
        }
    };
    auto store_sel = [&](const uint4 (&v)[kPer]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const uint32_t p = threadIdx.x + (uint32_t)i * 64 * NW;
            uint32_t row, q;
            piece(p, row, q);
            if (p < (uint32_t)kPieces) *reinterpret_cast<uint4*>(&s_sel[row * kRow + 4 * q]) = v[i];
        }
    };
    // DB pieces of a whole block (clamped past the range; never folded).
    auto load_db = [&](uint64_t sb, uint4 (&B)[SG][NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int sl = 0; sl < SG; ++sl) {
            const uint64_t S = sb + sl < s1 ? sb + sl : s1 - 1;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
#if DPF_FOLD_ABLATE == 2
                const uint32_t z = (uint32_t)((S * 256 + 32u * (w * NT + j) + r) * 2 + h) * 2246822519u;
                B[sl][j] = make_uint4(z, z + 1u, z ^ 0xAAAAu, ~z);           // no HBM read (measurement build)
#else
                B[sl][j] = fold_ld<NTDB>(&dbs[(S * 256 + 32u * (w * NT + j) + r) * 2 + h]);
#endif
            }
        }
    };
    fold_v16f acc[MT][NT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[m][j][e] = 0.0f;
    // One super-group: 4 K-blocks of 64 records x MT x NT MFMAs.
    auto fold_sg = [&](int sl, const uint4 (&B)[NT]) __attribute__((always_inline)) {
        uint4 A[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m)
            A[m] = *reinterpret_cast<const uint4*>(&s_sel[(32 * (MT * kg + m) + r) * kRow + 8 * sl + 4 * h]);
#if DPF_FOLD_ABLATE == 1
        // Measurement build: the operands are consumed by one XOR each, no
        // FP4 expansion and no MFMA (the load + staging structure alone).
        uint32_t x = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int j = 0; j < NT; ++j) x ^= u4w(B[j], t);
#pragma unroll
            for (int m = 0; m < MT; ++m) x ^= u4w(A[m], t);
        }
        acc[0][0][0] += (float)(x & 1u);
#else
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            fold_v8i bo[NT];
#pragma unroll
            for (int j = 0; j < NT; ++j) bo[j] = fp4_db<SC>(u4w(B[j], t));
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const fold_v8i ao = fp4_sel<SC>(u4w(A[m], t));
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[m][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ao, bo[j], acc[m][j], kFoldFp4, kFoldFp4,
                                                                               0, kE8M0One, 0, kE8M0One);
            }
        }
#endif
    };
#if DPF_FOLD_PD >= 2
    // Two blocks in flight: block i folds from buffer i%3 while blocks i+1
    // and i+2 load (selection words and DB pieces rotate over 3 sets).
    uint4 sv0[kPer], sv1[kPer], sv2[kPer];
    uint4 B0[SG][NT], B1[SG][NT], B2[SG][NT];
    load_sel(s0, sv0);
    load_db(s0, B0);
    load_sel(s0 + SG < s1 ? s0 + SG : s0, sv1);
    load_db(s0 + SG < s1 ? s0 + SG : s0, B1);
    auto block = [&](uint64_t sb, const uint4 (&Bc)[SG][NT], uint4 (&Bf)[SG][NT], const uint4 (&svc)[kPer],
                     uint4 (&svf)[kPer]) __attribute__((always_inline)) {
        fold_prio(sb - s0, s1 - s0);
        lds_barrier();                                          // previous block's operand reads are done
        store_sel(svc);
        lds_barrier();
        const uint64_t nb = sb + 2 * SG < s1 ? sb + 2 * SG : sb;   // block after next (clamped)
        load_sel(nb, svf);
        load_db(nb, Bf);
        const uint64_t n = s1 - sb;
#pragma unroll
        for (int sl = 0; sl < SG; ++sl)
            if ((uint64_t)sl < n) fold_sg(sl, Bc[sl]);
    };
    uint64_t sb = s0;
    for (; sb + 2 * SG < s1; sb += 3 * SG) {
        block(sb, B0, B2, sv0, sv2);
        block(sb + SG, B1, B0, sv1, sv0);
        block(sb + 2 * SG, B2, B1, sv2, sv1);
    }
    if (sb < s1) block(sb, B0, B2, sv0, sv2);
    if (sb + SG < s1) block(sb + SG, B1, B0, sv1, sv0);
#else
    uint4 sv[kPer];
    uint4 BA[SG][NT], BB[SG][NT];
    load_sel(s0, sv);
    load_db(s0, BA);
    // One staged block: its selection rows to LDS, the next block's loads
    // issued, then its super-groups folded.
    auto block = [&](uint64_t sb, const uint4 (&Bc)[SG][NT], uint4 (&Bn)[SG][NT]) __attribute__((always_inline)) {
        fold_prio(sb - s0, s1 - s0);
        lds_barrier();                                          // previous block's operand reads are done
        store_sel(sv);
        lds_barrier();
        const uint64_t nb = sb + SG < s1 ? sb + SG : sb;        // next block (clamped)
        load_sel(nb, sv);
        load_db(nb, Bn);
        const uint64_t n = s1 - sb;
#pragma unroll
        for (int sl = 0; sl < SG; ++sl)
            if ((uint64_t)sl < n) fold_sg(sl, Bc[sl]);
    };
    uint64_t sb = s0;
    for (; sb + SG < s1; sb += 2 * SG) {
        block(sb, BA, BB);
        block(sb + SG, BB, BA);
    }
    if (sb < s1) block(sb, BA, BB);
#endif
    // Parities -> answer words: parts[block][key][8] (word = bit tile).
    constexpr uint32_t pkeys = 32 * MT * KG;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            uint32_t out = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t p = ((uint32_t)acc[m][j][e]) & 1u;
                const uint64_t b = __builtin_amdgcn_ballot_w64(p != 0);
                const uint32_t row0 = (e & 3) + 8 * (e >> 2);
                out = l == row0 ? (uint32_t)b : out;
                out = l == row0 + 4 ? (uint32_t)(b >> 32) : out;
            }
            if (l < 32) parts[((uint64_t)blockIdx.x * pkeys + 32 * (MT * kg + m) + l) * 8 + w * NT + j] = out;
        }
}

#ifndef DPF_FOLD_GLDS_KERNEL
#define DPF_FOLD_GLDS_KERNEL 0   // k_fold_glds: experimental build only (measured slower, r05)
#endif
#if DPF_FOLD_GLDS_KERNEL
// ---------------------------------------------------------------------------
// k_fold_glds: k_fold_mfma with its operands staged by LDS-DMA (r05).
// PMC on k_fold_mfma<2,2,2,1> at configs[4] (profiles/r05/pmc_fold64): MFMA
// busy 43% of cycles, TA busy 61-69%, HBM 5.2 TB/s (0.84 of the measured
// streaming rate), waves waiting on memory 46% of their cycles, 3 waves per
// SIMD: no unit is saturated; the fold is bound by the bytes it keeps in
// flight (one staged block of ~20 KiB per workgroup in VGPRs, ~60 KiB per CU
// against the ~60 KiB that Little's law asks at 6 TB/s and ~2.5 us of loaded
// latency).  Here global_load_lds_dwordx4 moves every operand straight into
// a P-deep ring in LDS (no VGPR cost), so P - 1 blocks stay in flight while
// one is folded; a raw s_barrier plus a counted vmcnt wait per block (never
// vmcnt(0) in the loop) keeps them in flight across the barrier.
//   stage = selection rows [kRows][2 SG x 16 B] (XOR-swizzled pieces:
//           conflict-free ds_read_b128 of a key tile) + each wave's DB
//           pieces [SG][NT][64 lanes x 16 B];
//   every wave issues G = 1 + SG * NT LDS-DMAs per block (its share of the
//   selection rows, then its own DB pieces), so one vmcnt count fits all.
// Blocks past the end are issued with clamped addresses into the stage that
// will not be read again, so the count holds to the last block.
// Only the key-major selection layout (sgm_keys == 0).
template <int MT, int NT, int SG, int KG, int P>
struct GldsShape {
    static constexpr int NS = 8 / NT, NW = NS * KG;
    static constexpr int kRows = 32 * MT * KG;
    static constexpr int PR = 2 * SG;                        // 16-byte pieces per selection row
    static constexpr int kSelPieces = kRows * PR;
    static constexpr int kSelLanes = kSelPieces / NW;        // per wave (one LDS-DMA, <= 64 lanes)
    static constexpr int kDbPieces = NW * SG * NT * 64;
    static constexpr int kStage = kSelPieces + kDbPieces;    // 16-byte slots per stage
    static constexpr int G = 1 + SG * NT;                    // LDS-DMAs per wave per block
    static_assert(kSelPieces % NW == 0 && kSelLanes <= 64, "selection rows: one DMA per wave");
    static_assert(16 % PR == 0, "swizzle: pieces per row divide a bank row");
};
template <int PR>
__device__ __forceinline__ uint32_t sel_slot(uint32_t row, uint32_t q) {
    constexpr uint32_t rpb = 16 / PR;                        // rows per 256-byte bank row
    return row * PR + (q ^ ((row / rpb) & (PR - 1)));
}
// The gfx950-only builtins sit behind the device pass: in the host pass
// clang treats them as invalid in the kernel template's body and silently
// drops the kernel's host stub (undefined symbol at link time).
template <int N>
__device__ __forceinline__ void wait_vm() {                  // s_waitcnt vmcnt(N), nothing else
    static_assert(N >= 0 && N < 64, "vmcnt range");
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
#endif
}
__device__ __forceinline__ void wait_lgkm0() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_waitcnt((15) | (3 << 14) | (7 << 4) | (0 << 8));
#endif
}
// ds_read_b128 hidden from the compiler: an ordinary LDS read of the ring
// makes hipcc wait vmcnt(0) for every LDS-DMA in flight (it cannot tell the
// stages apart), which drains the pipeline each block.  The caller passes
// the results through lgkm_ready() before using them: the compiler sees no
// dependence between the asm load and a plain s_waitcnt, and would hoist
// the uses above the wait.
typedef uint32_t fold_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ fold_u4 lds_read16(const uint4* p) {
    fold_u4 v;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint4*)p;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
#else
    v = fold_u4{p->x, p->y, p->z, p->w};
#endif
    return v;
}
// s_waitcnt lgkmcnt(0) tied to v: uses of v stay below the wait.
__device__ __forceinline__ void lgkm_ready(fold_u4& v) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
#else
    (void)v;
#endif
}
// global_load_lds_dwordx4: 16 bytes per lane from g to LDS at l + 16 * lane
// (l wave-uniform).
__device__ __forceinline__ void glds16(const void* g, void* l) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
#else
    (void)g;
    (void)l;
#endif
}

template <int MT, int NT, int SG, int KG, int P>
__global__ __launch_bounds__(64 * (8 / NT) * KG, 2) void k_fold_glds(
    const uint32_t* __restrict__ bits, uint64_t wpk, const uint4* __restrict__ dbs, uint64_t nsg, uint32_t nkeys,
    uint64_t sg_per_block, uint32_t* __restrict__ parts, uint32_t* __restrict__ zero, uint64_t zero_words,
    uint64_t wlim) {
    using Sh = GldsShape<MT, NT, SG, KG, P>;
    constexpr int NS = Sh::NS, PR = Sh::PR;
    constexpr bool SC = DPF_FOLD_SEL_CHEAP >= 0 ? DPF_FOLD_SEL_CHEAP == 1 : NT < MT;
    __shared__ __attribute__((aligned(16))) uint4 s_ring[P * Sh::kStage];   // the only LDS object (glds waits)
    zero_answers(zero, zero_words);
    const uint32_t l = threadIdx.x & 63, h = l >> 5, r = l & 31;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t w = wv % NS, kg = wv / NS;
    const uint64_t s0 = (uint64_t)blockIdx.x * sg_per_block;
    const uint64_t s1 = s0 + sg_per_block < nsg ? s0 + sg_per_block : nsg;
    if (s0 >= s1) return;                                    // uniform over the workgroup
    const uint64_t nblk = (s1 - s0 + SG - 1) / SG;
    // Issue block b into stage b % P (clamped past the end).
    auto issue = [&](uint64_t b) __attribute__((always_inline)) {
        uint4* st = s_ring + (uint32_t)(b % P) * Sh::kStage;
        const uint64_t sb = s0 + (b < nblk ? b : nblk - 1) * SG;
        // selection rows: this wave's kSelLanes slots
        if (l < (uint32_t)Sh::kSelLanes) {
            const uint32_t slot = wv * Sh::kSelLanes + l;
            const uint32_t row = slot / PR, qs = slot % PR;
            const uint32_t q = qs ^ ((row / (16 / PR)) & (PR - 1));
            const uint32_t krow = row < nkeys ? row : nkeys - 1;
            uint64_t word = sb * 8 + 4 * q;
            if (word + 4 > wlim) word = wlim - 4;
            glds16(bits + (uint64_t)krow * wpk + word, st + wv * Sh::kSelLanes);
        }
        // this wave's DB pieces
#pragma unroll
        for (int sl = 0; sl < SG; ++sl) {
            const uint64_t S = sb + sl < s1 ? sb + sl : s1 - 1;
#pragma unroll
            for (int j = 0; j < NT; ++j)
                glds16(dbs + (S * 256 + 32u * (w * NT + j) + r) * 2 + h,
                       st + Sh::kSelPieces + ((wv * SG + sl) * NT + j) * 64);
        }
    };
    fold_v16f acc[MT][NT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[m][j][e] = 0.0f;
#pragma unroll
    for (int b = 0; b < P - 1; ++b) issue((uint64_t)b);
    for (uint64_t b = 0; b < nblk; ++b) {
        fold_prio(b, nblk);
        wait_vm<Sh::G * (P - 2)>();                          // this wave's DMAs of block b have landed
        wait_lgkm0();
        __builtin_amdgcn_s_barrier();                        // ... and every wave's; block b - 1 fully read
        issue(b + P - 1);                                    // into the stage block b - 1 used
        const uint4* st = s_ring + (uint32_t)(b % P) * Sh::kStage;
        const uint64_t n = s1 - (s0 + b * SG);
#pragma unroll
        for (int sl = 0; sl < SG; ++sl) {
            if ((uint64_t)sl >= n) break;
            fold_u4 A[MT], B[NT];
#pragma unroll
            for (int m = 0; m < MT; ++m) A[m] = lds_read16(st + sel_slot<PR>(32 * (MT * kg + m) + r, 2 * sl + h));
#pragma unroll
            for (int j = 0; j < NT; ++j) B[j] = lds_read16(st + Sh::kSelPieces + ((wv * SG + sl) * NT + j) * 64 + l);
#pragma unroll
            for (int m = 0; m < MT; ++m) lgkm_ready(A[m]);
#pragma unroll
            for (int j = 0; j < NT; ++j) lgkm_ready(B[j]);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                fold_v8i bo[NT];
#pragma unroll
                for (int j = 0; j < NT; ++j) bo[j] = fp4_db<SC>(B[j][t]);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const fold_v8i ao = fp4_sel<SC>(A[m][t]);
#pragma unroll
                    for (int j = 0; j < NT; ++j)
                        acc[m][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ao, bo[j], acc[m][j], kFoldFp4,
                                                                                   kFoldFp4, 0, kE8M0One, 0, kE8M0One);
                }
            }
        }
    }
    wait_vm<0>();                                            // the clamped tail DMAs, before the waves exit
    constexpr uint32_t pkeys = 32 * MT * KG;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            uint32_t out = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t p = ((uint32_t)acc[m][j][e]) & 1u;
                const uint64_t b = __builtin_amdgcn_ballot_w64(p != 0);
                const uint32_t row0 = (e & 3) + 8 * (e >> 2);
                out = l == row0 ? (uint32_t)b : out;
                out = l == row0 + 4 ? (uint32_t)(b >> 32) : out;
            }
            if (l < 32) parts[((uint64_t)blockIdx.x * pkeys + 32 * (MT * kg + m) + l) * 8 + w * NT + j] = out;
        }
}

#endif  // DPF_FOLD_GLDS_KERNEL

// The sliced layout (above) from a row-major DB of 32-byte records: one wave
// per 64 records (record groups 2q', 2q'+1 of a super-group); lane l holds
// record l's 8 words and one ballot per bit position transposes 32 x 32 bits.
__global__ __launch_bounds__(256) void k_slice_db(const uint4* __restrict__ db, uint64_t nrec,
                                                   uint32_t* __restrict__ dbs, uint64_t nwaves) {
    const uint64_t q = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (q >= nwaves) return;
    const uint32_t l = threadIdx.x & 63;
    const uint64_t rec = q * 64 + l;
    uint4 a = make_uint4(0, 0, 0, 0), b = a;
    if (rec < nrec) {
        a = db[2 * rec];
        b = db[2 * rec + 1];
    }
    const uint32_t wd[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint64_t S = q >> 2;
    const uint32_t g = 2 * (uint32_t)(q & 3) + (l >> 5);
#pragma unroll
    for (int wi = 0; wi < 8; ++wi) {
        uint32_t out = 0;
#pragma unroll
        for (int bb = 0; bb < 32; ++bb) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(((wd[wi] >> bb) & 1u) != 0);
            out = l == (uint32_t)bb ? (uint32_t)m : out;
            out = l == (uint32_t)bb + 32 ? (uint32_t)(m >> 32) : out;
        }
        dbs[(S * 256 + 32 * wi + (l & 31)) * 8 + g] = out;
    }
}

// Few keys over the sliced DB: no matrix product needed.  Thread n of a
// 256-thread workgroup owns bit position n; per super-group it reads its 8
// words dbs[S][n][0..7] (the workgroup: 8 KiB contiguous) and, for every key
// k, XORs (selection word & DB word) into acc[k] -- one v_bitop3 per word and
// key, the selection words wave-uniform (scalar loads).  The answer bit
// (k, n) is the parity of popcount(acc[k]).  Used for one key (97 us at
// configs[4] against the MFMA fold's 103): with 4 or 16 keys its per-key
// scalar loads serialise (131 / 388 us against 104 / 107,
// profiles/r04/fold_ab/).
// (Nontemporal DB loads, as the matrix-core fold takes them above 256 MiB,
// measured 95.2-95.8 against 93.9-94.4 us here at 2^24 records: not used.)
template <int KB, bool NTDB = false>
__global__ __launch_bounds__(256) void k_fold_sliced_direct(const uint32_t* __restrict__ bits, uint64_t wpk,
                                                            const uint4* __restrict__ dbs, uint64_t nsg,
                                                            uint32_t nkeys, uint64_t sg_per_block,
                                                            uint32_t* __restrict__ parts, uint32_t* __restrict__ zero,
                                                            uint64_t zero_words) {
    zero_answers(zero, zero_words);
    const uint32_t n = threadIdx.x, l = n & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t s0 = (uint64_t)blockIdx.x * sg_per_block;
    const uint64_t s1 = s0 + sg_per_block < nsg ? s0 + sg_per_block : nsg;
    uint32_t acc[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) acc[k] = 0;
    auto fold = [&](uint64_t S, const uint4& a, const uint4& b) __attribute__((always_inline)) {
        const uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        const bool in = 8 * S + 8 <= wpk;                      // uniform
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            if ((uint32_t)k >= nkeys || !in) continue;         // uniform
            const uint32_t* sel = bits + (uint64_t)k * wpk + 8 * S;
#pragma unroll
            for (int g = 0; g < 8; ++g) acc[k] = xam(acc[k], x[g], sel[g]);
        }
        if (!in) {                                             // the key rows end inside this super-group
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                if ((uint32_t)k >= nkeys) continue;
                const uint32_t* sel = bits + (uint64_t)k * wpk;
#pragma unroll
                for (int g = 0; g < 8; ++g)
                    if (8 * S + g < wpk) acc[k] = xam(acc[k], x[g], sel[8 * S + g]);
            }
        }
    };
    uint64_t S = s0;
    for (; S + 1 < s1; S += 2) {
        const uint4 a0 = fold_ld<NTDB>(&dbs[(S * 256 + n) * 2]), b0 = fold_ld<NTDB>(&dbs[(S * 256 + n) * 2 + 1]);
        const uint4 a1 = fold_ld<NTDB>(&dbs[((S + 1) * 256 + n) * 2]);
        const uint4 b1 = fold_ld<NTDB>(&dbs[((S + 1) * 256 + n) * 2 + 1]);
        fold(S, a0, b0);
        fold(S + 1, a1, b1);
    }
    if (S < s1) fold(S, fold_ld<NTDB>(&dbs[(S * 256 + n) * 2]), fold_ld<NTDB>(&dbs[(S * 256 + n) * 2 + 1]));
    // parts[block][key][8]: wave w holds answer words 2w (lanes 0-31) and 2w+1.
#pragma unroll
    for (int k = 0; k < KB; ++k) {
        const uint64_t m = __builtin_amdgcn_ballot_w64((__builtin_popcount(acc[k]) & 1) != 0);
        if (l < 2) parts[((uint64_t)blockIdx.x * KB + k) * 8 + 2 * w + l] = l ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
}

uint64_t pir_sliced_bytes(uint64_t nrec) { return (nrec + 255) / 256 * 256 * 32; }

hipError_t launch_slice_db(const uint8_t* db, uint64_t nrec, uint8_t* dbs, hipStream_t st) {
    const uint64_t nsg = (nrec + 255) / 256;
    if (nsg == 0) return hipSuccess;
    const uint64_t nwaves = nsg * 4;
    hipLaunchKernelGGL(k_slice_db, dim3((uint32_t)((nwaves + 3) / 4)), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(db), nrec, reinterpret_cast<uint32_t*>(dbs), nwaves);
    return hipGetLastError();
}

namespace {
#if DPF_FOLD_GLDS_KERNEL
template <int MT, int NT, int SG, int KG, int P>
hipError_t launch_glds(const uint32_t* bits, uint64_t wpk, uint64_t wlim, const uint8_t* dbs, uint64_t nsg, uint32_t nk,
                       uint32_t* parts, uint32_t* zero, uint64_t zero_words, uint64_t want, uint64_t& blocks,
                       hipStream_t st) {
    constexpr int NW = 8 / NT * KG;
    uint64_t spb;
    split_chunks(nsg, want, SG, blocks, spb);
    hipLaunchKernelGGL((k_fold_glds<MT, NT, SG, KG, P>), dim3((uint32_t)blocks), dim3(64 * NW), 0, st, bits, wpk,
                       reinterpret_cast<const uint4*>(dbs), nsg, nk, spb, parts, zero, zero_words, wlim);
    return hipGetLastError();
}

// DPF_FOLD_GLDS (env; measurement): 0 = register-staged k_fold_mfma, else
// the LDS-DMA ring k_fold_glds for 33-64 keys: 1 = SG 2, P 4; 2 = SG 2, P 3;
// 3 = SG 1, P 5; 4 = SG 1, P 6.
static int fold_glds_mode() {
    static const int m = [] {
        const char* e = getenv("DPF_FOLD_GLDS");
        return e ? atoi(e) : DPF_FOLD_GLDS_DEFAULT;
    }();
    return m;
}

#endif

// The DB pieces of a matrix-core fold over at least this many DB bytes are
// loaded nontemporal.  r05 (tools/archive/r05_nt.sh, profiles/r05/fold_nt/, B = 64,
// fold us, nontemporal vs default): 2^24 x 32 B (512 MiB, twice the chip's
// last-level cache) 123-125 vs 135-138, and B = 16 95 vs 105-107; 2^23 66-69
// vs 67-74; but 2^22 39-40 vs 35-36 and 2^21 (an N = 8 rank) 25.5 vs 24.7:
// slices that stay cached between batches lose.  DPF_FOLD_NT_MIN overrides.
constexpr uint64_t kFoldNtMinBytes = 256ull << 20;
static uint64_t fold_nt_min_bytes() {
    static const uint64_t v = [] {
        const char* e = getenv("DPF_FOLD_NT_MIN");
        return e && *e ? strtoull(e, nullptr, 0) : kFoldNtMinBytes;
    }();
    return v;
}

// One key group (<= 32 * MT * KG keys) over the sliced DB: passes of at most
// (workgroup cap) x kFoldMaxSgPerBlock super-groups, each a fold launch whose
// workgroups fold <= kFoldMaxSgPerBlock super-groups (fp32-exact counts, see
// k_fold_mfma) and a k_xor_parts launch that XORs the partials into ans.
template <int MT, int NT, int SG, int KG>
hipError_t launch_mfma_mt(const uint32_t* bits, uint64_t wpk, const uint8_t* dbs, uint64_t nsg, uint32_t nk,
                          uint32_t* parts, uint32_t* ans, uint32_t* zero, uint64_t zero_words, hipStream_t st,
                          uint32_t sgm_keys = 0, uint32_t sgm_g = 1) {
    constexpr int NW = 8 / NT * KG;
    // Resident workgroups only (one round): each takes a contiguous run of
    // whole staged blocks.  (A fixed 4 workgroups per CU left 1/4 - 3/4 of
    // them for a second round at 3 or 1 resident per CU.)
    static int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fold_mfma<MT, NT, SG, KG>, 64 * NW, 0) != hipSuccess || n < 1)
            n = 1;
        return n;
    }();
    static const int env_pcu = [] {                           // A/B runs: this many per CU (<= occupancy)
        const char* e = getenv("DPF_FOLD_PER_CU");
        return e && atoi(e) > 0 ? atoi(e) : 0;
    }();
    const uint64_t cap = g_fold_blocks.load(std::memory_order_relaxed);
    const uint64_t msg = (uint64_t)fold_max_sg() / SG * SG > 0 ? (uint64_t)fold_max_sg() / SG * SG : SG;
    // (The super-group-major layouts are measurement-only: one pass.)
    const uint64_t per_pass = sgm_keys ? nsg : cap * msg;
    const bool ntdb = nsg * 256 * 32 >= fold_nt_min_bytes();
    // Two workgroups per CU instead of the occupancy limit (3 at 33-64 keys)
    // for cached DB slices and for the one-key-tile shape: fewer partials to
    // combine and less per-workgroup overhead (r05, tools/archive/r05_fpercu.sh,
    // profiles/r05/fold_blocks/, medians of 5: 2^21 x 32 B 22.6 vs 24.7 us,
    // 2^22 34.8 vs 36.0, B = 16 at 2^24 91.9 vs 96.6, B = 32 96.3 vs 99.8;
    // but B = 64 at 2^23 / 2^24 67.9 / 130.7 vs 67.0 / 125.9).  One per CU
    // for 33-64 keys over a slice of <= 64 MiB (the PIR rank at N = 8): rank
    // step 0.0741-0.0750 vs 0.0742-0.0759 ms, lower in 5 of 6 interleaved
    // pairs; at N = 4 (128 MiB) the pairs split 3 / 3 and the fold alone was
    // slower (37.6 vs 33.9 us), so it keeps 2 (tools/archive/r05_fpercu1.sh,
    // profiles/r05/fold_blocks/per_cu1_*.txt).
    const bool small_slice = nsg * 256 * 32 <= (64ull << 20);
    uint64_t pcu = small_slice && MT == 2 ? 1 : (!ntdb || MT == 1) && per_cu > 2 ? 2 : (uint64_t)per_cu;
    if (env_pcu > 0) pcu = (uint64_t)(env_pcu < per_cu ? env_pcu : per_cu);
    if (pcu > (uint64_t)per_cu) pcu = (uint64_t)per_cu;
    const uint64_t resident = (uint64_t)cu_count_fold() * pcu;
    for (uint64_t S0 = 0; S0 < nsg; S0 += per_pass) {
        const uint64_t n = nsg - S0 < per_pass ? nsg - S0 : per_pass;
        // enough workgroups that none folds more than msg super-groups
        uint64_t want = (n + msg - 1) / msg;
        if (want < resident) want = resident;
        if (want > cap) want = cap;
        const uint32_t* b = bits + (sgm_keys ? S0 / (sgm_g ? sgm_g : 1) * sgm_keys * (sgm_g ? sgm_g : 1) * 8 : S0 * 8);
        const uint64_t wlim = wpk > S0 * 8 ? wpk - S0 * 8 : 0;
        const uint8_t* d = dbs + S0 * 256 * 32;
        uint32_t* z = S0 == 0 ? zero : nullptr;
        const uint64_t zw = S0 == 0 ? zero_words : 0;
        uint64_t blocks = 0;
        hipError_t e = hipErrorUnknown;
        bool done = false;
#if DPF_FOLD_GLDS_KERNEL
        if constexpr (MT == 2 && NT == 2 && KG == 1) {
            if (!sgm_keys) {
                done = true;
                switch (fold_glds_mode()) {
                    case 1: e = launch_glds<2, 2, 2, 1, 4>(b, wpk, wlim, d, n, nk, parts, z, zw, want, blocks, st); break;
                    case 2: e = launch_glds<2, 2, 2, 1, 3>(b, wpk, wlim, d, n, nk, parts, z, zw, want, blocks, st); break;
                    case 3: e = launch_glds<2, 2, 1, 1, 5>(b, wpk, wlim, d, n, nk, parts, z, zw, want, blocks, st); break;
                    case 4: e = launch_glds<2, 2, 1, 1, 6>(b, wpk, wlim, d, n, nk, parts, z, zw, want, blocks, st); break;
                    default: done = false;
                }
            }
        }
#endif
        if (!done) {
            uint64_t spb;
            split_chunks(n, want, SG, blocks, spb, cap);
            if (spb > msg) return hipErrorInvalidValue;    // fp32-exact counts: never more than msg per workgroup
            if (sgm_keys && sgm_g == 4)
                hipLaunchKernelGGL((k_fold_mfma<MT, NT, SG, KG, 4>), dim3((uint32_t)blocks), dim3(64 * NW), 0, st, b,
                                   wpk, reinterpret_cast<const uint4*>(d), n, nk, spb, parts, z, zw, wlim, sgm_keys);
            else if (sgm_keys)
                hipLaunchKernelGGL((k_fold_mfma<MT, NT, SG, KG, 1>), dim3((uint32_t)blocks), dim3(64 * NW), 0, st, b,
                                   wpk, reinterpret_cast<const uint4*>(d), n, nk, spb, parts, z, zw, wlim, sgm_keys);
            else if (ntdb)
                hipLaunchKernelGGL((k_fold_mfma<MT, NT, SG, KG, 0, true>), dim3((uint32_t)blocks), dim3(64 * NW), 0, st,
                                   b, wpk, reinterpret_cast<const uint4*>(d), n, nk, spb, parts, z, zw, wlim);
            else
                hipLaunchKernelGGL((k_fold_mfma<MT, NT, SG, KG>), dim3((uint32_t)blocks), dim3(64 * NW), 0, st, b, wpk,
                                   reinterpret_cast<const uint4*>(d), n, nk, spb, parts, z, zw, wlim);
            e = hipGetLastError();
        }
        if (e != hipSuccess) return e;
        if (hipError_t e2 = launch_xor_parts(parts, blocks, nk, 32u * MT * KG, 8u, ans, 8, 0u, st); e2 != hipSuccess)
            return e2;
    }
    return hipSuccess;
}
}  // namespace

// Tile shape per key count (32 keys per tile): MT key tiles x NT bit tiles
// per wave, KG key groups per workgroup.  DPF_FOLD_SHAPE picks among
// measured alternatives for 65-256 keys (A/B builds).
#ifndef DPF_FOLD_SLICED_DIRECT
#define DPF_FOLD_SLICED_DIRECT 1    // keys up to which the sliced fold uses k_fold_sliced_direct (0: MFMA always)
#endif
#ifndef DPF_FOLD_SHAPE
#define DPF_FOLD_SHAPE 0
#endif
#ifndef DPF_FOLD_SHAPE64
#define DPF_FOLD_SHAPE64 0   // 33-64 keys
#endif
hipError_t launch_pir_fold_sliced(const uint32_t* bits, uint64_t words_per_key, const uint8_t* dbs, uint64_t nrec,
                                  uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st, uint32_t sgm_keys,
                                  uint32_t sgm_g) {
    if (nkeys == 0) return hipSuccess;
    if (nrec == 0) return hipMemsetAsync(ans, 0, (size_t)nkeys * 32, st);
    if (words_per_key % 4 != 0 || words_per_key * 32 < nrec) return hipErrorInvalidValue;
    const uint64_t nsg = (nrec + 255) / 256;
    if (nkeys <= (uint32_t)DPF_FOLD_SLICED_DIRECT && !sgm_keys) {   // one key: popcount fold, no MFMA
        uint64_t blocks, spb;
        split_chunks(nsg, (uint64_t)cu_count_fold() * 8, 2, blocks, spb);
        const uint32_t kb = 1;
        hipLaunchKernelGGL(k_fold_sliced_direct<1>, dim3((uint32_t)blocks), dim3(256), 0, st, bits, words_per_key,
                           reinterpret_cast<const uint4*>(dbs), nsg, nkeys, spb, parts, ans, (uint64_t)nkeys * 8);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        return launch_xor_parts(parts, blocks, nkeys, kb, 8u, ans, 8, 0u, st);
    }
    for (uint32_t k0 = 0; k0 < nkeys; k0 += 256) {
        const uint32_t nk = nkeys - k0 < 256 ? nkeys - k0 : 256;
        const uint32_t* b = bits + (sgm_keys ? (uint64_t)k0 * 8 * sgm_g : (uint64_t)k0 * words_per_key);
        uint32_t* zero = k0 == 0 ? ans : nullptr;
        const uint64_t zw = k0 == 0 ? (uint64_t)nkeys * 8 : 0;
        uint32_t* a = ans + (uint64_t)k0 * 8;
        hipError_t e;
#define DPF_MT(MT_, NT_, SG_, KG_) \
    launch_mfma_mt<MT_, NT_, SG_, KG_>(b, words_per_key, dbs, nsg, nk, parts, a, zero, zw, st, sgm_keys, sgm_g)
        if (nk <= 32) e = DPF_MT(1, 2, 4, 1);
        else if (nk <= 64) {
            if (DPF_FOLD_SHAPE64 == 1) e = DPF_MT(2, 2, 4, 1);
            else if (DPF_FOLD_SHAPE64 == 2) e = DPF_MT(1, 2, 4, 2);
            else if (DPF_FOLD_SHAPE64 == 3) e = DPF_MT(2, 4, 2, 1);
            else if (DPF_FOLD_SHAPE64 == 4) e = DPF_MT(2, 2, 1, 1);
            else e = DPF_MT(2, 2, 2, 1);
        } else if (nk <= 128) {
            if (DPF_FOLD_SHAPE == 1) e = DPF_MT(2, 4, 2, 2);
            else e = DPF_MT(4, 2, 4, 1);
        } else {
            if (DPF_FOLD_SHAPE == 1) e = DPF_MT(2, 4, 2, 4);
            else if (DPF_FOLD_SHAPE == 2) e = DPF_MT(4, 4, 2, 2);
            else if (DPF_FOLD_SHAPE == 3) e = DPF_MT(2, 8, 2, 4);
            else e = DPF_MT(8, 2, 4, 1);
        }
#undef DPF_MT
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#ifndef DPF_PIR_FUSED_KERNEL
#define DPF_PIR_FUSED_KERNEL 0   // k_pir_fused is built only in the experimental build (make experimental)
#endif
#if DPF_PIR_FUSED_KERNEL
// ---------------------------------------------------------------------------
// Fused PIR answer: the subtree EvalFull and the matrix-core fold in ONE
// launch, so the fold's MFMA and HBM streams could run under the tree's
// LDS-bound AES instead of after it.  The selection bits
// never reach HBM.  Bit-exact, and measured SLOWER than the two launches
// (0.45-0.47 vs 0.41 ms per configs[4] step, profiles/r04/fused/): one key
// per lane and 3 producer waves per SIMD need 0.39 ms for the tree alone,
// against 0.25 ms for the one-key-per-wave kernel at 4 waves per SIMD.  So
// it is opt-in (dpf_set_pir_kernel(DPF_PIR_FUSED)).
//
// One 1024-thread workgroup (16 waves, the whole CU: one 64 KiB T-table)
// per block of 256 leaf pairs of the subtree, i.e. 256 super-groups (65,536
// records) of the DB, for up to 64 keys:
//   waves 0..11  producers: lane = key.  Wave p evaluates pairs [a0, a1) of
//                the block (21-22 of them) for all keys, depth-first as
//                evalFullRecursive does (dpf/dpf.go:213-241): a leaf pair is
//                the two leaves under a node at level stop-1, 32 bytes = 256
//                selection bits = one super-group of the sliced DB.  Each
//                pair goes to a ring slot in LDS, then a workgroup barrier.
//   waves 12..15 folders (one per SIMD): after the barrier of period t, the
//                12 pairs of period t are folded by v_mfma_scale_f32_32x32x64
//                _f8f6f4 exactly as k_fold_mfma does: folder f owns answer
//                bits 64f..64f+63 of every key (2 x 2 tiles, 64 accumulator
//                registers), selection words from the ring (ds_read_b128),
//                DB words from the sliced DB in HBM.
// The ring has two slots: a slot is refilled two periods later, after the
// folders passed the barrier that ends their fold of it, so one barrier per
// period orders both directions.  A producer walks from the block root
// (walked once for all keys by folder wave 0 at the start, in LDS) 3 levels
// down to each 32-pair piece of its range and expands only the nodes over
// its pairs (fz_visit: one AES where the range leaves one child).
#ifndef DPF_FZ_PRODONLY
#define DPF_FZ_PRODONLY 0     // measurement only: 16 producer waves, no folders, no ring flow control
#endif
constexpr int kFzProd = DPF_FZ_PRODONLY ? 16 : 12;   // producer waves
constexpr int kFzFold = DPF_FZ_PRODONLY ? 0 : 4;     // folder waves
constexpr int kFzThreads = 64 * (kFzProd + kFzFold);
constexpr uint32_t kFzBlockPairs = 256;      // leaf pairs (= DB super-groups) per workgroup
constexpr uint32_t kFzBlockLog = 8;
constexpr uint32_t kFzSubLog = 5;            // a walked piece: 32 pairs below a node 5 levels up
constexpr uint32_t kFzRow = 12;              // words per key row of a slot (8 + 4: conflict-free b128 reads)
constexpr uint32_t kFzSlot = kFzProd * 64 * kFzRow;
constexpr uint32_t kFzPeriods = (kFzBlockPairs + kFzProd - 1) / kFzProd;   // 22

__device__ __forceinline__ uint32_t fz_a0(uint32_t p) { return kFzBlockPairs * p / kFzProd; }

struct FzCtx {
    const uint8_t* tab;
    uint32_t lo;
    const uint32_t* ek;    // this lane's expanded key records (k_unpack)
    Blk fcw;
    uint32_t P;            // level of a leaf pair's parent: stop - 1
    uint32_t* row;         // this lane's row in ring slot 0 (slot 1 at + kFzSlot)
    uint32_t period;       // pairs emitted so far
    uint32_t live;         // ~0: lane < nkeys
    uint32_t p;            // producer index (wave)
    uint32_t* prod;        // s_prod: pairs written, per producer
    const uint32_t* fold;  // s_fold: ring entries folded, per folder
    const uint32_t* dbw;   // sliced DB as words; the producer's next super-group is touched into L2
    uint64_t sg;           // super-group of the pair being computed
    uint64_t nsg;
    uint32_t touch;        // last touch load (consumed one pair later)
};

// Workgroup-scope flags in LDS (ASYNC ring).  Every wait is bounded, so each
// wave reaches its exit even if a flag were never set; a wait that runs out
// records it in g_fz_timeout (a vector atomic), and the next launch_pir_fused
// reports hipErrorLaunchTimeOut instead of launching (the answers of the
// timed-out launch are not to be trusted).  All 16 waves of the workgroup
// are resident on one CU, so no wait should ever run out.
constexpr uint32_t kFzSpin = 1u << 22;
__device__ uint32_t g_fz_timeout;
__device__ __forceinline__ void fz_timed_out() { atomicOr(&g_fz_timeout, 1u); }
__device__ __forceinline__ uint32_t lds_acquire(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The pair under node n (level P): two leaves (dpf.go:214-224) = 256 bits.
template <bool ASYNC>
__device__ __forceinline__ void fz_emit(FzCtx& c, const Node& n) {
    const CW cw = load_cw(c.ek, c.P);
    Node L, R;
    expand<DPF_FZ_BATCH>(c.tab, c.lo, n, cw, L, R);
    Blk oL, oR;
    mmo_pair<DPF_FZ_BATCH>(c.tab, c.lo, KeyFixed<false>{}, L.s, oL, KeyFixed<false>{}, R.s, oR);
    oL = leaf_fix(oL, L.t, c.fcw);
    oR = leaf_fix(oR, R.t, c.fcw);
    const uint32_t m = c.live;
    const uint32_t i = c.period;
    // Touch the next pair's 8 KiB of the sliced DB (one 128-byte line per
    // lane) so the folders find it in L2 a period later; the value of the
    // previous touch is consumed here, long after it landed.
#if DPF_FZ_TOUCH
    asm volatile("" ::"v"(c.touch));
    {
        const uint64_t s = c.sg + 1 < c.nsg ? c.sg + 1 : c.nsg - 1;
        c.touch = c.dbw[s * 2048 + (threadIdx.x & 63) * 32];
        c.sg += 1;
    }
#endif
    if constexpr (ASYNC && !DPF_FZ_PRODONLY) {
        // Slot i & 1 is free once every folder has folded this producer's
        // pair i - 2 (ring entry (i - 2) * kFzProd + p in folding order).
        if (i >= 2) {
            const uint32_t need = (i - 2) * kFzProd + c.p + 1;
            for (uint32_t n = 0;; ++n) {
                uint32_t lo_ = lds_acquire(c.fold);
#pragma unroll
                for (int f = 1; f < kFzFold; ++f) {
                    const uint32_t v = lds_acquire(c.fold + f);
                    lo_ = v < lo_ ? v : lo_;
                }
                if (lo_ >= need) break;
                if (n == kFzSpin) {
                    if ((threadIdx.x & 63) == 0) fz_timed_out();
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    uint32_t* row = c.row + (DPF_FZ_PRODONLY ? 0 : (i & 1) * kFzSlot);
    *reinterpret_cast<uint4*>(row) = make_uint4(oL.c0 & m, oL.c1 & m, oL.c2 & m, oL.c3 & m);
    *reinterpret_cast<uint4*>(row + 4) = make_uint4(oR.c0 & m, oR.c1 & m, oR.c2 & m, oR.c3 & m);
    if constexpr (ASYNC) {
        lds_release(c.prod + c.p, i + 1);
    } else {
        __syncthreads();
    }
    c.period = i + 1;
}

// Pairs [lo, hi) of the 2^K pairs below node n (level P - K), in order.
// lo, hi are wave-uniform; a child outside the range is never computed.
template <int K, bool ASYNC>
__device__ __forceinline__ void fz_visit(FzCtx& c, const Node& n, uint32_t lo, uint32_t hi) {
    if constexpr (K == 0) {
        fz_emit<ASYNC>(c, n);
    } else {
        constexpr uint32_t half = 1u << (K - 1);
        const CW cw = load_cw(c.ek, c.P - K);
        const bool needL = lo < half, needR = hi > half;
        Node L, R;
        if (needL && needR) {
            expand<DPF_FZ_BATCH>(c.tab, c.lo, n, cw, L, R);
        } else {
            L = n;
            walk_step<DPF_FZ_BATCH>(c.tab, c.lo, L, cw, needR ? 1u : 0u);
            R = L;
        }
        Node ch = L;
        const Node pend = R;
        const uint32_t s0 = needL ? 0u : 1u, s1 = needR ? 2u : 1u;
#pragma nounroll
        for (uint32_t s = s0; s < s1; ++s) {
            const uint32_t clo = s == 0 ? lo : (lo > half ? lo - half : 0u);
            const uint32_t chi = s == 0 ? (hi < half ? hi : half) : hi - half;
            fz_visit<K - 1, ASYNC>(c, ch, clo, chi);
            ch = pend;
        }
    }
}

template <bool ASYNC>
__global__ __launch_bounds__(kFzThreads, 1) void k_pir_fused(const uint32_t* __restrict__ ek, uint32_t nkeys,
                                                            uint32_t stop, uint32_t pb, uint64_t prefix,
                                                            const uint4* __restrict__ dbs, uint64_t nsg,
                                                            uint32_t* __restrict__ parts, uint32_t* __restrict__ zero,
                                                            uint64_t zero_words) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    __shared__ __attribute__((aligned(16))) uint32_t s_ring[(DPF_FZ_PRODONLY ? 1 : 2) * kFzSlot];
    __shared__ uint32_t s_top[64 * 5];
    __shared__ uint32_t s_prod[kFzProd], s_fold[4];
    if (threadIdx.x < kFzProd) s_prod[threadIdx.x] = 0;
    if (threadIdx.x < 4) s_fold[threadIdx.x] = 0;
    zero_answers(zero, zero_words);
    fill_table(s_tab);
    const uint32_t l = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t P = stop - 1;
    const uint32_t lb = P - kFzBlockLog;                      // level of the block root
    const uint32_t* kek = ek + (uint64_t)(l < nkeys ? l : 0) * ((uint64_t)(stop + 2) * 8);
    if (wv == (DPF_FZ_PRODONLY ? 0 : kFzProd)) {
        // Block root of every key: prefix bits, then the block index (dpf.go:183-201 path).
        const uint64_t path = (prefix << (lb - pb)) | blockIdx.x;
        Node n;
        n.s = load_blk(kek);
        n.t = kek[4];
        for (uint32_t i = 0; i < lb; ++i)
            walk_step<DPF_WALK_BATCH_FZ>(tab, lo, n, load_cw(kek, i), (uint32_t)(path >> (lb - 1 - i)) & 1u);
        uint32_t* f = s_top + 5 * l;
        f[0] = n.s.c0; f[1] = n.s.c1; f[2] = n.s.c2; f[3] = n.s.c3; f[4] = n.t;
    }
    __syncthreads();
    if (wv < kFzProd) {
        FzCtx c;
        c.tab = tab;
        c.lo = lo;
        c.ek = kek;
        c.fcw = load_blk(kek + 8 + 8 * stop);
        c.P = P;
        c.row = s_ring + (wv * 64 + l) * kFzRow;
        c.period = 0;
        c.live = l < nkeys ? ~0u : 0u;
        c.p = wv;
        c.prod = s_prod;
        c.fold = s_fold;
        c.dbw = reinterpret_cast<const uint32_t*>(dbs);
        c.nsg = nsg;
        c.touch = 0;
        const uint32_t* f = s_top + 5 * l;
        Node top;
        top.s = {f[0], f[1], f[2], f[3]};
        top.t = f[4];
        const uint32_t a0 = fz_a0(wv), a1 = fz_a0(wv + 1);
        for (uint32_t a = a0; a < a1;) {
            const uint32_t j = a >> kFzSubLog;
            const uint32_t b = (j + 1) << kFzSubLog < a1 ? (j + 1) << kFzSubLog : a1;
            c.sg = (uint64_t)blockIdx.x * kFzBlockPairs + a;
            Node n = top;
#pragma nounroll
            for (uint32_t i = 0; i < kFzBlockLog - kFzSubLog; ++i)
                walk_step<false>(tab, lo, n, load_cw(kek, lb + i), (j >> (kFzBlockLog - kFzSubLog - 1 - i)) & 1u);
            fz_visit<kFzSubLog, ASYNC>(c, n, a - (j << kFzSubLog), b - (j << kFzSubLog));
            a = b;
        }
        if constexpr (!ASYNC) {
            while (c.period < kFzPeriods) {   // idle periods (21 of 22 pairs)
                __syncthreads();
                ++c.period;
            }
        }
        return;
    }
    // Folders.
    const uint32_t fw = wv - kFzProd, h = l >> 5, r = l & 31;
    const uint64_t S0 = (uint64_t)blockIdx.x * kFzBlockPairs;
    fold_v16f acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[m][j][e] = 0.0f;
    // DB words of step q = (period t, producer p): dbs[S][64 fw + 32 j + r][4h .. 4h+3]
    // for S = S0 + a0(p) + t; zero where p has no pair in t or S is past the DB.
    auto ldb = [&](uint32_t q, uint4 (&B)[2]) __attribute__((always_inline)) {
        const uint32_t t = q / kFzProd, p = q % kFzProd;
        const uint32_t a = fz_a0(p) + t;
        const uint64_t S = S0 + a;
        const bool ok = a < fz_a0(p + 1) && S < nsg;
        const uint64_t Sc = ok ? S : 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint4 x = dbs[(Sc * 256 + 64 * fw + 32 * j + r) * 2 + h];
            B[j] = ok ? x : make_uint4(0, 0, 0, 0);
        }
    };
    // Ring entries in folding order q = t * kFzProd + p.  The DB words of an
    // entry are loaded two entries before it is folded, and its producer
    // touched them a pair earlier (fz_emit), so they come from L2: one entry
    // is ~0.2 us of MFMA work against ~1-2 us of HBM latency, and with the
    // words fetched from HBM one entry ahead the folders, not the producers,
    // set the kernel time (0.45 vs 0.41 ms for the two-launch path).
    constexpr uint32_t Q = kFzPeriods * kFzProd;
    static_assert(Q % 2 == 0, "two DB buffers in rotation");
    auto fold_entry = [&](uint32_t q, const uint4 (&B)[2]) __attribute__((always_inline)) {
        const uint32_t t = q / kFzProd, p = q % kFzProd;
        if constexpr (!ASYNC) {
            if (p == 0) __syncthreads();                        // period t's pairs are in slot t & 1
        }
        const bool has = fz_a0(p) + t < fz_a0(p + 1);           // producer p has a pair t (uniform)
        if constexpr (ASYNC) {
            if (has)
                for (uint32_t n = 0; lds_acquire(s_prod + p) <= t; ++n) {
                    if (n == kFzSpin) {
                        if (l == 0) fz_timed_out();
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
        }
        const uint32_t* rows = s_ring + (t & 1) * kFzSlot + p * 64 * kFzRow;
        uint4 A[2];   // stale when !has: the DB words are zero then (e2m1 has no NaN/Inf)
#pragma unroll
        for (int m = 0; m < 2; ++m) A[m] = *reinterpret_cast<const uint4*>(rows + (32 * m + r) * kFzRow + 4 * h);
        if constexpr (ASYNC) lds_release(s_fold + fw, q + 1);  // after the reads: the slot may be refilled
        if (DPF_FZ_NOFOLD) return;
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4) {
            fold_v8i bo[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bo[j] = fp4_w5(u4w(B[j], t4));
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const fold_v8i ao = fp4_w7(u4w(A[m], t4));
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[m][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ao, bo[j], acc[m][j], kFoldFp4, kFoldFp4,
                                                                               0, kE8M0One, 0, kE8M0One);
            }
        }
    };
    auto nxt = [&](uint32_t q) { return q < Q ? q : Q - 1; };
    uint4 B0[2], B1[2];
    ldb(0, B0);
    ldb(1, B1);
    for (uint32_t q = 0; q < Q; q += 2) {
        fold_entry(q, B0);
        ldb(nxt(q + 2), B0);
        fold_entry(q + 1, B1);
        ldb(nxt(q + 3), B1);
    }
    // Parities -> parts[block][key][8]: folder fw holds answer words 2 fw + j.
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint32_t out = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t pbit = ((uint32_t)acc[m][j][e]) & 1u;
                const uint64_t b = __builtin_amdgcn_ballot_w64(pbit != 0);
                const uint32_t row0 = (e & 3) + 8 * (e >> 2);
                out = l == row0 ? (uint32_t)b : out;
                out = l == row0 + 4 ? (uint32_t)(b >> 32) : out;
            }
            if (l < 32) parts[((uint64_t)blockIdx.x * 64 + 32 * m + l) * 8 + 2 * fw + j] = out;
        }
}

bool pir_fused_built() { return true; }

bool pir_fused_ok(uint64_t nkeys, uint32_t stop, uint32_t prefix_bits, bool any_size) {
    if (nkeys == 0 || nkeys > 64 || stop < kFzBlockLog + 1 + prefix_bits) return false;
    const uint32_t wl = stop - 1 - kFzBlockLog - prefix_bits;   // log2 workgroups
    return (any_size || wl >= 8) && (1ull << wl) <= kFoldMaxBlocks;   // >= 256 (one per CU); parts area
}

hipError_t launch_pir_fused(const uint32_t* ek, uint32_t nkeys, uint32_t stop, uint32_t prefix_bits, uint64_t prefix,
                            const uint8_t* dbs, uint64_t nrec, uint32_t* ans, uint32_t* parts, hipStream_t st) {
    if (!pir_fused_ok(nkeys, stop, prefix_bits, true)) return hipErrorInvalidValue;
    uint32_t timed_out = 0;   // a ring wait of an earlier launch ran out (synchronises: test builds only)
    if (hipMemcpyFromSymbol(&timed_out, HIP_SYMBOL(g_fz_timeout), sizeof timed_out) != hipSuccess) return hipErrorUnknown;
    if (timed_out) {
        const uint32_t z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fz_timeout), &z, sizeof z);
        return hipErrorLaunchTimeOut;
    }
    if (nrec == 0) return hipMemsetAsync(ans, 0, (size_t)nkeys * 32, st);
    const uint64_t nsg = (nrec + 255) / 256;
    const uint32_t blocks = 1u << (stop - 1 - kFzBlockLog - prefix_bits);
    // DPF_PIR_FUSED_SYNC=1: producers and folders in lockstep (one workgroup
    // barrier per pair) instead of per-producer LDS flags (A/B runs).
    static const bool sync = [] {
        const char* e = getenv("DPF_PIR_FUSED_SYNC");
        return e && e[0] == '1';
    }();
    if (sync)
        hipLaunchKernelGGL(k_pir_fused<false>, dim3(blocks), dim3(kFzThreads), 0, st, ek, nkeys, stop, prefix_bits,
                           prefix, reinterpret_cast<const uint4*>(dbs), nsg, parts, ans, (uint64_t)nkeys * 8);
    else
        hipLaunchKernelGGL(k_pir_fused<true>, dim3(blocks), dim3(kFzThreads), 0, st, ek, nkeys, stop, prefix_bits,
                           prefix, reinterpret_cast<const uint4*>(dbs), nsg, parts, ans, (uint64_t)nkeys * 8);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    return launch_xor_parts(parts, blocks, nkeys, 64u, 8u, ans, 8, 0u, st);
}

#else
bool pir_fused_ok(uint64_t, uint32_t, uint32_t, bool) { return false; }
bool pir_fused_built() { return false; }
hipError_t launch_pir_fused(const uint32_t*, uint32_t, uint32_t, uint32_t, uint64_t, const uint8_t*, uint64_t, uint32_t*,
                            uint32_t*, hipStream_t) {
    return hipErrorInvalidValue;
}
#endif  // DPF_PIR_FUSED_KERNEL

FoldPlan plan_fold(uint64_t rec_bytes, uint32_t nkeys) {
    FoldPlan p{};
    const uint64_t c = rec_bytes / 32;
    p.cols = (c == 1 || c == 2 || c == 4 || c == 8) ? (uint32_t)c : 1;
    p.col_passes = p.cols == c ? 1 : (uint32_t)c;
    // Measured (tools/fold_bench, 2^24 x 32 B): direct is HBM-bound to 4 keys
    // (98 -> 101 us) but slower than Four-Russians from 8 (150 vs ~140 us);
    // wider records favour it longer (64 B, 16 keys: 69 us).
    p.direct = nkeys <= 4 || (p.cols >= 2 && nkeys <= (uint32_t)kDirectMaxKeys);
    const uint32_t kw_cap = p.cols >= 8 ? 1 : p.cols == 4 ? 2 : 4;
    uint32_t kw = 1;
    if (!p.direct)
        while (kw < kw_cap && 64u * kw < nkeys) kw *= 2;
    p.keys_per_pass = p.direct ? (uint32_t)kDirectMaxKeys : 64 * kw;
    p.kw = p.direct ? 0 : kw;
    return p;
}

hipError_t launch_pir_fold(const uint32_t* bits, uint64_t words_per_key, const uint8_t* db, uint64_t nrec,
                           uint64_t rec_bytes, uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st) {
    if (nkeys == 0) return hipSuccess;
    if (rec_bytes == 0 || rec_bytes % 32 != 0) return hipErrorInvalidValue;
    if (nrec == 0) return hipMemsetAsync(ans, 0, (size_t)nkeys * rec_bytes, st);
    const FoldPlan p = plan_fold(rec_bytes, nkeys);
    const uint64_t rec_u4 = rec_bytes / 16, ans_words = rec_bytes / 4;
    for (uint32_t col = 0; col < p.col_passes; ++col)
        for (uint32_t k0 = 0; k0 < nkeys; k0 += p.keys_per_pass) {
            const uint32_t nk = nkeys - k0 < p.keys_per_pass ? nkeys - k0 : p.keys_per_pass;
            FoldArgs a{bits + (uint64_t)k0 * words_per_key, words_per_key, reinterpret_cast<const uint4*>(db),
                       nrec,  rec_u4, col, nk, parts, nullptr, 0};
            if (col == 0 && k0 == 0) {
                a.zero = ans;
                a.zero_words = (uint64_t)nkeys * ans_words;
            }
            uint32_t* an = ans + (uint64_t)k0 * ans_words;
            hipError_t e;
            switch (p.cols) {
                case 2: e = fold_pass<2>(a, p.direct, (int)p.kw, an, ans_words, 0, st); break;
                case 4: e = fold_pass<4>(a, p.direct, (int)p.kw, an, ans_words, 0, st); break;
                case 8: e = fold_pass<8>(a, p.direct, (int)p.kw, an, ans_words, 0, st); break;
                default: e = fold_pass<1>(a, p.direct, (int)p.kw, an, ans_words, 8 * col, st); break;
            }
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}

}  // namespace dpfk
