// pir_kernels.hip — 2-server PIR answer fold on gfx950 (last
// row: a build-only operator with no reference counterpart).
//
//   ans_k = XOR over records i with bit_i(EvalFull(key_k)) = 1 of DB[i]
//
// Phase 1 (dpf_kernels.hip, subtree EvalFull) writes each key's selection
// bits for this GPU's DB slice into HBM: bits[k][i/32] bit (i%32), which is
// exactly EvalFull's packed LSB-first byte layout read as little-endian u32.
// Phase 2 (k_pir_fold4r, here) reads every DB record once from HBM and folds
// it into all B answers with a Four-Russians table per 4 records (below).
// The fold is the GF(2) inner product; it stays bitwise (VALU XOR + LDS
// table lookups), not reshaped into an int8 MFMA GEMM (8x data expansion).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../dpf-go_amd/csrc/pir_kernels.hpp"

namespace dpfk {

// ---------------------------------------------------------------------------
// Four-Russians fold.  The fold is a GF(2) product
// ans[64 keys][256 bits] = S[64 x n] . DB[n x 256]; done as 8 masked XORs per
// (key, record) it is VALU-bound at 8 n B lane-ops.  Here a wave takes 64
// records (a "chunk") x 64 keys (lane = key) at a time:
//   build : each of the chunk's 16 groups of 4 records gets a 16-entry table
//           of all XOR combinations (entry e = XOR of the records b with bit b
//           of e set), built in registers by the 4 lanes of a quad (DPP quad
//           broadcasts) and stored to a wave-private LDS table (8 KiB);
//   lookup: each key-lane uses its 4 selection bits of a group as the entry
//           index and XORs the 32-byte entry (2 ds_read_b128) into its
//           accumulator: 8 XORs per 4 records instead of 32.
// Lanes are keys, so there is no cross-lane reduction: the workgroup's waves
// combine in LDS into one 64 x 32-byte partial and k_xor_parts folds those.
// The 8 waves of a workgroup take interleaved chunks of one contiguous range,
// so each 128-B line of a key's selection bits is consumed by the workgroup
// within two iterations (L1-resident) rather than by one wave over 16.
// LDS layout of a wave's table: [group 16][half 2][slot 16] x 16 B, entry e of
// group g in slot pi(e) ^ (g & 1), pi(e) = e ^ ((e >> 2) & 2).  A lookup reads
// one (group, half) row of 256 B: distinct entries hit distinct banks (b128:
// bank (a/4) mod 64), equal ones broadcast.  The build stores lane (quad q,
// position p) entry 4p + j; pi makes the 8 lanes of each b128 store group hit
// 8 distinct 16-B bank groups (stores: bank (a/4) mod 32).
#ifndef DPF_FOLD_EXP
#define DPF_FOLD_EXP 0   // measurement knob (tools/fold_bench.hip): 1 no table stores, 2 no lookups, 3 no record loads
#endif
constexpr int kM4Waves = 8;          // waves per workgroup (8 KiB of LDS table each)
constexpr int kM4Groups = 16;        // 4-record groups per 64-record chunk
constexpr int kM4MaxKeys = 64;       // keys per launch (one per lane)
constexpr int kSelRow = 36;          // staged selection row: 32 words + pad (2-way ds_read_b64)

template <int SRC>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t x) {
    // quad_perm [SRC, SRC, SRC, SRC]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, SRC * 0x55, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t m4_slot(uint32_t e, uint32_t g) { return e ^ ((e >> 2) & 2u) ^ (g & 1u); }

__global__ __launch_bounds__(64 * kM4Waves, 4) void k_pir_fold4r(const uint32_t* __restrict__ bits, uint64_t wpk,
                                                              const uint4* __restrict__ db, uint64_t nrec,
                                                              uint32_t nkeys, uint64_t chunks_per_block,
                                                              uint32_t* __restrict__ parts) {
    __shared__ uint4 s_tab[kM4Waves][kM4Groups * 2 * 16];
    __shared__ __attribute__((aligned(16))) uint32_t s_sel[kM4MaxKeys][kSelRow];
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t nchunks = (nrec + 63) / 64;
    const uint64_t c0 = (uint64_t)blockIdx.x * chunks_per_block;
    const uint64_t cend = c0 + chunks_per_block < nchunks ? c0 + chunks_per_block : nchunks;
    // Lanes past nkeys read key 0's bits and mask them off; lanes past the
    // last record read the last record and the selection bits are masked.
    const uint32_t keymask = l < nkeys ? ~0u : 0u;
    // Selection-bit staging: thread t copies 16 B of key t/8's 128-B line
    // (16 chunks) per batch; rows padded to kSelRow words.
    const uint32_t sk = threadIdx.x >> 3, sp = threadIdx.x & 7;
    const uint32_t* srow = bits + (uint64_t)(sk < nkeys ? sk : 0) * wpk;
    auto load_sel = [&](uint64_t cb) {
        const uint64_t wo = cb * 2 + 4 * sp;
        return wo + 4 <= wpk ? *reinterpret_cast<const uint4*>(srow + wo) : make_uint4(0, 0, 0, 0);
    };
    uint4* tab = s_tab[w];
    const uint32_t q = l >> 2, p = l & 3;
    const uint32_t m2 = (p & 1) ? ~0u : 0u, m3 = (p & 2) ? ~0u : 0u;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // Chunk cc's record (lane l) and selection words; branch-free so the
    // loads of the next chunk stay in flight while this one is folded.
    auto load = [&](uint64_t cc, uint4& a, uint4& b) {
        if (cc >= nchunks) cc = nchunks - 1;
        uint64_t r = cc * 64 + l;
        if (r >= nrec) r = nrec - 1;
#if DPF_FOLD_EXP == 3
        a = make_uint4((uint32_t)r, (uint32_t)r * 3u, (uint32_t)r * 5u, (uint32_t)r * 7u);
        b = make_uint4((uint32_t)r * 9u, (uint32_t)r * 11u, (uint32_t)r * 13u, (uint32_t)r * 15u);
#else
        a = db[2 * r];
        b = db[2 * r + 1];
#endif
    };
    // Fold chunk cc (record words x, selection words sel) into acc.
    auto fold = [&](uint64_t cc, uint64_t cb, const uint4& ra, const uint4& rb) {
        const uint32_t x[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
        uint2 sel = *reinterpret_cast<const uint2*>(&s_sel[l][2 * (cc - cb)]);
        const uint64_t valid = cc < cend ? nrec - cc * 64 : 0;   // records of this chunk below nrec
        sel.x &= keymask & (valid >= 32 ? ~0u : (1u << valid) - 1u);
        sel.y &= keymask & (valid >= 64 ? ~0u : valid <= 32 ? 0u : (1u << (valid - 32)) - 1u);
        // Build: lane p of quad q computes entries 4p + j (j < 4) of group q,
        // E = A[j] ^ B[p] with A = {0, r0, r1, r0^r1}, B = {0, r2, r3, r2^r3};
        // one 16-byte half at a time.
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t e[4][4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t xi = x[4 * h + i];
                const uint32_t r0 = quad_bcast<0>(xi), r1 = quad_bcast<1>(xi);
                const uint32_t r2 = quad_bcast<2>(xi), r3 = quad_bcast<3>(xi);
                const uint32_t bp = __builtin_amdgcn_bitop3_b32(r2, m2, r3 & m3, 0x6a);   // (r2 & m2) ^ c
                e[0][i] = bp;
                e[1][i] = r0 ^ bp;
                e[2][i] = r1 ^ bp;
                e[3][i] = __builtin_amdgcn_bitop3_b32(r0, r1, bp, 0x96);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (DPF_FOLD_EXP == 1 && e[j][0] != 0x12345678u) continue;
                tab[(q * 2 + h) * 16 + m4_slot(4 * p + j, q)] = make_uint4(e[j][0], e[j][1], e[j][2], e[j][3]);
            }
        }
        // LDS operations of one wave complete in order: once the compiler
        // keeps program order (wavefront-scope fence), the lookups below see
        // the whole table and the next chunk's stores follow these reads.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if DPF_FOLD_EXP == 2
        acc[0] ^= sel.x; acc[1] ^= sel.y;
#pragma unroll
        for (int g = 0; g < 0; ++g) {
#else
#pragma unroll
        for (int g = 0; g < kM4Groups; ++g) {
#endif
            const uint32_t word = g < 8 ? sel.x : sel.y;
            const uint32_t slot = m4_slot((word >> (4 * (g & 7))) & 15u, g);
            const uint4 lo = tab[(g * 2 + 0) * 16 + slot], hi = tab[(g * 2 + 1) * 16 + slot];
            acc[0] ^= lo.x; acc[1] ^= lo.y; acc[2] ^= lo.z; acc[3] ^= lo.w;
            acc[4] ^= hi.x; acc[5] ^= hi.y; acc[6] ^= hi.z; acc[7] ^= hi.w;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // Batches of 16 chunks (one 128-B line of every key's selection bits);
    // each wave folds chunks cb + w and cb + 8 + w of a batch.  Record loads
    // ping-pong between two explicit buffers (no register copies at the loop
    // latch), so the next chunk's records are in flight during a fold.
    uint4 a0, b0, a1, b1;
    if (c0 + w < cend) load(c0 + w, a0, b0);
    uint4 snext = c0 < cend ? load_sel(c0) : make_uint4(0, 0, 0, 0);
    for (uint64_t cb = c0; cb < cend; cb += 2 * kM4Waves) {
        __syncthreads();                                  // previous batch's selection reads are done
        *reinterpret_cast<uint4*>(&s_sel[sk][4 * sp]) = snext;
        __syncthreads();
        if (cb + 2 * kM4Waves < cend) snext = load_sel(cb + 2 * kM4Waves);
        const uint64_t c = cb + w;
        if (c < cend) {
            load(c + kM4Waves, a1, b1);
            fold(c, cb, a0, b0);
        }
        if (c + kM4Waves < cend) {
            load(c + 2 * kM4Waves, a0, b0);
            fold(c + kM4Waves, cb, a1, b1);
        }
    }
    // Combine the workgroup's waves in LDS (reusing the tables), one partial per workgroup.
    __syncthreads();
    uint32_t* comb = reinterpret_cast<uint32_t*>(&s_tab[0][0]);   // [wave][key][8]
#pragma unroll
    for (int i = 0; i < 8; ++i) comb[(w * 64 + l) * 8 + i] = acc[i];
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < kM4MaxKeys * 8; t += blockDim.x) {
        uint32_t v = 0;
#pragma unroll
        for (int ww = 0; ww < kM4Waves; ++ww) v ^= comb[ww * kM4MaxKeys * 8 + t];
        parts[(uint64_t)blockIdx.x * kM4MaxKeys * 8 + t] = v;
    }
}

// ans[k][i] ^= XOR over workgroups of parts[wg][k][i] (k < nkeys).  Block
// (x, y): 256 answer words x parts y, y + gridDim.y, ...; one atomicXor each.
__global__ __launch_bounds__(256) void k_xor_parts(const uint32_t* __restrict__ parts, uint64_t nparts,
                                                   uint32_t nkeys, uint32_t* __restrict__ ans) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;   // word index k * 8 + i
    if (t >= nkeys * 8) return;
    uint32_t v = 0;
    for (uint64_t p = blockIdx.y; p < nparts; p += gridDim.y) v ^= parts[p * kM4MaxKeys * 8 + t];
    if (v) atomicXor(ans + t, v);
}

static int cu_count_fold() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return cus;
}

constexpr uint64_t kFoldMaxBlocks = 2048;   // partials area: max fold workgroups per launch

uint64_t pir_fold_parts_bytes() { return kFoldMaxBlocks * kM4MaxKeys * 32; }

hipError_t launch_pir_fold(const uint32_t* bits, uint64_t words_per_key, const uint8_t* db, uint64_t nrec,
                           uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st) {
    if (nrec == 0 || nkeys == 0) return hipSuccess;
    const uint64_t nchunks = (nrec + 63) / 64;
    // Two resident workgroups (16 waves) per CU, each over a contiguous chunk range.
    uint64_t blocks = (uint64_t)cu_count_fold() * 2;
    if (blocks > kFoldMaxBlocks) blocks = kFoldMaxBlocks;
    uint64_t cpb = (nchunks + blocks - 1) / blocks;
    cpb = (cpb + 2 * kM4Waves - 1) / (2 * kM4Waves) * (2 * kM4Waves);   // whole 16-chunk batches
    blocks = (nchunks + cpb - 1) / cpb;
    const uint32_t ys = (uint32_t)(blocks < 64 ? blocks : 64);
    for (uint32_t k0 = 0; k0 < nkeys; k0 += kM4MaxKeys) {
        const uint32_t nk = nkeys - k0 < (uint32_t)kM4MaxKeys ? nkeys - k0 : (uint32_t)kM4MaxKeys;
        hipLaunchKernelGGL(k_pir_fold4r, dim3((uint32_t)blocks), dim3(64 * kM4Waves), 0, st,
                           bits + (uint64_t)k0 * words_per_key, words_per_key, reinterpret_cast<const uint4*>(db),
                           nrec, nk, cpb, parts);
        hipLaunchKernelGGL(k_xor_parts, dim3((nk * 8 + 255) / 256, ys), dim3(256), 0, st, parts, blocks, nk,
                           ans + (uint64_t)k0 * 8);
    }
    return hipGetLastError();
}

}  // namespace dpfk
