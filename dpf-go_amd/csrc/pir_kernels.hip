// pir_kernels.hip — 2-server PIR answer fold on gfx950 (last
// row: a build-only operator with no reference counterpart).
//
//   ans_k = XOR over records i with bit_i(EvalFull(key_k)) = 1 of DB[i]
//
// Phase 1 (dpf_kernels.hip, subtree EvalFull) writes each key's selection
// bits for this GPU's DB slice into HBM: bits[k][i/32] bit (i%32), which is
// exactly EvalFull's packed LSB-first byte layout read as little-endian u32.
// Phase 2 (k_pir_fold, here) reads every DB record once from HBM and folds it
// into all B answers:
//   - a wave owns 64*R consecutive records; lane l holds records
//     chunk + 64 j + l (j < R) in registers (R*8 words), loaded coalesced;
//   - for each key: acc ^= rec_j & -(bit) -> one v_bitop3 per word;
//   - the 8 accumulator words are XOR-reduced across the wave with a
//     register-halving butterfly (10 lane exchanges instead of 48);
//   - the 4 waves of a workgroup combine in LDS and the workgroup issues one
//     32-bit atomicXor per answer word.
// The bitwise fold is the GF(2) inner product; it is kept as VALU AND/XOR,
// not reshaped into an int8 MFMA GEMM (8x data expansion for no gain).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pir_kernels.hpp"

namespace dpfk {

constexpr int kFoldWaves = 4;
#ifndef DPF_FOLD_R
#define DPF_FOLD_R 8
#endif
#ifndef DPF_FOLD_SHFL
#define DPF_FOLD_SHFL 0
#endif
constexpr int kFoldR = DPF_FOLD_R;   // records per lane held in registers (build knob: 8 or 16)
constexpr int kFoldMaxB = 64;    // keys per launch (LDS combine buffer)

__device__ __forceinline__ uint32_t xorsel(uint32_t acc, uint32_t rec, uint32_t m) {
    return __builtin_amdgcn_bitop3_b32(acc, rec, m, 0x78);   // acc ^ (rec & m): 0xF0 ^ (0xCC & 0xAA)
}

// DPP lane moves (VALU, no LDS): row_ror:8 = lane ^ 8 within a 16-lane row,
// row_half_mirror = lane -> 7 - lane within 8, quad_perm [1,0,3,2] / [2,3,0,1].
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_half_mirror(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_quad(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}

// XOR-reduce v[0..7] over the 64 lanes; afterwards lane l holds the full
// reduction of word (l >> 3) & 7 in v[0].  Register-halving butterfly on
// VALU-only lane exchanges: v_permlane32_swap (lanes l <-> l^32), then
// v_permlane16_swap (l <-> l^16 within each half), DPP row_ror:8 (l^8),
// and a 3-step DPP reduction inside each group of 8 lanes.
__device__ __forceinline__ uint32_t wave_xor8_dpp(uint32_t v[8]) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 4; ++i) {       // word i + 4*(l>>5)
        auto r = __builtin_amdgcn_permlane32_swap(v[i], v[4 + i], false, false);
        v[i] = r[0] ^ r[1];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {       // word i + 2*((l>>4)&1) + 4*(l>>5)
        auto r = __builtin_amdgcn_permlane16_swap(v[i], v[2 + i], false, false);
        v[i] = r[0] ^ r[1];
    }
    const bool hi = l & 8;              // word (l>>3)&7
    const uint32_t keep = hi ? v[1] : v[0], send = hi ? v[0] : v[1];
    uint32_t x = keep ^ dpp_ror8(send);
    x ^= dpp_half_mirror(x);            // pairs (j, 7-j) within 8 lanes
    x ^= dpp_quad<0xB1>(x);             // quad_perm [1,0,3,2]
    x ^= dpp_quad<0x4E>(x);             // quad_perm [2,3,0,1]
    return x;
}

// Reference form of the same reduction over __shfl_xor (kept for A/B).
__device__ __forceinline__ uint32_t wave_xor8(uint32_t v[8]) {
    const int l = threadIdx.x & 63;
    // step 1: lanes l and l^32 trade halves, each keeps 4 words
    {
        const bool hi = l & 32;
        uint32_t keep[4], send[4];
        for (int i = 0; i < 4; ++i) {
            keep[i] = hi ? v[4 + i] : v[i];
            send[i] = hi ? v[i] : v[4 + i];
        }
        for (int i = 0; i < 4; ++i) v[i] = keep[i] ^ __shfl_xor(send[i], 32);
    }
    // step 2: l ^ 16, keep 2 words
    {
        const bool hi = l & 16;
        uint32_t keep[2], send[2];
        for (int i = 0; i < 2; ++i) {
            keep[i] = hi ? v[2 + i] : v[i];
            send[i] = hi ? v[i] : v[2 + i];
        }
        for (int i = 0; i < 2; ++i) v[i] = keep[i] ^ __shfl_xor(send[i], 16);
    }
    // step 3: l ^ 8, keep 1 word
    {
        const bool hi = l & 8;
        uint32_t keep = hi ? v[1] : v[0], send = hi ? v[0] : v[1];
        v[0] = keep ^ __shfl_xor(send, 8);
    }
    // word index now = 4*(l>>5&1) + 2*(l>>4&1) + (l>>3&1); finish within 8 lanes
    v[0] ^= __shfl_xor(v[0], 4);
    v[0] ^= __shfl_xor(v[0], 2);
    v[0] ^= __shfl_xor(v[0], 1);
    return v[0];
}

__global__ __launch_bounds__(64 * kFoldWaves) void k_pir_fold(const uint32_t* __restrict__ bits,
                                                              uint64_t words_per_key,
                                                              const uint4* __restrict__ db, uint64_t nrec,
                                                              uint32_t nkeys, uint32_t* __restrict__ ans) {
    constexpr int kWordsPerWave = 64 * kFoldR / 32;
    constexpr int kWordsPerBlock = kFoldWaves * kWordsPerWave;
    __shared__ uint32_t s_part[kFoldWaves][kFoldMaxB][8];
    __shared__ uint32_t s_bits[kFoldMaxB][kWordsPerBlock];
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t chunk = ((uint64_t)blockIdx.x * kFoldWaves + w) * (64 * kFoldR);
    // Every key's selection words for this workgroup's records, one
    // coalesced pass (64 words = 256 B per key), into LDS.
    {
        const uint64_t wb = (uint64_t)blockIdx.x * kWordsPerBlock;
        for (uint32_t i = threadIdx.x; i < nkeys * kWordsPerBlock; i += blockDim.x) {
            const uint32_t k = i / kWordsPerBlock, o = i % kWordsPerBlock;
            s_bits[k][o] = wb + o < words_per_key ? bits[k * words_per_key + wb + o] : 0u;
        }
    }
    uint32_t rec[kFoldR][8];
#pragma unroll
    for (int j = 0; j < kFoldR; ++j) {
        const uint64_t r = chunk + 64 * j + l;
        if (r < nrec) {
            uint4 a = db[2 * r], b = db[2 * r + 1];
            rec[j][0] = a.x; rec[j][1] = a.y; rec[j][2] = a.z; rec[j][3] = a.w;
            rec[j][4] = b.x; rec[j][5] = b.y; rec[j][6] = b.z; rec[j][7] = b.w;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) rec[j][i] = 0;
        }
    }
    __syncthreads();
    const uint32_t sh = 31 - (l & 31);
    const int wbase = w * kWordsPerWave + (l >> 5);
    for (uint32_t k = 0; k < nkeys; ++k) {
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < kFoldR; ++j) {
            const uint32_t word = s_bits[k][wbase + 2 * j];
            const uint32_t m = (uint32_t)((int32_t)(word << sh) >> 31);   // -(bit l of the word)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = xorsel(acc[i], rec[j][i], m);
        }
#if DPF_FOLD_SHFL
        const uint32_t red = wave_xor8(acc);
#else
        const uint32_t red = wave_xor8_dpp(acc);
#endif
        if ((l & 7) == 0) s_part[w][k][l >> 3] = red;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nkeys * 8; i += blockDim.x) {
        const uint32_t k = i >> 3, word = i & 7;
        uint32_t v = 0;
#pragma unroll
        for (int ww = 0; ww < kFoldWaves; ++ww) v ^= s_part[ww][k][word];
        if (v) atomicXor(ans + k * 8 + word, v);
    }
}

hipError_t launch_pir_fold(const uint32_t* bits, uint64_t words_per_key, const uint8_t* db, uint64_t nrec,
                           uint32_t nkeys, uint32_t* ans, hipStream_t st) {
    if (nrec == 0 || nkeys == 0) return hipSuccess;
    const uint64_t per_block = (uint64_t)64 * kFoldR * kFoldWaves;
    const uint64_t blocks = (nrec + per_block - 1) / per_block;
    for (uint32_t k0 = 0; k0 < nkeys; k0 += kFoldMaxB) {
        const uint32_t nk = nkeys - k0 < (uint32_t)kFoldMaxB ? nkeys - k0 : (uint32_t)kFoldMaxB;
        hipLaunchKernelGGL(k_pir_fold, dim3((uint32_t)blocks), dim3(64 * kFoldWaves), 0, st,
                           bits + (uint64_t)k0 * words_per_key, words_per_key,
                           reinterpret_cast<const uint4*>(db), nrec, nk, ans + (uint64_t)k0 * 8);
    }
    return hipGetLastError();
}

}  // namespace dpfk
