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

#include "pir_kernels_r02.hpp"

namespace dpfk {

// ---------------------------------------------------------------------------
// Four-Russians fold.  The fold is a GF(2) product
// ans[64 keys][256 bits] = S[64 x n] . DB[n x 256]; done as 8 masked XORs per
// (key, record) it is VALU-bound at 8 n B lane-ops.  Here a wave takes 64
// records (a "chunk") x 64 keys (lane = key) at a time:
//   load  : the chunk's 2 KiB as two fully coalesced 1 KiB wave loads (each
//           16-B piece of the DB is requested exactly once), staged to the
//           wave's LDS area with two conflict-free 1 KiB stores;
//   build : group g = records 4g .. 4g+3; its 16 table entries (entry e =
//           XOR of the records whose bit is set in e) are built by lanes
//           4g .. 4g+3: lane j reads half h = j&1 of the group's 4 records
//           from the staged chunk and writes entries 8a + k (a = j>>1) of
//           that half, 16 B each, over the staged chunk (a wave's LDS
//           operations complete in order, so its own reads come first);
//   lookup: each key-lane takes the group's 4 selection bits -- nibble g of
//           its 64 selection bits, exactly EvalFull's LSB-first layout --
//           as the entry index and XORs the 32-byte entry (2 ds_read_b128)
//           into its accumulator: 8 XORs per 4 records instead of 32, done
//           as 3-input XORs over two groups.
// Table rows (group g, half h) of 16 slots x 16 B; entry e sits in slot
// e ^ (e >> 3) ^ (4*(g&1) + 2*h).  A lookup (ds_read_b128, 16-lane passes
// over 64 banks) reads one row: distinct entries hit distinct bank groups,
// equal ones broadcast.  A build store (ds_write_b128, 8-lane passes over
// 32 banks) comes from lanes whose (g&1, h, a) differ: 8 distinct slots
// mod 8.  Lanes are keys, so there is no cross-lane reduction: the
// workgroup's waves combine in LDS into one 64 x 32-byte partial and
// k_xor_parts folds those.  The 8 waves of a workgroup take interleaved
// chunks of one contiguous range, so each 128-B line of a key's selection
// bits is staged once per 16 chunks.
constexpr int kM4Waves = 8;          // waves per workgroup (8 KiB of LDS each)
constexpr int kM4Groups = 16;        // 4-record groups per 64-record chunk
constexpr int kM4MaxKeys = 64;       // keys per launch (one per lane)
constexpr int kSelRow = 34;          // staged selection row: 32 words + pad -> conflict-free ds_read_b64

__device__ __forceinline__ uint4 x4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }
__device__ __forceinline__ uint4 x4_3(uint4 a, uint4 b, uint4 c) {
    return make_uint4(__builtin_amdgcn_bitop3_b32(a.x, b.x, c.x, 0x96), __builtin_amdgcn_bitop3_b32(a.y, b.y, c.y, 0x96),
                      __builtin_amdgcn_bitop3_b32(a.z, b.z, c.z, 0x96), __builtin_amdgcn_bitop3_b32(a.w, b.w, c.w, 0x96));
}
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Records may be any multiple of 32 B (rec_u4 16-byte words each); a launch
// folds one 32-byte column `col` of every record (the PIR case: rec_u4 = 2,
// col = 0).
__global__ __launch_bounds__(64 * kM4Waves, 4) void k_pir_fold4r(const uint32_t* __restrict__ bits, uint64_t wpk,
                                                              const uint4* __restrict__ db, uint64_t nrec,
                                                              uint64_t rec_u4, uint32_t col, uint32_t nkeys,
                                                              uint64_t chunks_per_block,
                                                              uint32_t* __restrict__ parts) {
    __shared__ uint4 s_tab[kM4Waves][kM4Groups * 2 * 16];
    __shared__ __attribute__((aligned(16))) uint32_t s_sel[kM4MaxKeys * kSelRow];
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t nchunks = (nrec + 63) / 64;
    const uint64_t c0 = (uint64_t)blockIdx.x * chunks_per_block;
    const uint64_t cend = c0 + chunks_per_block < nchunks ? c0 + chunks_per_block : nchunks;
    // Lanes past nkeys read key 0's bits and mask them off; loads past the
    // last record re-read the last record (selection bits are masked).
    const uint32_t keymask = l < nkeys ? ~0u : 0u;
    // Selection-bit staging: thread t copies 16 B of key t/8's 128-B line
    // (16 chunks) per batch into row t/8 (two 8-byte stores).
    const uint32_t sk = threadIdx.x >> 3, sp = threadIdx.x & 7;
    const uint32_t* srow = bits + (uint64_t)(sk < nkeys ? sk : 0) * wpk;
    auto load_sel = [&](uint64_t cb) {
        const uint64_t wo = cb * 2 + 4 * sp;
        return wo + 4 <= wpk ? *reinterpret_cast<const uint4*>(srow + wo) : make_uint4(0, 0, 0, 0);
    };
    uint4* tab = s_tab[w];
    const uint32_t g = l >> 2, j = l & 3, h = j & 1, a = j >> 1;
    const uint32_t amask = a ? ~0u : 0u;
    uint4* wrow = tab + (g * 2 + h) * 16;                         // this lane's build row
    const uint32_t wsw = (4 * (g & 1) + 2 * h) ^ a;              // slot of entry 8a + k: (8a + k) ^ wsw
    const uint4* grec = tab + 8 * g + h;                          // staged half h of record 4g (+2 per record)
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // The chunk's 2 KiB: lane l gets bytes [16l, 16l+16) of each 1 KiB half.
    auto load = [&](uint64_t cc, uint4& A, uint4& B) {
        if (cc >= nchunks) cc = nchunks - 1;
        uint64_t ra = cc * 64 + (l >> 1), rb = ra + 32;
        if (ra >= nrec) ra = nrec - 1;
        if (rb >= nrec) rb = nrec - 1;
        A = db[rec_u4 * ra + 2 * col + (l & 1)];
        B = db[rec_u4 * rb + 2 * col + (l & 1)];
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto fold = [&](uint64_t cc, uint64_t cb, const uint4& A, const uint4& B) {
        tab[l] = A;                                 // staged chunk: record r half hh at 16-B slot 2r + hh
        tab[64 + l] = B;
        wave_sync();
        const uint4 R0 = grec[0], R1 = grec[2], R2 = grec[4], R3 = grec[6];
        wave_sync();
        // entries 8a + k = (XOR of R0/R1/R2 by the bits of k) ^ (a ? R3 : 0)
        const uint4 R3m = make_uint4(R3.x & amask, R3.y & amask, R3.z & amask, R3.w & amask);
        const uint4 R01 = x4(R0, R1);
        const uint32_t b8 = 8 * a;
        wrow[(b8 + 0) ^ wsw] = R3m;
        wrow[(b8 + 1) ^ wsw] = x4(R0, R3m);
        wrow[(b8 + 2) ^ wsw] = x4(R1, R3m);
        wrow[(b8 + 3) ^ wsw] = x4(R01, R3m);
        wrow[(b8 + 4) ^ wsw] = x4(R2, R3m);
        wrow[(b8 + 5) ^ wsw] = x4_3(R2, R0, R3m);
        wrow[(b8 + 6) ^ wsw] = x4_3(R2, R1, R3m);
        wrow[(b8 + 7) ^ wsw] = x4_3(R01, R2, R3m);
        wave_sync();
        uint2 sel = *reinterpret_cast<const uint2*>(&s_sel[l * kSelRow + 2 * (cc - cb)]);
        const uint64_t valid = cc < cend ? nrec - cc * 64 : 0;   // records of this chunk below nrec
        sel.x &= keymask & (valid >= 32 ? ~0u : (1u << valid) - 1u);
        sel.y &= keymask & (valid >= 64 ? ~0u : valid <= 32 ? 0u : (1u << (valid - 32)) - 1u);
        // Pre-swizzle the nibbles: slot = e ^ (e >> 3) ^ 4 (odd groups); the half-1 slot is that ^ 2.
        const uint32_t zx = sel.x ^ ((sel.x >> 3) & 0x11111111u) ^ 0x40404040u;
        const uint32_t zy = sel.y ^ ((sel.y >> 3) & 0x11111111u) ^ 0x40404040u;
#pragma unroll
        for (int gg = 0; gg < kM4Groups; gg += 2) {
            const uint32_t z = gg < 8 ? zx : zy;
            const uint32_t s0 = (z >> (4 * (gg & 7))) & 15u, s1 = (z >> (4 * ((gg + 1) & 7))) & 15u;
            const uint4 lo0 = tab[(gg * 2 + 0) * 16 + s0], hi0 = tab[(gg * 2 + 1) * 16 + (s0 ^ 2)];
            const uint4 lo1 = tab[(gg * 2 + 2) * 16 + s1], hi1 = tab[(gg * 2 + 3) * 16 + (s1 ^ 2)];
            acc[0] = x3(acc[0], lo0.x, lo1.x); acc[1] = x3(acc[1], lo0.y, lo1.y);
            acc[2] = x3(acc[2], lo0.z, lo1.z); acc[3] = x3(acc[3], lo0.w, lo1.w);
            acc[4] = x3(acc[4], hi0.x, hi1.x); acc[5] = x3(acc[5], hi0.y, hi1.y);
            acc[6] = x3(acc[6], hi0.z, hi1.z); acc[7] = x3(acc[7], hi0.w, hi1.w);
        }
        wave_sync();
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
        *reinterpret_cast<uint2*>(&s_sel[sk * kSelRow + 4 * sp]) = make_uint2(snext.x, snext.y);
        *reinterpret_cast<uint2*>(&s_sel[sk * kSelRow + 4 * sp + 2]) = make_uint2(snext.z, snext.w);
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

// ans[k * ans_words + i] ^= XOR over workgroups of parts[wg][k][i] (k <
// nkeys, i < 8).  Block (x, y): 256 answer words x parts y, y + gridDim.y,
// ...; one atomicXor each.
__global__ __launch_bounds__(256) void k_xor_parts(const uint32_t* __restrict__ parts, uint64_t nparts,
                                                   uint32_t nkeys, uint32_t* __restrict__ ans, uint64_t ans_words) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;   // word index k * 8 + i
    if (t >= nkeys * 8) return;
    uint32_t v = 0;
    for (uint64_t p = blockIdx.y; p < nparts; p += gridDim.y) v ^= parts[p * kM4MaxKeys * 8 + t];
    if (v) atomicXor(ans + (t >> 3) * ans_words + (t & 7), v);
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
                           uint64_t rec_bytes, uint32_t nkeys, uint32_t* ans, uint32_t* parts, hipStream_t st) {
    if (nrec == 0 || nkeys == 0) return hipSuccess;
    if (rec_bytes == 0 || rec_bytes % 32 != 0) return hipErrorInvalidValue;
    const uint64_t nchunks = (nrec + 63) / 64;
    // Two resident workgroups (16 waves) per CU, each over a contiguous chunk range.
    uint64_t blocks = (uint64_t)cu_count_fold() * 2;
    if (blocks > kFoldMaxBlocks) blocks = kFoldMaxBlocks;
    uint64_t cpb = (nchunks + blocks - 1) / blocks;
    cpb = (cpb + 2 * kM4Waves - 1) / (2 * kM4Waves) * (2 * kM4Waves);   // whole 16-chunk batches
    blocks = (nchunks + cpb - 1) / cpb;
    const uint32_t ys = (uint32_t)(blocks < 64 ? blocks : 64);
    const uint64_t rec_u4 = rec_bytes / 16, ans_words = rec_bytes / 4;
    for (uint32_t col = 0; col < rec_bytes / 32; ++col)
        for (uint32_t k0 = 0; k0 < nkeys; k0 += kM4MaxKeys) {
            const uint32_t nk = nkeys - k0 < (uint32_t)kM4MaxKeys ? nkeys - k0 : (uint32_t)kM4MaxKeys;
            hipLaunchKernelGGL(k_pir_fold4r, dim3((uint32_t)blocks), dim3(64 * kM4Waves), 0, st,
                               bits + (uint64_t)k0 * words_per_key, words_per_key, reinterpret_cast<const uint4*>(db),
                               nrec, rec_u4, col, nk, cpb, parts);
            hipLaunchKernelGGL(k_xor_parts, dim3((nk * 8 + 255) / 256, ys), dim3(256), 0, st, parts, blocks, nk,
                               ans + (uint64_t)k0 * ans_words + 8 * col, ans_words);
        }
    return hipGetLastError();
}

}  // namespace dpfk
