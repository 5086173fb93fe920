// lane16_mmo.hip — r06 microbenchmark: the latency of one dependent
// AES-128-MMO step (aes128MMO, /root/reference/dpf/aes_amd64.s:50-82) with
// one block spread over a 16-lane DPP row, one state byte per lane, so that a
// round is ONE LDS T-table lookup per lane plus DPP data movement:
//   lane (d, r) = (L >> 2, L & 3) holds byte r of column (d + r) mod 4, so the
//   four T-table terms of output column d sit in quad d (ShiftRows folded into
//   the layout): lookup Te_r[b], quad XOR-reduce (2 DPP), XOR the round key,
//   fetch byte r of column (d + r) mod 4 from quad (d + r) mod 4 (row_ror by
//   4, 8, 12 + selects).  The quad form of the product's shared walk
//   (tree_ops.hpp walk_step_quad: one column per lane, 4 lookups) takes ~1.1 us
//   per level; the one-lane form 1.85 us (profiles/r06/walk_latency.log).
// Table: the product's LDS layout (aes_ttable.hpp: Te0 and rotl8(Te0), 32 lane
// copies, conflict-free).  Prints one JSON line; checks the 4 blocks of the
// wave against the host T-table math.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lane16_mmo.hip -o tools/bin/lane16_mmo
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../dpf-go_amd/csrc/aes_ttable.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

using namespace dpfk;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int kQ1032 = 0xB1, kQ2301 = 0x4E;                 // quad_perm [1,0,3,2], [2,3,0,1]
constexpr int kRor4 = 0x124, kRor8 = 0x128, kRor12 = 0x12C; // row_ror:4/8/12

// The word held by quad (d + r) mod 4 of this row: row_ror:k gives lane L the
// value of lane (L - k) mod 16, so quad d + r is row_ror by 16 - 4r (measured:
// the other direction fails the check below).
__device__ __forceinline__ uint32_t from_quad(uint32_t w, uint32_t r) {
    const uint32_t a4 = dpp<kRor4>(w), a8 = dpp<kRor8>(w), a12 = dpp<kRor12>(w);
    const uint32_t lo = (r & 1) ? a12 : w;
    const uint32_t hi = (r & 1) ? a4 : a8;
    return (r & 2) ? hi : lo;
}

__global__ __launch_bounds__(64) void k_lane16(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t reps,
                                               uint32_t ror_dir) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lane = threadIdx.x & 63, L = lane & 15, d = L >> 2, r = L & 3;
    const uint32_t lo = (lane & 31) * 4;
    const uint32_t blk = threadIdx.x >> 4;
    const uint4 X = in[blk];
    // this lane's column word of the block (column d), for the feed-forward
    uint32_t x = d == 0 ? X.x : d == 1 ? X.y : d == 2 ? X.z : X.w;
    const dpfc::RoundKeys& K = dpfc::kRkL;
    uint32_t rk[11];
#pragma unroll
    for (int t = 0; t < 11; ++t) rk[t] = d == 0 ? K.w[4 * t] : d == 1 ? K.w[4 * t + 1] : d == 2 ? K.w[4 * t + 2] : K.w[4 * t + 3];
    const uint32_t sh16 = (r & 2) ? 16u : 0u, rot8 = (r & 1) ? 128u : 0u;
    for (uint32_t it = 0; it < reps; ++it) {
        // round 0: byte r of (column (d + r) ^ rk0 of that column) = byte r of from_quad(x ^ rk0)
        uint32_t w = x ^ rk[0];
        uint32_t b = (from_quad(w, r) >> (8 * r)) & 255u;
#pragma unroll
        for (int t = 1; t < 10; ++t) {
            uint32_t v = *reinterpret_cast<const uint32_t*>(tab + b * 256 + lo + rot8);   // Te0 or rotl8(Te0)
            v = __builtin_amdgcn_alignbit(v, v, sh16);                                     // rotr 16 = rotl 16 (rows 2, 3)
            v ^= dpp<kQ1032>(v);
            v ^= dpp<kQ2301>(v);                                                           // column d of the round
            w = v ^ rk[t];
            b = (from_quad(w, r) >> (8 * r)) & 255u;
        }
        // final round: S[b] is byte 1 of Te0[b]; lane (d, r) holds output byte (d, r)
        const uint32_t sb = (*reinterpret_cast<const uint32_t*>(tab + b * 256 + lo) >> 8) & 255u;
        uint32_t o = sb << (8 * r);
        o |= dpp<kQ1032>(o);
        o |= dpp<kQ2301>(o);
        x = o ^ rk[10] ^ x;                                                                // MMO feed-forward
    }
    if (r == 0) reinterpret_cast<uint32_t*>(&out[blk])[d] = x;
    (void)ror_dir;
}

// The product's quad form (aes_ttable.hpp mmo_quad: lane j of a quad holds
// column j, 4 lookups per round) on 16 blocks per wave, left key.
__global__ __launch_bounds__(64) void k_quad(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t reps) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t j = threadIdx.x & 3, blk = (threadIdx.x >> 2) & 3;   // 4 distinct blocks, 4 copies each
    const uint32_t lo = (threadIdx.x & 31) * 4;
    const QuadKeys k = quad_keys(j);
    const uint4 X = in[blk];
    uint32_t x = j == 0 ? X.x : j == 1 ? X.y : j == 2 ? X.z : X.w;
    for (uint32_t it = 0; it < reps; ++it) x = mmo_quad(tab, lo, k, 0u, x);
    if (threadIdx.x < 16) reinterpret_cast<uint32_t*>(&out[blk])[j] = x;
}

static uint32_t hrotl(uint32_t x, int n) { return n ? (x << n) | (x >> (32 - n)) : x; }
static void host_mmo(uint32_t x[4]) {
    const dpfc::RoundKeys& K = dpfc::kRkL;
    auto T = [](int i, uint32_t e) { return hrotl(dpfc::kTe0.v[e], 8 * i); };
    uint32_t s[4] = {x[0] ^ K.w[0], x[1] ^ K.w[1], x[2] ^ K.w[2], x[3] ^ K.w[3]};
    for (int rr = 1; rr < 10; ++rr) {
        uint32_t n[4];
        for (int j = 0; j < 4; ++j)
            n[j] = T(0, s[j] & 255) ^ T(1, (s[(j + 1) & 3] >> 8) & 255) ^ T(2, (s[(j + 2) & 3] >> 16) & 255) ^
                   T(3, s[(j + 3) & 3] >> 24) ^ K.w[4 * rr + j];
        memcpy(s, n, 16);
    }
    uint32_t o[4];
    for (int j = 0; j < 4; ++j)
        o[j] = ((uint32_t)dpfc::kSbox.v[s[j] & 255] | ((uint32_t)dpfc::kSbox.v[(s[(j + 1) & 3] >> 8) & 255] << 8) |
                ((uint32_t)dpfc::kSbox.v[(s[(j + 2) & 3] >> 16) & 255] << 16) |
                ((uint32_t)dpfc::kSbox.v[s[(j + 3) & 3] >> 24] << 24)) ^ K.w[40 + j];
    for (int j = 0; j < 4; ++j) x[j] ^= o[j];
}

int main() {
    std::vector<uint32_t> in(16);
    uint64_t z = 0x243F6A8885A308D3ull;
    for (auto& w : in) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; w = (uint32_t)z; }
    uint32_t *d_in, *d_out;
    CK(hipMalloc(&d_in, 64));
    CK(hipMalloc(&d_out, 64));
    CK(hipMemcpy(d_in, in.data(), 64, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_us = [&](uint32_t reps) {
        float best = 1e30f;
        for (int t = 0; t < 5; ++t) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_lane16, dim3(1), dim3(64), 0, 0, (const uint4*)d_in, (uint4*)d_out, reps, 0u);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return best * 1e3;
    };
    auto time_quad = [&](uint32_t reps) {
        float best = 1e30f;
        for (int t = 0; t < 5; ++t) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_quad, dim3(1), dim3(64), 0, 0, (const uint4*)d_in, (uint4*)d_out, reps);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return best * 1e3;
    };
    time_us(50);
    const double per = (time_us(400) - time_us(200)) / 200.0;
    const double perq = (time_quad(400) - time_quad(200)) / 200.0;
    hipLaunchKernelGGL(k_quad, dim3(1), dim3(64), 0, 0, (const uint4*)d_in, (uint4*)d_out, 3u);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> gq(16);
    CK(hipMemcpy(gq.data(), d_out, 64, hipMemcpyDeviceToHost));
    int badq = 0;
    for (int b = 0; b < 4; ++b) {
        uint32_t x[4] = {in[4 * b], in[4 * b + 1], in[4 * b + 2], in[4 * b + 3]};
        for (int i = 0; i < 3; ++i) host_mmo(x);
        badq += memcmp(x, &gq[4 * b], 16) != 0;
    }
    hipLaunchKernelGGL(k_lane16, dim3(1), dim3(64), 0, 0, (const uint4*)d_in, (uint4*)d_out, 3u, 0u);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> got(16);
    CK(hipMemcpy(got.data(), d_out, 64, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int b = 0; b < 4; ++b) {
        uint32_t x[4] = {in[4 * b], in[4 * b + 1], in[4 * b + 2], in[4 * b + 3]};
        for (int i = 0; i < 3; ++i) host_mmo(x);
        bad += memcmp(x, &got[4 * b], 16) != 0;
        if (b == 0) fprintf(stderr, "want %08x %08x %08x %08x got %08x %08x %08x %08x\n", x[0], x[1], x[2], x[3], got[0], got[1], got[2], got[3]);
    }
    printf("{\"lane16_us_per_dependent_mmo\": %.4f, \"blocks_bad\": %d, \"quad_us_per_dependent_mmo\": %.4f, "
           "\"quad_blocks_bad\": %d}\n", per, bad, perq, badq);
    return bad || badq ? 1 : 0;
}
