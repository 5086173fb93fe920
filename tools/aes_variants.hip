// aes_variants.hip — AES-128-MMO throughput of the two PRG back ends on
// MI355X, the measurement behind the T-table-vs-bitsliced choice (north
// star: "a choice that rocprof must justify").
//
//   ttable   : the production back end (dpf-go_amd/csrc/aes_ttable.hpp),
//              two independent MMO chains per thread (keyL and keyR, as in
//              the PRG), 512-thread workgroups, 64 KiB LDS table each.
//   bs_aes   : bitsliced AES (tools/gen_bitsliced.py, 560 v_bitop3 per
//              block), 32 blocks per lane, no feed-forward (AES only: the
//              back end's upper bound).
//   bs_mmo   : bitsliced AES-MMO (keeps the 128-word input live for the
//              feed-forward, as the GGM tree must).
// Prints JSON: G blocks/s per variant.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../dpf-go_amd/csrc/aes_ttable.hpp"
#include "aes_bitsliced.inc"

using namespace dpfk;

constexpr int kTT = 512;

__global__ __launch_bounds__(kTT, 4) void k_ttable(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk a = {t, t * 3u, t * 5u, t * 7u}, b = {t ^ 0x55u, t * 11u, t * 13u, t * 17u};
    for (int i = 0; i < iters; ++i) {
        Blk oa, ob;
        mmo2(tab, lo, KeyFixed<false>{}, a, oa, KeyFixed<true>{}, b, ob);
        a = oa;
        b = ob;
    }
    out[t] = a.c0 ^ a.c1 ^ a.c2 ^ a.c3 ^ b.c0 ^ b.c1 ^ b.c2 ^ b.c3;
}

// Shape variants of the T-table back end (same work: 2 blocks per iteration).
template <int SHAPE>
__global__ __launch_bounds__(kTT, 4) void k_tt_shape(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk a = {t, t * 3u, t * 5u, t * 7u}, b = {t ^ 0x55u, t * 11u, t * 13u, t * 17u};
    const uint32_t m = (t & 1) ? 0xffffffffu : 0u;
    for (int i = 0; i < iters; ++i) {
        if constexpr (SHAPE == 0) {          // one chain, fixed key, two MMOs back to back
            a = mmo1(tab, lo, KeyFixed<false>{}, a);
            a = mmo1(tab, lo, KeyFixed<true>{}, a);
        } else if constexpr (SHAPE == 1) {   // two independent chains written sequentially
            a = mmo1(tab, lo, KeyFixed<false>{}, a);
            b = mmo1(tab, lo, KeyFixed<true>{}, b);
        } else if constexpr (SHAPE == 2) {   // one chain, per-lane key select (k_eval's walk)
            a = mmo1(tab, lo, KeySel{m}, a);
            a = mmo1(tab, lo, KeySel{~m}, a);
        }
    }
    out[t] = a.c0 ^ a.c1 ^ a.c2 ^ a.c3 ^ b.c0 ^ b.c1 ^ b.c2 ^ b.c3;
}

__global__ __launch_bounds__(256, 2) void k_bs_aes(uint32_t* out, int iters) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s[128];
    for (int i = 0; i < 128; ++i) s[i] = (t + i) * 0x9e3779b9u;
    for (int i = 0; i < iters; ++i) aes_bs_L(s);
    uint32_t r = 0;
    for (int i = 0; i < 128; ++i) r ^= s[i];
    out[t] = r;
}

__global__ __launch_bounds__(256, 1) void k_bs_mmo(uint32_t* out, int iters) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[128], s[128];
    for (int i = 0; i < 128; ++i) x[i] = (t + i) * 0x9e3779b9u;
    for (int i = 0; i < iters; ++i) {
        for (int j = 0; j < 128; ++j) s[j] = x[j];
        aes_bs_L(s);
        for (int j = 0; j < 128; ++j) x[j] ^= s[j];
    }
    uint32_t r = 0;
    for (int i = 0; i < 128; ++i) r ^= x[i];
    out[t] = r;
}

template <class F>
static float best_ms(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    if (hipMalloc(&out, (size_t)cus * 16 * 1024 * 4) != hipSuccess) return 1;
    const int tt_blocks = cus * 2, tt_iters = 256;
    float t_tt = best_ms([&] { hipLaunchKernelGGL(k_ttable, dim3(tt_blocks), dim3(kTT), 0, 0, out, tt_iters); });
    const double tt_blk = (double)tt_blocks * kTT * tt_iters * 2;
    float t_s0 = best_ms([&] { hipLaunchKernelGGL(k_tt_shape<0>, dim3(tt_blocks), dim3(kTT), 0, 0, out, tt_iters); });
    float t_s1 = best_ms([&] { hipLaunchKernelGGL(k_tt_shape<1>, dim3(tt_blocks), dim3(kTT), 0, 0, out, tt_iters); });
    float t_s2 = best_ms([&] { hipLaunchKernelGGL(k_tt_shape<2>, dim3(tt_blocks), dim3(kTT), 0, 0, out, tt_iters); });
    const int bs_blocks = cus * 8, bs_iters = 16;
    float t_bs = best_ms([&] { hipLaunchKernelGGL(k_bs_aes, dim3(bs_blocks), dim3(256), 0, 0, out, bs_iters); });
    float t_bm = best_ms([&] { hipLaunchKernelGGL(k_bs_mmo, dim3(bs_blocks), dim3(256), 0, 0, out, bs_iters); });
    const double bs_blk = (double)bs_blocks * 256 * 32 * bs_iters;
    if (hipGetLastError() != hipSuccess) return 2;
    printf("{\"ttable_mmo_Gblocks_s\": %.1f, \"ttable_1chain_Gblocks_s\": %.1f, \"ttable_2chain_seq_Gblocks_s\": %.1f, "
           "\"ttable_keysel_Gblocks_s\": %.1f, \"bitsliced_aes_Gblocks_s\": %.1f, \"bitsliced_mmo_Gblocks_s\": %.1f}\n",
           tt_blk / t_tt / 1e6, tt_blk / t_s0 / 1e6, tt_blk / t_s1 / 1e6, tt_blk / t_s2 / 1e6, bs_blk / t_bs / 1e6,
           bs_blk / t_bm / 1e6);
    return 0;
}
