// hy_bench.hip — measurement behind the hybrid PRG back end (aes_hybrid.hpp).
//
// 1. ISA issue rates on gfx950 with the clock spun up (1 s of load first) and
//    >= 20 ms per kernel: v_xor_b32, v_bitop3_b32, v_perm_b32, v_alignbit_b32,
//    v_lshlrev_b32 and 1:1 mixes, at 2 and 4 waves per SIMD.
// 2. AES-128-MMO throughput of
//      tt   : T-table only (two blocks per thread, L and R keys), 4 waves/SIMD;
//      bs   : byte-sliced only (one 8-block set per thread), 3 waves/SIMD;
//      hyNT : lockstep hybrid, NT T-table blocks + one byte-sliced set per
//             thread, 512-thread workgroups, 2 waves/SIMD.
// 3. A bit-exactness check of the hybrid core against mmo1 / aes_mmo8.
// Prints one JSON object.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <string>

#include "aes_hybrid.hpp"

using namespace dpfk;

#define CHK(x)                                                                 \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

#define REP8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

template <int KIND, int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_isa(uint32_t* out, uint32_t seed, int iters) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint32_t b = seed * 0x9e3779b9u + threadIdx.x, c = b ^ 0x5555u;
    for (int i = 0; i < iters; ++i) {
#define XOR_(n) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a##n) : "v"(b));
#define BOP_(n) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(a##n) : "v"(b), "v"(c));
#define PERM_(n) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a##n) : "v"(b), "v"(c));
#define ALIGN_(n) asm volatile("v_alignbit_b32 %0, %0, %0, 8" : "+v"(a##n));
#define LSH_(n) asm volatile("v_lshlrev_b32 %0, 8, %0" : "+v"(a##n));
#define BP_(n) BOP_(n) PERM_(n)
#define BA_(n) BOP_(n) ALIGN_(n)
        if constexpr (KIND == 0) { REP8(XOR_) REP8(XOR_) }
        if constexpr (KIND == 1) { REP8(BOP_) REP8(BOP_) }
        if constexpr (KIND == 2) { REP8(PERM_) REP8(PERM_) }
        if constexpr (KIND == 3) { REP8(ALIGN_) REP8(ALIGN_) }
        if constexpr (KIND == 4) { REP8(LSH_) REP8(LSH_) }
        if constexpr (KIND == 5) { REP8(BP_) }
        if constexpr (KIND == 6) { REP8(BA_) }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ __launch_bounds__(512, 4) void k_tt(uint32_t* out, int iters) {
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

__global__ __launch_bounds__(256, 3) void k_bs(uint32_t* out, int iters) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t X[32], O[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) X[w] = t * (2 * w + 1) + w;
    for (int i = 0; i < iters; ++i) {
        bs::aes_mmo8(X, O, 0);
#pragma unroll
        for (int w = 0; w < 32; ++w) X[w] = O[w];
    }
    uint32_t r = 0;
#pragma unroll
    for (int w = 0; w < 32; ++w) r ^= X[w];
    out[t] = r;
}

#ifndef HY_WAVES
#define HY_WAVES 2
#endif
constexpr int kHyThreads = HY_WAVES * 256;

template <int NT>
__global__ __launch_bounds__(kHyThreads, HY_WAVES) void k_hy(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk x[NT / 2], s[NT];
#pragma unroll
    for (int p = 0; p < NT / 2; ++p) x[p] = {t + p, t * 3u + p, t * 5u, t * 7u ^ p};
    uint32_t X[32], O[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) X[w] = t * (2 * w + 1) + w;
    for (int i = 0; i < iters; ++i) {
        hy::mmo_lockstep<NT>(tab, lo, x, s, X, O);
#pragma unroll
        for (int p = 0; p < NT / 2; ++p) x[p] = bxor(s[2 * p], s[2 * p + 1]);
#pragma unroll
        for (int w = 0; w < 32; ++w) X[w] = O[w];
    }
    uint32_t r = 0;
#pragma unroll
    for (int p = 0; p < NT / 2; ++p) r ^= x[p].c0 ^ x[p].c1 ^ x[p].c2 ^ x[p].c3;
#pragma unroll
    for (int w = 0; w < 32; ++w) r ^= X[w];
    out[t] = r;
}

// Bit-exactness of the lockstep core: T-table blocks vs mmo1 with the fixed
// keys, the byte-sliced set vs aes_mmo8.  Counts mismatching words.
template <int NT>
__global__ __launch_bounds__(512, 2) void k_hy_check(uint32_t* bad) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk x[NT / 2], s[NT];
#pragma unroll
    for (int p = 0; p < NT / 2; ++p) x[p] = {t * 0x9e3779b9u + p, t * 3u + p, t * 5u ^ 0xdeadbeefu, t * 7u ^ p};
    uint32_t X[32], O[32], O2[32];
#pragma unroll
    for (int w = 0; w < 32; ++w) X[w] = (t + 1) * (2 * w + 1) * 0x01000193u + w;
    hy::mmo_lockstep<NT>(tab, lo, x, s, X, O);
    uint32_t n = 0;
#pragma unroll
    for (int b = 0; b < NT; ++b) {
        const Blk r = (b & 1) ? mmo1(tab, lo, KeyFixed<true>{}, x[b >> 1]) : mmo1(tab, lo, KeyFixed<false>{}, x[b >> 1]);
        n += (r.c0 != s[b].c0) + (r.c1 != s[b].c1) + (r.c2 != s[b].c2) + (r.c3 != s[b].c3);
    }
    bs::aes_mmo8(X, O2, 0);
#pragma unroll
    for (int w = 0; w < 32; ++w) n += O[w] != O2[w];
    if (n) atomicAdd(bad, n);
}

static hipEvent_t g_a, g_b;

template <class F>
static double time_ms(F launch, int reps = 5) {
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHK(hipEventRecord(g_a, 0));
        launch();
        CHK(hipEventRecord(g_b, 0));
        CHK(hipEventSynchronize(g_b));
        float ms;
        CHK(hipEventElapsedTime(&ms, g_a, g_b));
        if (ms < best) best = ms;
    }
    return best;
}

template <class F>
static void spin(F launch, double seconds) {
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        launch();
        CHK(hipDeviceSynchronize());
    }
}

int main(int argc, char** argv) {
    const bool quick = argc > 1 && std::string(argv[1]) == "quick";
    const bool aes_only = argc > 1 && std::string(argv[1]) == "aes";
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    CHK(hipEventCreate(&g_a));
    CHK(hipEventCreate(&g_b));
    uint32_t* out;
    CHK(hipMalloc(&out, (size_t)cus * 8 * 1024 * 4));
    std::string js = "{";
    auto put = [&](const char* k, double v) {
        char buf[128];
        snprintf(buf, sizeof buf, "%s\"%s\": %.2f", js.size() > 1 ? ", " : "", k, v);
        js += buf;
    };
    // Correctness first.
    uint32_t* bad;
    CHK(hipMalloc(&bad, 4));
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_hy_check<14>, dim3(cus), dim3(512), 0, 0, bad);
    CHK(hipDeviceSynchronize());
    uint32_t nbad = 0;
    CHK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
    put("hy14_check_bad_words", nbad);

    // ISA rates: 2 / 4 waves per SIMD = 8 / 16 waves per CU.
    const int it = quick ? 20000 : 60000;
    auto isa = [&](auto kern, int waves, const char* name, double ops_per_iter) {
        const int blocks = cus * waves * 4 / 4;   // 256-thread blocks: 4 waves each
        auto L = [&] { hipLaunchKernelGGL(kern, dim3(blocks * 1), dim3(256), 0, 0, out, 1u, it); };
        spin(L, 0.3);
        const double ms = time_ms(L);
        put(name, (double)blocks * 256 * it * ops_per_iter / (ms * 1e-3) / 1e12);
    };
    if (!aes_only) {
    spin([&] { hipLaunchKernelGGL((k_isa<1, 2>), dim3(cus * 2), dim3(256), 0, 0, out, 1u, it); }, 1.0);
    isa(k_isa<0, 2>, 2, "xor_w2_Tops", 16);
    isa(k_isa<1, 2>, 2, "bitop3_w2_Tops", 16);
    isa(k_isa<2, 2>, 2, "perm_w2_Tops", 16);
    isa(k_isa<3, 2>, 2, "alignbit_w2_Tops", 16);
    isa(k_isa<4, 2>, 2, "lshl_w2_Tops", 16);
    isa(k_isa<5, 2>, 2, "bitop3+perm_w2_Tops", 16);
    isa(k_isa<6, 2>, 2, "bitop3+alignbit_w2_Tops", 16);
    isa(k_isa<1, 4>, 4, "bitop3_w4_Tops", 16);
    isa(k_isa<2, 4>, 4, "perm_w4_Tops", 16);
    isa(k_isa<5, 4>, 4, "bitop3+perm_w4_Tops", 16);
    }

    // AES-MMO rates.
    const int ai = quick ? 200 : 600;
    {
        const int blocks = cus * 2 * 4;   // several rounds of 2 WG/CU
        auto L = [&] { hipLaunchKernelGGL(k_tt, dim3(blocks), dim3(512), 0, 0, out, ai); };
        spin(L, 0.5);
        put("tt_Gblocks_s", (double)blocks * 512 * ai * 2 / (time_ms(L) * 1e-3) / 1e9);
    }
    {
        const int blocks = cus * 3 * 4;
        auto L = [&] { hipLaunchKernelGGL(k_bs, dim3(blocks), dim3(256), 0, 0, out, ai / 2); };
        spin(L, 0.5);
        put("bs_Gblocks_s", (double)blocks * 256 * (ai / 2) * 8 / (time_ms(L) * 1e-3) / 1e9);
    }
    auto hy = [&](auto kern, int nt, const char* name) {
        const int blocks = cus * 4;
        auto L = [&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(kHyThreads), 0, 0, out, ai / 8); };
        spin(L, 0.5);
        put(name, (double)blocks * kHyThreads * (ai / 8) * (nt + 8) / (time_ms(L) * 1e-3) / 1e9);
    };
    hy(k_hy<14>, 14, "hy14_Gblocks_s");
    hy(k_hy<10>, 10, "hy10_Gblocks_s");
    hy(k_hy<18>, 18, "hy18_Gblocks_s");
    CHK(hipGetLastError());
    js += "}";
    printf("%s\n", js.c_str());
    return 0;
}
