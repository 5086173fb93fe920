// tt_bench.hip — T-table AES-MMO layout experiments and VALU issue rates on
// gfx950, with the clock spun up and every kernel timed in 3 interleaved
// rounds (max reported).
//
//   tt2   : production layout (aes_ttable.hpp): Te0 + rotl8(Te0) in one 64 KiB
//           table, one v_alignbit per column; 512-thread WGs, 2 per CU.
//   tt4   : four tables Te0..Te3 (128 KiB: rows [Te0|Te1] then [Te2|Te3]),
//           no rotation, column = xor3(Ta, Tb, xor3(Tc, Td, rk)); one
//           1024-thread WG per CU (4 waves/SIMD).
//   tt4w2 : tt4 with 512-thread WGs (1 per CU, 2 waves/SIMD).
//   isa_* : lane-op rates of single instructions (8 chains per lane).
// Prints one JSON object.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <string>
#include <vector>

#include "../dpf-go_amd/csrc/aes_ttable.hpp"

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

template <int KIND>
__global__ __launch_bounds__(256) void k_isa(uint32_t* out, uint32_t seed, int iters) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint32_t b = seed * 0x9e3779b9u + threadIdx.x, c = b ^ 0x5555u;
    for (int i = 0; i < iters; ++i) {
#define XOR_(n) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(a##n) : "v"(b));
#define AND_(n) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(a##n) : "v"(b));
#define BOP_(n) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(a##n) : "v"(b), "v"(c));
#define PERM_(n) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a##n) : "v"(b), "v"(c));
#define ALIGN_(n) asm volatile("v_alignbit_b32 %0, %0, %0, 8" : "+v"(a##n));
#define LSH_(n) asm volatile("v_lshrrev_b32_e32 %0, 8, %0" : "+v"(a##n));
#define BFE_(n) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a##n));
#define XOR3_(n) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(a##n) : "v"(b));
        if constexpr (KIND == 0) { REP8(XOR_) REP8(XOR_) }
        if constexpr (KIND == 1) { REP8(AND_) REP8(AND_) }
        if constexpr (KIND == 2) { REP8(BOP_) REP8(BOP_) }
        if constexpr (KIND == 3) { REP8(PERM_) REP8(PERM_) }
        if constexpr (KIND == 4) { REP8(ALIGN_) REP8(ALIGN_) }
        if constexpr (KIND == 5) { REP8(LSH_) REP8(LSH_) }
        if constexpr (KIND == 6) { REP8(BFE_) REP8(BFE_) }
        if constexpr (KIND == 7) { REP8(XOR3_) REP8(XOR3_) }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ __launch_bounds__(512, 4) void k_tt2(uint32_t* out, int iters) {
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

// ---- four-table layout ----------------------------------------------------
constexpr uint32_t kTab4Words = 2 * kTabWords;   // 128 KiB

__device__ __forceinline__ void fill_table4(uint32_t* tab) {
    for (uint32_t i = threadIdx.x; i < 2 * 256 * 16; i += blockDim.x) {
        const uint32_t reg = i / (256 * 16), e = (i / 16) % 256, q = i & 15;
        const uint32_t k = 2 * reg + (q >= 8 ? 1 : 0);        // table Te_k
        const uint32_t v = rotl(c_te0.v[e], 8 * k);
        reinterpret_cast<uint4*>(tab)[reg * 4096 + e * 16 + q] = make_uint4(v, v, v, v);
    }
    __syncthreads();
}

// Te_K[byte K of x]: region K/2, half K&1; lo01 = lane*4, lo23 = lane*4 | 0x10000.
template <int K>
__device__ __forceinline__ uint32_t tl4(const uint8_t* tab, uint32_t x, uint32_t lo01, uint32_t lo23) {
    const uint32_t a = K < 2 ? __builtin_amdgcn_perm(x, lo01, 0x0c0c0000u | ((4u + K) << 8))
                             : __builtin_amdgcn_perm(x, lo23, 0x0c020000u | ((4u + K) << 8));
    return *reinterpret_cast<const uint32_t*>(tab + a + ((K & 1) ? 128 : 0));
}

template <int R, class K>
__device__ __forceinline__ void round4(const uint8_t* tab, uint32_t l01, uint32_t l23, const K& k, Blk& s) {
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
        return xor3(tl4<0>(tab, a, l01, l23), tl4<1>(tab, b, l01, l23),
                    xor3(tl4<2>(tab, c, l01, l23), tl4<3>(tab, d, l01, l23), rk));
    };
    uint32_t n0 = col(s.c0, s.c1, s.c2, s.c3, k.template get<4 * R + 0>());
    uint32_t n1 = col(s.c1, s.c2, s.c3, s.c0, k.template get<4 * R + 1>());
    uint32_t n2 = col(s.c2, s.c3, s.c0, s.c1, k.template get<4 * R + 2>());
    uint32_t n3 = col(s.c3, s.c0, s.c1, s.c2, k.template get<4 * R + 3>());
    s.c0 = n0; s.c1 = n1; s.c2 = n2; s.c3 = n3;
}

template <int R, class KA, class KB>
__device__ __forceinline__ void rounds4(const uint8_t* tab, uint32_t l01, uint32_t l23, const KA& ka, Blk& a,
                                        const KB& kb, Blk& b) {
    if constexpr (R <= 9) {
        round4<R>(tab, l01, l23, ka, a);
        round4<R>(tab, l01, l23, kb, b);
        rounds4<R + 1>(tab, l01, l23, ka, a, kb, b);
    }
}

template <class KA, class KB>
__device__ __forceinline__ void mmo2_4(const uint8_t* tab, uint32_t l01, uint32_t l23, const KA& ka, Blk xa, Blk& oa,
                                       const KB& kb, Blk xb, Blk& ob) {
    Blk a = bxor(xa, bkey4(ka.template get<0>(), ka.template get<1>(), ka.template get<2>(), ka.template get<3>()));
    Blk b = bxor(xb, bkey4(kb.template get<0>(), kb.template get<1>(), kb.template get<2>(), kb.template get<3>()));
    rounds4<1>(tab, l01, l23, ka, a, kb, b);
    aes_last(tab, l01, ka, a);   // region 0 rows hold Te0 at offset 0: same as the 2-table layout
    aes_last(tab, l01, kb, b);
    oa = bxor(a, xa);
    ob = bxor(b, xb);
}

template <int THREADS, int WAVES>
__global__ __launch_bounds__(THREADS, WAVES) void k_tt4(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTab4Words];
    fill_table4(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t l01 = (threadIdx.x & 31u) * 4u, l23 = l01 | 0x10000u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk a = {t, t * 3u, t * 5u, t * 7u}, b = {t ^ 0x55u, t * 11u, t * 13u, t * 17u};
    for (int i = 0; i < iters; ++i) {
        Blk oa, ob;
        mmo2_4(tab, l01, l23, KeyFixed<false>{}, a, oa, KeyFixed<true>{}, b, ob);
        a = oa;
        b = ob;
    }
    out[t] = a.c0 ^ a.c1 ^ a.c2 ^ a.c3 ^ b.c0 ^ b.c1 ^ b.c2 ^ b.c3;
}

// Bit-exactness of tt4 against tt2 (same inputs, one MMO pair).
__global__ __launch_bounds__(1024, 4) void k_tt4_check(uint32_t* bad) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTab4Words];
    fill_table4(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t l01 = (threadIdx.x & 31u) * 4u, l23 = l01 | 0x10000u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk a = {t * 0x9e3779b9u, t * 3u + 1, t ^ 0xdeadbeefu, t * 7u}, b = {t ^ 0x55u, t * 11u, t * 13u, ~t};
    Blk oa, ob;
    mmo2_4(tab, l01, l23, KeyFixed<false>{}, a, oa, KeyFixed<true>{}, b, ob);
    // reference: the 2-table layout's rows are region 0 with Te1 = rotl8(Te0) beside Te0
    const Blk ra = mmo1(tab, l01, KeyFixed<false>{}, a), rb = mmo1(tab, l01, KeyFixed<true>{}, b);
    const uint32_t n = (ra.c0 != oa.c0) + (ra.c1 != oa.c1) + (ra.c2 != oa.c2) + (ra.c3 != oa.c3) +
                       (rb.c0 != ob.c0) + (rb.c1 != ob.c1) + (rb.c2 != ob.c2) + (rb.c3 != ob.c3);
    if (n) atomicAdd(bad, n);
}

static hipEvent_t g_a, g_b;

static double time_ms(const std::function<void()>& launch) {
    CHK(hipEventRecord(g_a, 0));
    launch();
    CHK(hipEventRecord(g_b, 0));
    CHK(hipEventSynchronize(g_b));
    float ms;
    CHK(hipEventElapsedTime(&ms, g_a, g_b));
    return ms;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    CHK(hipEventCreate(&g_a));
    CHK(hipEventCreate(&g_b));
    uint32_t* out;
    CHK(hipMalloc(&out, (size_t)cus * 16 * 1024 * 4));
    uint32_t* bad;
    CHK(hipMalloc(&bad, 4));
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_tt4_check, dim3(cus), dim3(1024), 0, 0, bad);
    CHK(hipDeviceSynchronize());
    uint32_t nbad = 0;
    CHK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));

    struct Case {
        std::string name;
        std::function<void()> launch;
        double units;   // lane-ops or AES blocks per launch
        double best = 0;
    };
    const int it = 40000, ai = 400;
    std::vector<Case> cs;
    auto isa = [&](const char* name, void (*k)(uint32_t*, uint32_t, int)) {
        const int blocks = cus * 4;   // 16 waves per CU
        cs.push_back({name, [=] { hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, it); },
                      (double)blocks * 256 * it * 16});
    };
    isa("isa_xor_Tops", k_isa<0>);
    isa("isa_and_Tops", k_isa<1>);
    isa("isa_bitop3_Tops", k_isa<2>);
    isa("isa_perm_Tops", k_isa<3>);
    isa("isa_alignbit_Tops", k_isa<4>);
    isa("isa_lshr_Tops", k_isa<5>);
    isa("isa_bfe_Tops", k_isa<6>);
    isa("isa_xor_e64_Tops", k_isa<7>);
    cs.push_back({"tt2_Gblocks_s", [=] { hipLaunchKernelGGL(k_tt2, dim3(cus * 8), dim3(512), 0, 0, out, ai); },
                  (double)cus * 8 * 512 * ai * 2});
    cs.push_back({"tt4_Gblocks_s",
                  [=] { hipLaunchKernelGGL((k_tt4<1024, 4>), dim3(cus * 4), dim3(1024), 0, 0, out, ai); },
                  (double)cus * 4 * 1024 * ai * 2});
    cs.push_back({"tt4w2_Gblocks_s",
                  [=] { hipLaunchKernelGGL((k_tt4<512, 2>), dim3(cus * 8), dim3(512), 0, 0, out, ai); },
                  (double)cus * 8 * 512 * ai * 2});
    // spin up the clock
    {
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 1.0) {
            cs[2].launch();
            CHK(hipDeviceSynchronize());
        }
    }
    for (int round = 0; round < 3; ++round)
        for (auto& c : cs) {
            c.launch();
            const double ms = time_ms(c.launch);
            const double rate = c.units / (ms * 1e-3) / (c.name.rfind("isa", 0) == 0 ? 1e12 : 1e9);
            c.best = std::max(c.best, rate);
        }
    CHK(hipGetLastError());
    printf("{\"tt4_check_bad_words\": %u", nbad);
    for (auto& c : cs) printf(", \"%s\": %.2f", c.name.c_str(), c.best);
    printf("}\n");
    return 0;
}
