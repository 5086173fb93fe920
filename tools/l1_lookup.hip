// l1_lookup.hip — can the vector-memory path (L1 / TA) serve table lookups
// beside LDS?  The tree kernel is LDS-lookup bound (~88% of the measured
// ds_read_b32 rate); lookups served from a small global table through
// buffer_load ... idxen use a different pipe.  Measures:
//   lds_chain       : ds_read_b32 lookups, production split-row layout
//   l1_chain_<B>    : buffer_load_dword idxen lookups into a B-byte table
//   l1_ubyte        : buffer_load_ubyte idxen lookups into the 256-B S-box
//   mix             : both, independent chains in the same loop
//   aes_g<N>_l<L>   : AES-MMO (two chains, as the PRG) with N of the 4
//                     columns of every full round served from global Te0..Te3
//                     (4 KiB) and, if L, the last round from the global S-box
// Prints one JSON object (G lookups/s, G blocks/s).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../dpf-go_amd/csrc/aes_ttable.hpp"

using namespace dpfk;

constexpr int kTT = 512;

__device__ uint32_t sload32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.ptr.buffer.load.i32");
__device__ uint8_t sload8(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.ptr.buffer.load.i8");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int stride) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)stride, 1 << 20, 0x00020000);
}

template <int K>
__device__ __forceinline__ uint32_t byte_of(uint32_t x) {
    if constexpr (K == 0) return x & 0xffu;
    else if constexpr (K == 3) return x >> 24;
    else return __builtin_amdgcn_perm(x, 0u, 0x0c0c0c00u | (4u + K));
}

// ---------------------------------------------------------------- raw rates
template <int ILP>
__global__ __launch_bounds__(kTT, 4) void k_lds_chain(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[ILP];
    for (int j = 0; j < ILP; ++j) x[j] = t * 2654435761u + j;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < ILP; ++j) x[j] = tl<1>(tab, x[j], lo) + x[j];
    uint32_t r = 0;
    for (int j = 0; j < ILP; ++j) r ^= x[j];
    out[t] = r;
}

template <int ILP, int TB>
__global__ __launch_bounds__(kTT, 4) void k_l1_chain(const uint32_t* g, uint32_t* out, int iters) {
    const auto r = rsrc(g, 4);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[ILP];
    for (int j = 0; j < ILP; ++j) x[j] = t * 2654435761u + j;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < ILP; ++j) {
            uint32_t idx = TB == 1024 ? byte_of<1>(x[j]) : (x[j] >> 22);   // 256 or 1024 entries
            x[j] = sload32(r, (int)idx, 0, 0, 0) + x[j];
        }
    uint32_t s = 0;
    for (int j = 0; j < ILP; ++j) s ^= x[j];
    out[t] = s;
}

template <int ILP>
__global__ __launch_bounds__(kTT, 4) void k_l1_ubyte(const uint32_t* g, uint32_t* out, int iters) {
    const auto r = rsrc(g, 1);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[ILP];
    for (int j = 0; j < ILP; ++j) x[j] = t * 2654435761u + j;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int j = 0; j < ILP; ++j) x[j] = (uint32_t)sload8(r, (int)byte_of<1>(x[j]), 0, 0, 0) * 0x01010101u + x[j] * 3u;
    uint32_t s = 0;
    for (int j = 0; j < ILP; ++j) s ^= x[j];
    out[t] = s;
}

template <int NL, int NG>
__global__ __launch_bounds__(kTT, 4) void k_mix(const uint32_t* g, uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const auto r = rsrc(g, 4);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x[NL], y[NG];
    for (int j = 0; j < NL; ++j) x[j] = t * 2654435761u + j;
    for (int j = 0; j < NG; ++j) y[j] = t * 40503u + 7 * j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NL; ++j) x[j] = tl<1>(tab, x[j], lo) + x[j];
#pragma unroll
        for (int j = 0; j < NG; ++j) y[j] = sload32(r, (int)byte_of<1>(y[j]), 0, 0, 0) + y[j];
    }
    uint32_t s = 0;
    for (int j = 0; j < NL; ++j) s ^= x[j];
    for (int j = 0; j < NG; ++j) s ^= y[j];
    out[t] = s;
}

// ------------------------------------------------------------- hybrid AES
// Global tables: Te0 | Te1 | Te2 | Te3 (4 x 1 KiB, stride 4) and S (256 B).
struct GTabs {
    __amdgpu_buffer_rsrc_t te, sb, sw;   // sw: S[x] as 32-bit words (1 KiB)
};

template <int R, int NG, class K>
__device__ __forceinline__ void round_hyb(const uint8_t* tab, uint32_t lo, const GTabs& gt, const K& k, Blk& s) {
    auto col_lds = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk16) {
        uint32_t ta = tl<0>(tab, a, lo), tb = tl<1, true>(tab, b, lo), tc = tl<2>(tab, c, lo),
                 td = tl<3, true>(tab, d, lo);
        return xor3(ta, tb, rotl(xor3(tc, td, rk16), 16));
    };
    auto col_g = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
        uint32_t ta = sload32(gt.te, (int)byte_of<0>(a), 0, 0, 0), tb = sload32(gt.te, (int)byte_of<1>(b), 0, 1024, 0),
                 tc = sload32(gt.te, (int)byte_of<2>(c), 0, 2048, 0), td = sload32(gt.te, (int)byte_of<3>(d), 0, 3072, 0);
        return xor3(xor3(ta, tb, tc), td, rk);
    };
    uint32_t n[4];
    const uint32_t c[4] = {s.c0, s.c1, s.c2, s.c3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j < NG) n[j] = col_g(c[j], c[(j + 1) & 3], c[(j + 2) & 3], c[(j + 3) & 3], k.template get<4 * R + 0>() * 0 + (j == 0 ? k.template get<4 * R + 0>() : j == 1 ? k.template get<4 * R + 1>() : j == 2 ? k.template get<4 * R + 2>() : k.template get<4 * R + 3>()));
        else n[j] = col_lds(c[j], c[(j + 1) & 3], c[(j + 2) & 3], c[(j + 3) & 3], j == 0 ? k.template get16<4 * R + 0>() : j == 1 ? k.template get16<4 * R + 1>() : j == 2 ? k.template get16<4 * R + 2>() : k.template get16<4 * R + 3>());
    }
    s.c0 = n[0]; s.c1 = n[1]; s.c2 = n[2]; s.c3 = n[3];
}

template <int LG, class K>
__device__ __forceinline__ void last_g(const GTabs& gt, const K& k, Blk& s) {
    auto ld = [&](uint32_t i) -> uint32_t {
        if constexpr (LG == 1) return sload8(gt.sb, (int)i, 0, 0, 0);
        else return sload32(gt.sw, (int)i, 0, 0, 0);
    };
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
        uint32_t sa = ld(byte_of<0>(a)), sb = ld(byte_of<1>(b)), sc = ld(byte_of<2>(c)), sd = ld(byte_of<3>(d));
        uint32_t p = __builtin_amdgcn_perm(sb, sa, 0x0c0c0400u);   // {sa, sb, 0, 0}
        uint32_t q = __builtin_amdgcn_perm(sd, sc, 0x04000c0cu);   // {0, 0, sc, sd}
        return __builtin_amdgcn_bitop3_b32(p, q, rk, kOrXor);
    };
    uint32_t n0 = col(s.c0, s.c1, s.c2, s.c3, k.template get<40>());
    uint32_t n1 = col(s.c1, s.c2, s.c3, s.c0, k.template get<41>());
    uint32_t n2 = col(s.c2, s.c3, s.c0, s.c1, k.template get<42>());
    uint32_t n3 = col(s.c3, s.c0, s.c1, s.c2, k.template get<43>());
    s.c0 = n0; s.c1 = n1; s.c2 = n2; s.c3 = n3;
}

template <int R, int NG, class K>
__device__ __forceinline__ void rounds_hyb(const uint8_t* tab, uint32_t lo, const GTabs& gt, const K& k, Blk& s) {
    if constexpr (R <= 9) {
        round_hyb<R, NG>(tab, lo, gt, k, s);
        rounds_hyb<R + 1, NG>(tab, lo, gt, k, s);
    }
}

template <int NG, int LG, class K>
__device__ __forceinline__ Blk mmo_hyb(const uint8_t* tab, uint32_t lo, const GTabs& gt, const K& k, Blk x) {
    Blk s = bxor(x, bkey4(k.template get<0>(), k.template get<1>(), k.template get<2>(), k.template get<3>()));
    rounds_hyb<1, NG>(tab, lo, gt, k, s);
    if constexpr (LG != 0) last_g<LG>(gt, k, s);
    else aes_last(tab, lo, k, s);
    return bxor(s, x);
}

template <int NG, int LG>
__global__ __launch_bounds__(kTT, 4) void k_aes_hyb(const uint32_t* g, uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const GTabs gt{rsrc(g, 4), rsrc(g + 1024, 1), rsrc(g + 1088, 4)};
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    Blk a = {t, t * 3u, t * 5u, t * 7u}, b = {t ^ 0x55u, t * 11u, t * 13u, t * 17u};
    for (int i = 0; i < iters; ++i) {
        a = mmo_hyb<NG, LG>(tab, lo, gt, KeyFixed<false>{}, a);
        b = mmo_hyb<NG, LG>(tab, lo, gt, KeyFixed<true>{}, b);
    }
    out[t] = a.c0 ^ a.c1 ^ a.c2 ^ a.c3 ^ b.c0 ^ b.c1 ^ b.c2 ^ b.c3;
}

// Host check of one hybrid MMO against the LDS-only path.
template <int NG, int LG>
__global__ __launch_bounds__(kTT, 4) void k_aes_check(const uint32_t* g, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabWords];
    fill_table(s_tab);
    const uint8_t* tab = reinterpret_cast<const uint8_t*>(s_tab);
    const uint32_t lo = (threadIdx.x & 31u) * 4u;
    const GTabs gt{rsrc(g, 4), rsrc(g + 1024, 1), rsrc(g + 1088, 4)};
    const uint32_t t = threadIdx.x;
    Blk x = {t * 0x9e3779b9u, t * 3u + 1, t ^ 0xabcdefu, t * 77u};
    Blk p = mmo1(tab, lo, KeyFixed<true>{}, x), q = mmo_hyb<NG, LG>(tab, lo, gt, KeyFixed<true>{}, x);
    out[t] = (p.c0 ^ q.c0) | (p.c1 ^ q.c1) | (p.c2 ^ q.c2) | (p.c3 ^ q.c3);
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
    const int blocks = cus * 2, iters = 1024;
    const double lanes = (double)blocks * kTT;
    uint32_t* out;
    uint32_t* g;
    if (hipMalloc(&out, (size_t)blocks * kTT * 4) != hipSuccess) return 1;
    // Te0..Te3, then the S-box bytes
    uint32_t host[1024 + 64 + 256];
    for (int i = 0; i < 256; ++i)
        for (int r = 0; r < 4; ++r) host[r * 256 + i] = crotl(dpfc::kTe0.v[i], 8 * r);
    uint8_t* sb = reinterpret_cast<uint8_t*>(host + 1024);
    for (int i = 0; i < 256; ++i) sb[i] = (uint8_t)(dpfc::kTe0.v[i] >> 8);
    for (int i = 0; i < 256; ++i) host[1088 + i] = sb[i];
    if (hipMalloc(&g, sizeof host) != hipSuccess) return 1;
    (void)hipMemcpy(g, host, sizeof host, hipMemcpyHostToDevice);

    uint32_t chk[kTT];
    int bad = 0;
#define CHECK_HYB(NG, LG)                                                            \
    hipLaunchKernelGGL((k_aes_check<NG, LG>), dim3(1), dim3(kTT), 0, 0, g, out);    \
    (void)hipMemcpy(chk, out, sizeof chk, hipMemcpyDeviceToHost);                   \
    for (int i = 0; i < kTT; ++i) bad += chk[i] != 0;
    CHECK_HYB(1, 0) CHECK_HYB(2, 1) CHECK_HYB(4, 1) CHECK_HYB(0, 2)

    auto rate = [&](float ms, double per_lane) { return lanes * per_lane / ms / 1e6; };
    float t;
    printf("{\"check_mismatches\": %d", bad);
    t = best_ms([&] { hipLaunchKernelGGL(k_lds_chain<8>, dim3(blocks), dim3(kTT), 0, 0, out, iters); });
    printf(", \"lds_chain8_Glookups_s\": %.1f", rate(t, 8.0 * iters));
    t = best_ms([&] { hipLaunchKernelGGL((k_l1_chain<8, 1024>), dim3(blocks), dim3(kTT), 0, 0, g, out, iters); });
    printf(", \"l1_chain8_1KiB_Glookups_s\": %.1f", rate(t, 8.0 * iters));
    t = best_ms([&] { hipLaunchKernelGGL((k_l1_chain<8, 4096>), dim3(blocks), dim3(kTT), 0, 0, g, out, iters); });
    printf(", \"l1_chain8_4KiB_Glookups_s\": %.1f", rate(t, 8.0 * iters));
    t = best_ms([&] { hipLaunchKernelGGL(k_l1_ubyte<8>, dim3(blocks), dim3(kTT), 0, 0, g + 1024, out, iters); });
    printf(", \"l1_ubyte8_Glookups_s\": %.1f", rate(t, 8.0 * iters));
    t = best_ms([&] { hipLaunchKernelGGL((k_mix<8, 2>), dim3(blocks), dim3(kTT), 0, 0, g, out, iters); });
    printf(", \"mix_8lds_2l1_Glookups_s\": %.1f", rate(t, 10.0 * iters));
    t = best_ms([&] { hipLaunchKernelGGL((k_mix<8, 4>), dim3(blocks), dim3(kTT), 0, 0, g, out, iters); });
    printf(", \"mix_8lds_4l1_Glookups_s\": %.1f", rate(t, 12.0 * iters));
    const int ai = 128;
#define AES_HYB(NG, LG)                                                                                    \
    t = best_ms([&] { hipLaunchKernelGGL((k_aes_hyb<NG, LG>), dim3(blocks), dim3(kTT), 0, 0, g, out, ai); }); \
    printf(", \"aes_g%d_l%d_Gblocks_s\": %.1f", NG, (int)LG, rate(t, 2.0 * ai));
    AES_HYB(0, 0) AES_HYB(0, 1) AES_HYB(0, 2) AES_HYB(1, 0)
    printf("}\n");
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
