// valu_peak.hip — measures the chip's int32 VALU issue rate on gfx950, the
// denominator of the PRG roofline (SURVEY §8d asks for an on-box check of
// v_xor_b32 / v_bitop3_b32 before quoting a ceiling).
//
// Each lane runs 8 independent dependency chains of one instruction
// (inline asm, so nothing folds), 2048 threads per CU, grid = 8 x CUs.
// Prints lane-ops/s for v_xor_b32, v_bitop3_b32 (3-input XOR), v_perm_b32,
// v_alignbit_b32, and ds_read_b32 from a per-lane LDS table (the T-table
// lookup), as JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                            \
        }                                                                        \
    } while (0)

constexpr int kIters = 4096;

#define REP8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

template <int KIND>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
             a6 = a0 * 17, a7 = a0 * 19;
    uint32_t b = seed * 0x9e3779b9u + threadIdx.x, c = b ^ 0x5555u;
    for (int i = 0; i < kIters; ++i) {
#define XOR_(n) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a##n) : "v"(b));
#define BOP_(n) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(a##n) : "v"(b), "v"(c));
#define PERM_(n) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a##n) : "v"(b), "v"(c));
#define ALIGN_(n) asm volatile("v_alignbit_b32 %0, %0, %0, 8" : "+v"(a##n));
#define ANDOR_(n) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a##n) : "v"(b), "v"(c));
#define LSHLOR_(n) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a##n) : "v"(b));
#define BFE_(n) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a##n));
#define SDWA_(n) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a##n) : "v"(b));
#define LSHR_(n) asm volatile("v_lshrrev_b32 %0, 8, %0" : "+v"(a##n));
#define CND_(n) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##n) : "v"(b));
        if constexpr (KIND == 0) { REP8(XOR_) REP8(XOR_) }
        if constexpr (KIND == 1) { REP8(BOP_) REP8(BOP_) }
        if constexpr (KIND == 2) { REP8(PERM_) REP8(PERM_) }
        if constexpr (KIND == 3) { REP8(ALIGN_) REP8(ALIGN_) }
        if constexpr (KIND == 4) { REP8(ANDOR_) REP8(ANDOR_) }
        if constexpr (KIND == 5) { REP8(LSHLOR_) REP8(LSHLOR_) }
        if constexpr (KIND == 6) { REP8(BFE_) REP8(BFE_) }
        if constexpr (KIND == 7) { REP8(SDWA_) REP8(SDWA_) }
        if constexpr (KIND == 8) { REP8(LSHR_) REP8(LSHR_) }
        if constexpr (KIND == 9) { REP8(CND_) REP8(CND_) }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// ds_read_b32 lookups, one private table copy per lane (the engine's layout).
__global__ __launch_bounds__(1024) void k_lds(uint32_t* out, uint32_t seed) {
    __shared__ uint32_t tab[256 * 64];
    for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x) tab[i] = i * 0x9e3779b9u;
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 63) * 4;
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = (seed + threadIdx.x * 8 + j) * 2654435761u;
    // Issue priority by progress (dpf_kernels.hip prio_step): without it a
    // SIMD's waves finish oldest-first and the tail of the one round runs on
    // fewer waves (r01's 16.44 T lookups/s was measured that way).
    __builtin_amdgcn_s_setprio(3);
    for (int i = 0; i < kIters; ++i) {
        if (i == kIters * 3 / 4) __builtin_amdgcn_s_setprio(2);
        if (i == kIters * 7 / 8) __builtin_amdgcn_s_setprio(1);
        if (i == kIters * 15 / 16) __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t a = __builtin_amdgcn_perm(x[j], lo, 0x0c0c0500u);
            x[j] ^= *(const uint32_t*)((const char*)tab + a);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t a = __builtin_amdgcn_perm(x[j], lo, 0x0c0c0600u);
            x[j] ^= *(const uint32_t*)((const char*)tab + a);
        }
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ __launch_bounds__(1024) void k_lds64(uint32_t* out, uint32_t seed) {
    __shared__ uint2 tab[256 * 32];
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) tab[i] = make_uint2(i * 0x9e3779b9u, i);
    __syncthreads();
    const uint32_t lo = (threadIdx.x & 31) * 8;
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = (seed + threadIdx.x * 8 + j) * 2654435761u;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t a = __builtin_amdgcn_perm(x[j], lo, 0x0c0c0500u);
            uint2 v = *(const uint2*)((const char*)tab + a);
            x[j] ^= v.x + v.y;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t a = __builtin_amdgcn_perm(x[j], lo, 0x0c0c0600u);
            uint2 v = *(const uint2*)((const char*)tab + a);
            x[j] ^= v.x + v.y;
        }
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <class F>
double time_ms(F launch) {
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
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8, threads = 256;
    uint32_t* out;
    CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
    const double lane_ops = (double)blocks * threads * kIters * 16;
    double t_xor = time_ms([&] { hipLaunchKernelGGL(k_valu<0>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_bop = time_ms([&] { hipLaunchKernelGGL(k_valu<1>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_prm = time_ms([&] { hipLaunchKernelGGL(k_valu<2>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_aln = time_ms([&] { hipLaunchKernelGGL(k_valu<3>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    const int lblocks = cus * 2;   // 64 KiB LDS each -> 2 per CU
    double t_lds = time_ms([&] { hipLaunchKernelGGL(k_lds, dim3(lblocks), dim3(1024), 0, 0, out, 1u); });
    const double lds_ops = (double)lblocks * 1024 * kIters * 16;
    double t_lds64 = time_ms([&] { hipLaunchKernelGGL(k_lds64, dim3(lblocks), dim3(1024), 0, 0, out, 1u); });
    double t_andor = time_ms([&] { hipLaunchKernelGGL(k_valu<4>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_lshlor = time_ms([&] { hipLaunchKernelGGL(k_valu<5>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_bfe = time_ms([&] { hipLaunchKernelGGL(k_valu<6>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_sdwa = time_ms([&] { hipLaunchKernelGGL(k_valu<7>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_lshr = time_ms([&] { hipLaunchKernelGGL(k_valu<8>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    double t_cnd = time_ms([&] { hipLaunchKernelGGL(k_valu<9>, dim3(blocks), dim3(threads), 0, 0, out, 1u); });
    CHK(hipGetLastError());
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %d, "
           "\"v_xor_b32_Tops\": %.2f, \"v_bitop3_b32_Tops\": %.2f, \"v_perm_b32_Tops\": %.2f, "
           "\"v_alignbit_b32_Tops\": %.2f, \"ds_read_b32_lookup_G_per_s\": %.1f, \"ds_read_b64_lookup_G_per_s\": %.1f, "
           "\"v_and_or_b32_Tops\": %.2f, \"v_lshl_or_b32_Tops\": %.2f, \"v_bfe_u32_Tops\": %.2f, "
           "\"v_mov_b32_sdwa_Tops\": %.2f, \"v_lshrrev_b32_Tops\": %.2f, \"v_cndmask_b32_Tops\": %.2f}\n",
           p.gcnArchName, cus, p.clockRate / 1000, lane_ops / t_xor / 1e9, lane_ops / t_bop / 1e9,
           lane_ops / t_prm / 1e9, lane_ops / t_aln / 1e9, lds_ops / t_lds / 1e6, lds_ops / t_lds64 / 1e6,
           lane_ops / t_andor / 1e9, lane_ops / t_lshlor / 1e9, lane_ops / t_bfe / 1e9, lane_ops / t_sdwa / 1e9,
           lane_ops / t_lshr / 1e9, lane_ops / t_cnd / 1e9);
    return 0;
}
