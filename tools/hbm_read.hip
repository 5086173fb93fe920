// hbm_read.hip — achievable HBM read rate on this MI355X: XOR-reduce a
// 512 MiB buffer (the configs[4] DB size) with 16-byte loads, several grid
// shapes, steady clock.  The fold's bar: it reads the same bytes (+ 128 MiB of
// selection bits).  One JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

// Each block reads a contiguous range (like the fold's per-workgroup chunk
// ranges), U loads in flight per thread.
template <int U>
__global__ __launch_bounds__(512) void k_read(const uint4* __restrict__ p, uint64_t n_per_block, uint4* out) {
    const uint4* b = p + (uint64_t)blockIdx.x * n_per_block;
    uint4 a = make_uint4(0, 0, 0, 0);
    for (uint64_t i = threadIdx.x; i < n_per_block; i += (uint64_t)blockDim.x * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * blockDim.x;
            v[u] = j < n_per_block ? b[j] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { a.x ^= v[u].x; a.y ^= v[u].y; a.z ^= v[u].z; a.w ^= v[u].w; }
    }
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u) out[blockIdx.x] = a;   // keep the loads
}

int main() {
    const uint64_t bytes = 512ull << 20, n = bytes / 16;
    uint4 *p, *out;
    CK(hipMalloc(&p, bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(p, 1, bytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](int blocks, int threads, int u) {
        const uint64_t per = (n + blocks - 1) / blocks;
        auto launch = [&]() {
            if (u == 1) hipLaunchKernelGGL(k_read<1>, dim3(blocks), dim3(threads), 0, 0, p, per, out);
            else if (u == 2) hipLaunchKernelGGL(k_read<2>, dim3(blocks), dim3(threads), 0, 0, p, per, out);
            else hipLaunchKernelGGL(k_read<4>, dim3(blocks), dim3(threads), 0, 0, p, per, out);
        };
        float el = 0;
        CK(hipEventRecord(e0, 0));
        while (el < 300.0f) {   // clock spin-up
            for (int i = 0; i < 10; ++i) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&el, e0, e1));
        }
        const int iters = 30;
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&el, e0, e1));
        return bytes / (el / iters * 1e-3) / 1e9;
    };
    printf("{\"bytes\": %llu", (unsigned long long)bytes);
    const int shapes[][3] = {{2, 512, 1}, {2, 512, 2}, {2, 512, 4}, {4, 256, 2}, {8, 256, 4}, {16, 256, 4}};
    double best = 0;
    for (auto& sh : shapes) {
        const double g = run(cus * sh[0], sh[1], sh[2]);
        best = g > best ? g : best;
        printf(", \"wg_per_cu%d_t%d_u%d_GBs\": %.0f", sh[0], sh[1], sh[2], g);
    }
    printf(", \"best_GBs\": %.0f}\n", best);
    return 0;
}
