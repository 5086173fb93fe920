// fold_bench.hip — isolates the PIR fold kernel at configs[4] shape (2^24
// records x 32 B, 64 keys, random selection bits laid out as EvalFull
// writes them) and times it with HIP events.  Build with -DFOLD_SRC=<file>
// to A/B another revision of pir_kernels.hip (tools/ab/).  One JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#ifndef FOLD_SRC
#define FOLD_SRC "../dpf-go_amd/csrc/pir_kernels.hip"
#endif
#include FOLD_SRC

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint64_t nrec = 1ull << 24;
    const uint32_t nkeys = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
    const int iters = 20;
    const uint64_t wpk = nrec / 32;
    void *bits, *db, *ans, *parts;
    CK(hipMalloc(&bits, (size_t)nkeys * wpk * 4));
    CK(hipMalloc(&db, nrec * 32));
    CK(hipMalloc(&ans, (size_t)nkeys * 32));
    CK(hipMalloc(&parts, dpfk::pir_fold_parts_bytes()));
    std::vector<uint32_t> h((size_t)nkeys * wpk);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7);
    CK(hipMemcpy(bits, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(db, 0x5a, nrec * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i)
        CK(dpfk::launch_pir_fold((const uint32_t*)bits, wpk, (const uint8_t*)db, nrec, 32, nkeys, (uint32_t*)ans,
                                 (uint32_t*)parts, 0));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i)
        CK(dpfk::launch_pir_fold((const uint32_t*)bits, wpk, (const uint8_t*)db, nrec, 32, nkeys, (uint32_t*)ans,
                                 (uint32_t*)parts, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    std::vector<uint32_t> a((size_t)nkeys * 8);
    CK(hipMemcpy(a.data(), ans, a.size() * 4, hipMemcpyDeviceToHost));
    uint32_t chk = 0;
    for (uint32_t v : a) chk = chk * 31 + v;
    printf("{\"src\": \"%s\", \"nkeys\": %u, \"fold_us\": %.1f, \"GBs\": %.0f, \"check\": %u}\n", FOLD_SRC, nkeys,
           ms * 1e3, (nrec * 32 + (double)nkeys * wpk * 4) / (ms * 1e-3) / 1e9, chk);
    return 0;
}
