// fold_bench.hip — isolates the PIR fold kernel (k_pir_fold4r) at configs[4]
// shape (2^24 records x 32 B, 64 keys, selection bits as EvalFull writes
// them) and times it with HIP events.  Built once per DPF_FOLD_EXP variant
// (tools/exp_fold.sh): 0 full, 1 no table stores, 2 no lookups, 3 no loads.
// Prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../dpf-go_amd/csrc/pir_kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint64_t nrec = 1ull << 24;
    const uint32_t nkeys = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
    const int iters = 20;
    const uint64_t wpk = nrec / 32;
    void *bits, *db, *ans, *parts;
    CK(hipMalloc(&bits, nkeys * wpk * 4));
    CK(hipMalloc(&db, nrec * 32));
    CK(hipMalloc(&ans, nkeys * 32));
    CK(hipMalloc(&parts, dpfk::pir_fold_parts_bytes()));
    CK(hipMemset(bits, 0x5a, nkeys * wpk * 4));
    CK(hipMemset(db, 0x3c, nrec * 32));
    CK(hipMemset(ans, 0, nkeys * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i)
        CK(dpfk::launch_pir_fold((const uint32_t*)bits, wpk, (const uint8_t*)db, nrec, nkeys, (uint32_t*)ans,
                                 (uint32_t*)parts, 0));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i)
        CK(dpfk::launch_pir_fold((const uint32_t*)bits, wpk, (const uint8_t*)db, nrec, nkeys, (uint32_t*)ans,
                                 (uint32_t*)parts, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("{\"exp\": %d, \"nkeys\": %u, \"fold_us\": %.1f, \"GBs\": %.0f}\n", DPF_FOLD_EXP, nkeys, ms * 1e3,
           (nrec * 32.0 + nkeys * wpk * 4.0) / (ms * 1e-3) / 1e9);
    return 0;
}
