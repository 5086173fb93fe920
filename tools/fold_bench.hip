// fold_bench.hip — isolates the XOR fold (pir_kernels.hip) at configs[4]
// shape by default (2^24 records x 32 B, 64 keys, random selection bits laid
// out as EvalFull writes them), times it with HIP events and checks 2 keys'
// answers against a plain host fold.  Args: [nkeys] [rec_bytes] [log2 nrec].
// Build with -DFOLD_SRC=<file> to A/B another revision (tools/ab/).  One
// JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#ifndef FOLD_SRC
#define FOLD_SRC "../dpf-go_amd/csrc/pir_kernels.hip"
#endif
#include FOLD_SRC

// pir_kernels.hip sizes its grids with dpfk::cu_count() (dpf_kernels.hip in
// the library): the whole device here.
namespace dpfk {
int cu_count() {
    int d = 0, c = 256;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
        c = 256;
    return c;
}
}  // namespace dpfk

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint32_t nkeys = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
    const uint64_t rec_bytes = argc > 2 ? (uint64_t)atoll(argv[2]) : 32;
    const uint64_t nrec = argc > 3 ? 1ull << atoi(argv[3]) : 1ull << 24;
    const int iters = 20;
    const uint64_t wpk = (nrec + 127) / 128 * 4;
    void *bits, *db, *ans, *parts;
    CK(hipMalloc(&bits, (size_t)nkeys * wpk * 4));
    CK(hipMalloc(&db, nrec * rec_bytes));
    CK(hipMalloc(&ans, (size_t)nkeys * rec_bytes));
    CK(hipMalloc(&parts, dpfk::pir_fold_parts_bytes()));
    std::vector<uint32_t> h((size_t)nkeys * wpk);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (auto& v : h) v = (uint32_t)rnd();
    std::vector<uint8_t> hdb(nrec * rec_bytes);
    for (size_t i = 0; i < hdb.size(); i += 8) { uint64_t r = rnd(); memcpy(&hdb[i], &r, 8); }
    CK(hipMemcpy(bits, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hdb.data(), hdb.size(), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // FOLD_MODE=mfma: the matrix-core fold over the bit-sliced DB (32-byte
    // records), built once here as the PIR server does at load time; its
    // answers must equal the Four-Russians / direct fold's for every key.
    const bool mfma = getenv("FOLD_MODE") && getenv("FOLD_MODE")[0] == 'm';
    // FOLD_BLOCKS=n: at most n workgroups per fold launch (dpf_set_fold_limits).
    if (getenv("FOLD_BLOCKS")) dpfk::set_fold_limits((uint32_t)atoi(getenv("FOLD_BLOCKS")), 0);
    void* dbs = nullptr;
    float slice_ms = 0;
    std::vector<uint8_t> ref((size_t)nkeys * rec_bytes);
    if (mfma) {
        if (rec_bytes != 32) { fprintf(stderr, "mfma mode: 32-byte records only\n"); return 2; }
        CK(hipMalloc(&dbs, dpfk::pir_sliced_bytes(nrec)));
        CK(hipEventRecord(e0, 0));
        CK(dpfk::launch_slice_db((const uint8_t*)db, nrec, (uint8_t*)dbs, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&slice_ms, e0, e1));
        CK(dpfk::launch_pir_fold((const uint32_t*)bits, wpk, (const uint8_t*)db, nrec, rec_bytes, nkeys,
                                 (uint32_t*)ans, (uint32_t*)parts, 0));
        CK(hipMemcpy(ref.data(), ans, ref.size(), hipMemcpyDeviceToHost));
    }
    // FOLD_SGM=1 (with FOLD_MODE=mfma): the selection bits super-group-major,
    // sgm[S][key][8 words] = bits[key][8S .. 8S+8), as a tree pass could write them.
    // FOLD_SGM=4: chunks of 4 super-groups, sgm[S/4][key][32 words] (one
    // 128-byte line of a key per chunk, as the PIR tree kernel writes them).
    const uint32_t sgm_g = mfma && getenv("FOLD_SGM") ? (uint32_t)atoi(getenv("FOLD_SGM")) : 0;
    const bool sgm = sgm_g == 1 || sgm_g == 4;
    void* bits_sgm = nullptr;
    if (sgm) {
        const uint64_t nsgs = (nrec + 255) / 256, nch = (nsgs + sgm_g - 1) / sgm_g;
        std::vector<uint32_t> t(nch * sgm_g * nkeys * 8, 0);
        for (uint64_t S = 0; S < nsgs; ++S)
            for (uint32_t k = 0; k < nkeys; ++k)
                for (int w = 0; w < 8; ++w)
                    if (8 * S + w < wpk)
                        t[((S / sgm_g * nkeys + k) * sgm_g + S % sgm_g) * 8 + w] = h[(size_t)k * wpk + 8 * S + w];
        CK(hipMalloc(&bits_sgm, t.size() * 4));
        CK(hipMemcpy(bits_sgm, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    }
    auto run = [&]() {
        CK(hipMemsetAsync(ans, 0, (size_t)nkeys * rec_bytes, 0));
        if (sgm)
            CK(dpfk::launch_pir_fold_sliced((const uint32_t*)bits_sgm, wpk, (const uint8_t*)dbs, nrec, nkeys,
                                            (uint32_t*)ans, (uint32_t*)parts, 0, nkeys, sgm_g));
        else if (mfma)
            CK(dpfk::launch_pir_fold_sliced((const uint32_t*)bits, wpk, (const uint8_t*)dbs, nrec, nkeys,
                                            (uint32_t*)ans, (uint32_t*)parts, 0));
        else
            CK(dpfk::launch_pir_fold((const uint32_t*)bits, wpk, (const uint8_t*)db, nrec, rec_bytes, nkeys,
                                     (uint32_t*)ans, (uint32_t*)parts, 0));
    };
    // Clock spin-up: an idle MI355X needs a few hundred ms of load to reach
    // its steady clock.
    {
        CK(hipEventRecord(e0, 0));
        float el = 0;
        while (el < 400.0f) {
            for (int i = 0; i < 10; ++i) run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&el, e0, e1));
        }
    }
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    std::vector<uint8_t> a((size_t)nkeys * rec_bytes);
    CK(hipMemcpy(a.data(), ans, a.size(), hipMemcpyDeviceToHost));
    int bad = 0;
    if (mfma) bad += memcmp(ref.data(), a.data(), a.size()) != 0;     // every key vs the LDS fold
    const uint32_t check_keys[2] = {0, nkeys - 1};
    for (uint32_t k : check_keys) {
        std::vector<uint8_t> want(rec_bytes, 0);
        for (uint64_t i = 0; i < nrec; ++i)
            if ((h[(size_t)k * wpk + i / 32] >> (i % 32)) & 1)
                for (uint64_t b = 0; b < rec_bytes; ++b) want[b] ^= hdb[i * rec_bytes + b];
        bad += memcmp(want.data(), &a[(size_t)k * rec_bytes], rec_bytes) != 0;
    }
#ifdef DPF_FOLD_PLAN
    const dpfk::FoldPlan p = dpfk::plan_fold(rec_bytes, nkeys);
#else
    struct { uint32_t cols, col_passes, keys_per_pass, kw; bool direct; } p{1, (uint32_t)(rec_bytes / 32), 64, 1, false};
#endif
    const double bytes = (double)nrec * rec_bytes + (double)nkeys * nrec / 8;
    printf("{\"src\": \"%s\", \"nkeys\": %u, \"rec_bytes\": %llu, \"nrec\": %llu, \"kernel\": \"%s\", \"kw\": %u, "
           "\"col_passes\": %u, \"fold_us\": %.1f, \"GBs\": %.0f, \"db_reads\": %u, \"slice_db_us\": %.1f, \"ok\": %s}\n",
           FOLD_SRC, nkeys, (unsigned long long)rec_bytes, (unsigned long long)nrec,
           mfma ? "mfma" : p.direct ? "direct" : "4r", p.kw,
           p.col_passes, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           p.col_passes * ((nkeys + p.keys_per_pass - 1) / p.keys_per_pass), slice_ms * 1e3, bad ? "false" : "true");
#ifdef DPF_FOLD_TIMES
    {   // per-wave start / end of the last launch (k_fold4r only)
        std::vector<uint64_t> t(4 * dpfk::kFoldTimesMax);
        CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(dpfk::g_fold_times), t.size() * 8));
        int rate_khz = 0;
        CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
        uint64_t t0 = ~0ull;
        for (size_t w = 0; w < dpfk::kFoldTimesMax; ++w)
            if (t[4 * w + 1]) t0 = t[4 * w] < t0 ? t[4 * w] : t0;
        FILE* f = fopen(getenv("FOLD_TIMES_CSV") ? getenv("FOLD_TIMES_CSV") : "fold_times.csv", "w");
        fprintf(f, "wave,start_us,end_us,hw_id,xcc_id\n");
        for (size_t w = 0; w < dpfk::kFoldTimesMax; ++w)
            if (t[4 * w + 1])
                fprintf(f, "%zu,%.3f,%.3f,%llu,%llu\n", w, (t[4 * w] - t0) * 1e3 / rate_khz,
                        (t[4 * w + 1] - t0) * 1e3 / rate_khz, (unsigned long long)t[4 * w + 2],
                        (unsigned long long)t[4 * w + 3]);
        fclose(f);
    }
#endif
    return bad ? 1 : 0;
}
