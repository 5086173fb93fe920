// wave_times.hip — per-wave start/end times of the configs[1] tree kernel
// (k_evalfull built with -DDPF_WAVE_TIMES): how evenly the one round of
// 4096 waves finishes, i.e. what a dynamic (work-stealing) schedule could
// gain.  Random key bytes are structurally valid keys, enough for timing.
// Args: [nkeys=4096] [logN=20] [prefix_bits=0] (subtree 0 of every key: the
// per-rank shape of an N = 2^prefix_bits split).  Also reports when each
// wave finished its root-to-subtree walk (the serial, latency-bound part of a
// small launch).  Prints one JSON line; per-wave rows go to the file named by
// WAVE_TIMES_CSV when set.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define DPF_WAVE_TIMES 1
#include "../dpf-go_amd/csrc/dpf_kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint64_t nkeys = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const uint32_t logN = argc > 2 ? (uint32_t)atoi(argv[2]) : 20;
    const uint32_t pb = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
    const uint32_t stop = logN > 7 ? logN - 7 : 0;
    const uint64_t klen = 33 + 18 * (uint64_t)stop;
    std::vector<uint8_t> keys(nkeys * klen);
    uint64_t x = 0x243F6A8885A308D3ull;
    for (auto& b : keys) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = (uint8_t)x; }
    void *d_keys, *d_ek, *d_out;
    CK(hipMalloc(&d_keys, keys.size()));
    CK(hipMalloc(&d_ek, nkeys * (stop + 2) * 32));
    const uint64_t out_stride = 16ull << (stop - pb);
    CK(hipMalloc(&d_out, nkeys * out_stride));
    CK(hipMemcpy(d_keys, keys.data(), keys.size(), hipMemcpyHostToDevice));
    CK(dpfk::launch_unpack((const uint8_t*)d_keys, klen, nkeys, stop, (uint32_t*)d_ek, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float el = 0;
    CK(hipEventRecord(e0, 0));
    while (el < 500.0f) {   // clock spin-up
        for (int i = 0; i < 20; ++i)
            CK(dpfk::launch_evalfull((const uint32_t*)d_ek, nkeys, stop, pb, 0, (uint8_t*)d_out, out_stride, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&el, e0, e1));
    }
    CK(hipEventRecord(e0, 0));
    CK(dpfk::launch_evalfull((const uint32_t*)d_ek, nkeys, stop, pb, 0, (uint8_t*)d_out, out_stride, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&el, e0, e1));
    std::vector<uint64_t> t(5 * dpfk::kWaveTimesMax);
    CK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(dpfk::g_wave_times), t.size() * 8));
    int dev = 0, rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev));
    const uint64_t nw = std::min<uint64_t>((nkeys << stop) / 128 / 64 * (stop >= 7 ? 1 : 1), dpfk::kWaveTimesMax);
    uint64_t t0 = ~0ull, t1 = 0;
    uint64_t nwaves = 0;
    double busy = 0;
    std::vector<double> ends;
    for (uint64_t w = 0; w < dpfk::kWaveTimesMax; ++w) {
        const uint64_t a = t[5 * w], b = t[5 * w + 1];
        if (b == 0) continue;
        ++nwaves;
        t0 = std::min(t0, a);
        t1 = std::max(t1, b);
    }
    const double us = 1e3 / rate_khz;   // microseconds per tick
    FILE* csv = getenv("WAVE_TIMES_CSV") ? fopen(getenv("WAVE_TIMES_CSV"), "w") : nullptr;
    if (csv) fprintf(csv, "wave,start_us,end_us,hw_id,xcc_id,walk_end_us\n");
    double walk_sum = 0, walk_max = 0;
    for (uint64_t w = 0; w < dpfk::kWaveTimesMax; ++w) {
        const uint64_t a = t[5 * w], b = t[5 * w + 1];
        if (b == 0) continue;
        busy += (double)(b - a);
        ends.push_back((double)(b - t0) * us);
        const double wk = (double)(t[5 * w + 4] - t0) * us;
        walk_sum += (double)(t[5 * w + 4] - a) * us;
        walk_max = std::max(walk_max, wk);
        if (csv) fprintf(csv, "%llu,%.3f,%.3f,%llu,%llu,%.3f\n", (unsigned long long)w, (double)(a - t0) * us,
                         (double)(b - t0) * us, (unsigned long long)t[5 * w + 2], (unsigned long long)t[5 * w + 3], wk);
    }
    if (csv) fclose(csv);
    std::vector<double> starts;
    for (uint64_t w = 0; w < dpfk::kWaveTimesMax; ++w)
        if (t[5 * w + 1]) starts.push_back((double)(t[5 * w] - t0) * us);
    std::sort(starts.begin(), starts.end());
    std::sort(ends.begin(), ends.end());
    const double span = (double)(t1 - t0) * us;
    auto pct = [&](double p) { return ends.empty() ? 0.0 : ends[(size_t)(p * (ends.size() - 1))]; };
    printf("{\"nkeys\": %llu, \"logN\": %u, \"waves\": %llu, \"event_ms\": %.4f, \"span_us\": %.1f, "
           "\"mean_wave_us\": %.1f, \"end_p0_us\": %.1f, \"end_p10_us\": %.1f, \"end_p50_us\": %.1f, \"end_p90_us\": %.1f, "
           "\"end_p100_us\": %.1f, \"start_p50_us\": %.1f, \"start_p100_us\": %.1f, \"mean_busy_frac\": %.4f, "
           "\"expected_waves\": %llu, \"prefix_bits\": %u, \"mean_walk_us\": %.2f, \"walk_end_max_us\": %.2f}\n",
           (unsigned long long)nkeys, logN, (unsigned long long)nwaves, el, span, busy * us / nwaves, pct(0), pct(0.1),
           pct(0.5), pct(0.9), pct(1.0), starts.empty() ? 0.0 : starts[starts.size() / 2],
           starts.empty() ? 0.0 : starts.back(), busy * us / nwaves / span, (unsigned long long)nw, pb,
           walk_sum / nwaves, walk_max);
    return 0;
}
