// dpf_capi.hip — the C ABI (include/dpf_hip.h) over the gfx950 kernels.
//
// Host-buffer entry points stage keys into HBM, run the kernels on a
// per-device stream under a per-device mutex and copy results back;
// device-resident (_dev) entry points only enqueue on the caller's stream.
// There is no CPU evaluation path: without a usable gfx950 device every
// evaluation call fails with DPF_ERR_NODEV.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dpf_hip.h"
#include "dpf_internal.hpp"
#include "dpf_kernels.hpp"
#include "pir_kernels.hpp"

using dpfh::full_len;
using dpfh::key_len;
using dpfh::stop_of;

namespace {

thread_local std::string t_err;

int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return fail(DPF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct Dev {
    int id = 0;
    hipStream_t st = nullptr;
    std::mutex mu;
    DevBuf keys, work, out, xs;
};

std::mutex g_mu;
std::vector<std::unique_ptr<Dev>> g_devs;

// Largest output slab staged in HBM per launch by the host-buffer paths.
constexpr size_t kMaxSlab = (size_t)1 << 30;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(d);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int open_devices(int ngpus) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_devs.empty()) return (int)g_devs.size();
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return fail(DPF_ERR_NODEV, "dpf: no HIP device visible (gfx950 required)");
    if (ngpus > 0) n = std::min(n, ngpus);
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) != hipSuccess) return fail(DPF_ERR_NODEV, "dpf: device query failed");
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(DPF_ERR_NODEV, std::string("dpf: device is ") + prop.gcnArchName + ", need gfx950");
    }
    for (int i = 0; i < n; ++i) {
        auto d = std::make_unique<Dev>();
        d->id = i;
        DeviceGuard g(i);
        if (hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking) != hipSuccess)
            return fail(DPF_ERR_HIP, "dpf: hipStreamCreate failed");
        g_devs.push_back(std::move(d));
    }
    return n;
}

int ensure_open() {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_devs.empty()) return (int)g_devs.size();
    }
    return open_devices(0);
}

int check_key(size_t klen, uint32_t logN) {
    if (logN > 63) return fail(DPF_ERR_PARAM, "dpf: logN > 63");
    if (klen < key_len(logN)) return fail(DPF_ERR_KEYLEN, "dpf: key shorter than 33+18*(logN-7) bytes");
    return DPF_OK;
}

// Evaluate subtree (prefix_bits, prefix) of nk keys already resident at
// d_keys into d_out (2^(stop-prefix_bits) leaves per key), on stream st.
int enqueue_full(const uint8_t* d_keys, size_t klen, size_t nk, uint32_t logN, uint32_t prefix_bits,
                 uint64_t prefix, uint8_t* d_out, uint32_t* d_work, hipStream_t st) {
    const uint32_t stop = stop_of(logN);
    HIP_TRY(dpfk::launch_unpack(d_keys, klen, nk, stop, d_work, st));
    const uint64_t stride = (uint64_t)16 << (stop - prefix_bits);
    HIP_TRY(dpfk::launch_evalfull(d_work, nk, stop, prefix_bits, prefix, d_out, stride, st));
    return DPF_OK;
}

// Host-buffer EvalFull of keys [0, nk) on one device, output slab-chunked.
int full_on_device(Dev& d, const uint8_t* keys, size_t klen, size_t nk, uint32_t logN, uint8_t* out) {
    std::lock_guard<std::mutex> lk(d.mu);
    DeviceGuard g(d.id);
    const uint32_t stop = stop_of(logN);
    const size_t olen = full_len(logN);
    if (olen <= kMaxSlab) {
        const size_t per = std::max<size_t>(1, kMaxSlab / olen);
        for (size_t k0 = 0; k0 < nk; k0 += per) {
            const size_t n = std::min(per, nk - k0);
            HIP_TRY(hipError_t(d.keys.ensure(n * klen)));
            HIP_TRY(hipError_t(d.work.ensure(n * dpfk::ek_words(stop) * 4)));
            HIP_TRY(hipError_t(d.out.ensure(n * olen)));
            HIP_TRY(hipMemcpyAsync(d.keys.p, keys + k0 * klen, n * klen, hipMemcpyHostToDevice, d.st));
            int rc = enqueue_full((const uint8_t*)d.keys.p, klen, n, logN, 0, 0, (uint8_t*)d.out.p,
                                  (uint32_t*)d.work.p, d.st);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(out + k0 * olen, d.out.p, n * olen, hipMemcpyDeviceToHost, d.st));
            HIP_TRY(hipStreamSynchronize(d.st));
        }
        return DPF_OK;
    }
    // One key's output exceeds a slab: walk it subtree by subtree.
    uint32_t pb = 0;
    while ((olen >> pb) > kMaxSlab) ++pb;
    const size_t slab = olen >> pb;
    HIP_TRY(hipError_t(d.keys.ensure(klen)));
    HIP_TRY(hipError_t(d.work.ensure(dpfk::ek_words(stop) * 4)));
    HIP_TRY(hipError_t(d.out.ensure(slab)));
    for (size_t k = 0; k < nk; ++k) {
        HIP_TRY(hipMemcpyAsync(d.keys.p, keys + k * klen, klen, hipMemcpyHostToDevice, d.st));
        for (uint64_t p = 0; p < (1ull << pb); ++p) {
            int rc = enqueue_full((const uint8_t*)d.keys.p, klen, 1, logN, pb, p, (uint8_t*)d.out.p,
                                  (uint32_t*)d.work.p, d.st);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(out + k * olen + p * slab, d.out.p, slab, hipMemcpyDeviceToHost, d.st));
            HIP_TRY(hipStreamSynchronize(d.st));
        }
    }
    return DPF_OK;
}

size_t pir_ek_bytes(size_t nkeys, uint32_t logN);
size_t eval_work_bytes(size_t nkeys, size_t ppk, uint32_t logN);

int eval_on_device(Dev& d, const uint8_t* keys, size_t klen, size_t nk, const uint64_t* xs, size_t ppk,
                   uint32_t logN, uint8_t* out) {
    std::lock_guard<std::mutex> lk(d.mu);
    DeviceGuard g(d.id);
    const uint32_t stop = stop_of(logN);
    const size_t nq = nk * ppk;
    HIP_TRY(hipError_t(d.keys.ensure(std::max<size_t>(1, nk * klen))));
    const size_t wbytes = eval_work_bytes(nk, ppk, logN);
    HIP_TRY(hipError_t(d.work.ensure(std::max<size_t>(16, wbytes))));
    HIP_TRY(hipError_t(d.xs.ensure(std::max<size_t>(8, nq * 8))));
    HIP_TRY(hipError_t(d.out.ensure(std::max<size_t>(1, nq))));
    HIP_TRY(hipMemcpyAsync(d.keys.p, keys, nk * klen, hipMemcpyHostToDevice, d.st));
    HIP_TRY(hipMemcpyAsync(d.xs.p, xs, nq * 8, hipMemcpyHostToDevice, d.st));
    HIP_TRY(dpfk::launch_unpack((const uint8_t*)d.keys.p, klen, nk, stop, (uint32_t*)d.work.p, d.st));
    const size_t ekb = pir_ek_bytes(nk, logN);
    HIP_TRY(dpfk::launch_eval((const uint32_t*)d.work.p, stop, logN, (const uint64_t*)d.xs.p, nq, ppk,
                              (uint8_t*)d.out.p, (uint8_t*)d.work.p + ekb, wbytes - ekb, d.st));
    HIP_TRY(hipMemcpyAsync(out, d.out.p, nq, hipMemcpyDeviceToHost, d.st));
    HIP_TRY(hipStreamSynchronize(d.st));
    return DPF_OK;
}

// Run fn(device_index, lo, hi) over `n` items split evenly across g devices.
template <class F>
int shard(size_t n, int g, F fn) {
    if (g <= 1 || n <= 1) return fn(0, (size_t)0, n);
    std::vector<int> rc((size_t)g, DPF_OK);
    std::vector<std::string> errs((size_t)g);
    std::vector<std::thread> th;
    for (int i = 0; i < g; ++i) {
        const size_t lo = n * (size_t)i / (size_t)g, hi = n * (size_t)(i + 1) / (size_t)g;
        th.emplace_back([&, i, lo, hi] {
            rc[(size_t)i] = lo < hi ? fn(i, lo, hi) : DPF_OK;
            errs[(size_t)i] = t_err;
        });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < g; ++i)
        if (rc[(size_t)i]) return fail(rc[(size_t)i], errs[(size_t)i]);
    return DPF_OK;
}

int pick_ngpus(int ngpus) {
    int have = ensure_open();
    if (have <= 0) return have;
    return ngpus <= 0 ? have : std::min(ngpus, have);
}

// Expanded keys at the start of a PIR workspace, padded to 256 B.
size_t pir_ek_bytes(size_t nkeys, uint32_t logN) {
    return (nkeys * dpfk::ek_words(stop_of(logN)) * 4 + 255) & ~(size_t)255;
}

// Batched-Eval workspace: expanded keys (256-B padded), then the frontier.
size_t eval_work_bytes(size_t nkeys, size_t ppk, uint32_t logN) {
    return pir_ek_bytes(nkeys, logN) + dpfk::eval_frontier_bytes(nkeys, stop_of(logN), ppk);
}

}  // namespace

extern "C" {

const char* dpf_last_error(void) { return t_err.c_str(); }

size_t dpf_key_len(uint32_t logN) { return key_len(logN); }
size_t dpf_evalfull_len(uint32_t logN) { return full_len(logN); }
size_t dpf_workspace_size(size_t nkeys, uint32_t logN) {
    return std::max<size_t>(16, nkeys * dpfk::ek_words(stop_of(logN)) * 4);
}

int dpf_gpu_init(int ngpus) { return open_devices(ngpus); }

void dpf_gpu_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& d : g_devs) {
        std::lock_guard<std::mutex> dl(d->mu);
        DeviceGuard g(d->id);
        (void)hipStreamSynchronize(d->st);
        d->keys.release();
        d->work.release();
        d->out.release();
        d->xs.release();
        (void)hipStreamDestroy(d->st);
    }
    g_devs.clear();
}

int dpf_gpu_count(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return (int)g_devs.size();
}

int dpf_gen_seeded(uint64_t alpha, uint32_t logN, const uint8_t s0[16], const uint8_t s1[16], uint8_t* ka,
                   uint8_t* kb) {
    int rc = dpfh::gen_seeded(alpha, logN, s0, s1, ka, kb);
    return rc ? fail(rc, "dpf: invalid parameters") : DPF_OK;
}

int dpf_gen(uint64_t alpha, uint32_t logN, uint8_t* ka, uint8_t* kb) {
    int rc = dpfh::gen_random(alpha, logN, ka, kb);
    return rc ? fail(rc, "dpf: invalid parameters") : DPF_OK;
}

int dpf_gen_batch_seeded(const uint64_t* alphas, uint32_t logN, const uint8_t* s0s, const uint8_t* s1s, size_t n,
                         uint8_t* kas, uint8_t* kbs, int nthreads) {
    int rc = dpfh::gen_batch_seeded(alphas, logN, s0s, s1s, n, kas, kbs, nthreads);
    return rc ? fail(rc, "dpf: invalid parameters") : DPF_OK;
}

int dpf_evalfull_batch(const uint8_t* keys, size_t klen, size_t nkeys, uint32_t logN, uint8_t* out, int ngpus) {
    if (int rc = check_key(klen, logN)) return rc;
    if (nkeys == 0) return DPF_OK;
    const int g = pick_ngpus(ngpus);
    if (g <= 0) return g;
    const size_t olen = full_len(logN);
    return shard(nkeys, g, [&](int dev, size_t lo, size_t hi) {
        return full_on_device(*g_devs[(size_t)dev], keys + lo * klen, klen, hi - lo, logN, out + lo * olen);
    });
}

int dpf_evalfull(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out) {
    return dpf_evalfull_batch(key, klen, 1, logN, out, 1);
}

int dpf_eval_batch(const uint8_t* keys, size_t klen, size_t nkeys, const uint64_t* xs, size_t ppk, uint32_t logN,
                   uint8_t* out, int ngpus) {
    if (int rc = check_key(klen, logN)) return rc;
    if (nkeys == 0 || ppk == 0) return DPF_OK;
    const int g = pick_ngpus(ngpus);
    if (g <= 0) return g;
    return shard(nkeys, g, [&](int dev, size_t lo, size_t hi) {
        return eval_on_device(*g_devs[(size_t)dev], keys + lo * klen, klen, hi - lo, xs + lo * ppk, ppk, logN,
                              out + lo * ppk);
    });
}

int dpf_eval(const uint8_t* key, size_t klen, uint64_t x, uint32_t logN, uint8_t* out_bit) {
    return dpf_eval_batch(key, klen, 1, &x, 1, logN, out_bit, 1);
}

int dpf_evalfull_split(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out, int ngpus) {
    if (int rc = check_key(klen, logN)) return rc;
    const int have = pick_ngpus(ngpus);
    if (have <= 0) return have;
    const uint32_t stop = stop_of(logN);
    const int want = ngpus <= 0 ? have : ngpus;
    if (want > have) return fail(DPF_ERR_PARAM, "dpf: more GPUs requested than opened");
    uint32_t pb = 0;
    while ((1 << pb) < want) ++pb;
    if ((1 << pb) != want || pb > stop) return fail(DPF_ERR_PARAM, "dpf: ngpus must be a power of two <= 2^(logN-7)");
    const size_t slab = full_len(logN) >> pb;
    return shard((size_t)want, want, [&](int dev, size_t lo, size_t hi) {
        (void)hi;
        Dev& d = *g_devs[(size_t)dev];
        std::lock_guard<std::mutex> lk(d.mu);
        DeviceGuard gd(d.id);
        HIP_TRY(hipError_t(d.keys.ensure(klen)));
        HIP_TRY(hipError_t(d.work.ensure(dpfk::ek_words(stop) * 4)));
        HIP_TRY(hipError_t(d.out.ensure(slab)));
        HIP_TRY(hipMemcpyAsync(d.keys.p, key, klen, hipMemcpyHostToDevice, d.st));
        int rc = enqueue_full((const uint8_t*)d.keys.p, klen, 1, logN, pb, lo, (uint8_t*)d.out.p,
                              (uint32_t*)d.work.p, d.st);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(out + lo * slab, d.out.p, slab, hipMemcpyDeviceToHost, d.st));
        HIP_TRY(hipStreamSynchronize(d.st));
        return DPF_OK;
    });
}

int dpf_evalfull_subtree_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN,
                             uint32_t prefix_bits, uint64_t prefix, uint8_t* d_out, void* d_work, void* stream) {
    if (int rc = check_key(klen, logN)) return rc;
    const uint32_t stop = stop_of(logN);
    if (prefix_bits > stop || (prefix_bits < 64 && (prefix >> prefix_bits) != 0))
        return fail(DPF_ERR_PARAM, "dpf: subtree prefix out of range");
    if (nkeys == 0) return DPF_OK;
    DeviceGuard g(device);
    return enqueue_full(d_keys, klen, nkeys, logN, prefix_bits, prefix, d_out, (uint32_t*)d_work,
                        (hipStream_t)stream);
}

int dpf_evalfull_batch_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN,
                           uint8_t* d_out, void* d_work, void* stream) {
    return dpf_evalfull_subtree_dev(device, d_keys, klen, nkeys, logN, 0, 0, d_out, d_work, stream);
}

size_t dpf_eval_workspace_size(size_t nkeys, size_t pts_per_key, uint32_t logN) {
    return std::max<size_t>(16, eval_work_bytes(nkeys, pts_per_key, logN));
}

int dpf_eval_batch_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, const uint64_t* d_xs,
                       size_t ppk, uint32_t logN, uint8_t* d_out, void* d_work, size_t work_bytes, void* stream) {
    if (int rc = check_key(klen, logN)) return rc;
    if (nkeys == 0 || ppk == 0) return DPF_OK;
    const uint32_t stop = stop_of(logN);
    const size_t ekb = pir_ek_bytes(nkeys, logN);
    if (work_bytes < nkeys * dpfk::ek_words(stop) * 4) return fail(DPF_ERR_PARAM, "dpf: Eval workspace too small");
    DeviceGuard g(device);
    HIP_TRY(dpfk::launch_unpack(d_keys, klen, nkeys, stop, (uint32_t*)d_work, (hipStream_t)stream));
    // The frontier (if it fits in the rest of the workspace) lets queries share the tree's top levels.
    void* frontier = work_bytes > ekb ? (uint8_t*)d_work + ekb : nullptr;
    HIP_TRY(dpfk::launch_eval((const uint32_t*)d_work, stop, logN, d_xs, nkeys * ppk, ppk, d_out, frontier,
                              work_bytes > ekb ? work_bytes - ekb : 0, (hipStream_t)stream));
    return DPF_OK;
}

int dpf_expand_keys_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN, void* d_work,
                        void* stream) {
    if (int rc = check_key(klen, logN)) return rc;
    DeviceGuard g(device);
    HIP_TRY(dpfk::launch_unpack(d_keys, klen, nkeys, stop_of(logN), (uint32_t*)d_work, (hipStream_t)stream));
    return DPF_OK;
}

int dpf_evalfull_expanded_dev(int device, const void* d_work, size_t nkeys, uint32_t logN, uint32_t prefix_bits,
                              uint64_t prefix, uint8_t* d_out, void* stream) {
    if (logN > 63) return fail(DPF_ERR_PARAM, "dpf: logN > 63");
    const uint32_t stop = stop_of(logN);
    if (prefix_bits > stop || (prefix >> prefix_bits) != 0) return fail(DPF_ERR_PARAM, "dpf: subtree prefix out of range");
    if (nkeys == 0) return DPF_OK;
    DeviceGuard g(device);
    const uint64_t stride = (uint64_t)16 << (stop - prefix_bits);
    HIP_TRY(dpfk::launch_evalfull((const uint32_t*)d_work, nkeys, stop, prefix_bits, prefix, d_out, stride,
                                  (hipStream_t)stream));
    return DPF_OK;
}

// ------------------------------------------------------------------ PIR ---

size_t dpf_pir_workspace_size(size_t nkeys, uint32_t logN, uint32_t prefix_bits) {
    const uint32_t stop = stop_of(logN);
    const uint32_t pb = prefix_bits > stop ? stop : prefix_bits;
    return pir_ek_bytes(nkeys, logN) + nkeys * ((size_t)16 << (stop - pb)) + dpfk::pir_fold_parts_bytes();
}

int dpf_pir_answer_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN,
                       uint32_t prefix_bits, uint64_t prefix, const uint8_t* d_db, uint64_t nrec, uint8_t* d_ans,
                       void* d_work, void* stream) {
    if (int rc = check_key(klen, logN)) return rc;
    const uint32_t stop = stop_of(logN);
    if (prefix_bits > stop || (prefix >> prefix_bits) != 0) return fail(DPF_ERR_PARAM, "dpf: subtree prefix out of range");
    const uint64_t slice = logN - prefix_bits >= 64 ? ~0ull : (1ull << (logN - prefix_bits));
    if (nrec > slice) return fail(DPF_ERR_PARAM, "dpf: more DB records than the subtree's domain");
    DeviceGuard g(device);
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(d_ans, 0, nkeys * 32, st));
    if (nkeys == 0 || nrec == 0) return DPF_OK;
    uint32_t* ek = (uint32_t*)d_work;
    uint8_t* bits = (uint8_t*)d_work + pir_ek_bytes(nkeys, logN);
    const uint64_t per_key = (uint64_t)16 << (stop - prefix_bits);
    int rc = enqueue_full(d_keys, klen, nkeys, logN, prefix_bits, prefix, bits, ek, st);
    if (rc) return rc;
    uint32_t* parts = (uint32_t*)(bits + nkeys * per_key);
    HIP_TRY(dpfk::launch_pir_fold((const uint32_t*)bits, per_key / 4, d_db, nrec, (uint32_t)nkeys, (uint32_t*)d_ans, parts,
                                  st));
    return DPF_OK;
}

struct PirDb {
    uint32_t logN = 0, pbits = 0;
    uint64_t nrec = 0;
    std::vector<void*> shard;      // per device: its DB slice
    std::vector<uint64_t> shard_n; // records in that slice
};

int dpf_pir_db_create(const uint8_t* db, uint64_t nrec, uint32_t logN, int ngpus, void** handle) {
    if (!handle) return fail(DPF_ERR_PARAM, "dpf: null handle");
    *handle = nullptr;
    if (logN > 63 || (logN < 64 && nrec > (1ull << logN))) return fail(DPF_ERR_PARAM, "dpf: DB larger than 2^logN");
    const int have = pick_ngpus(ngpus);
    if (have <= 0) return have;
    const int want = ngpus <= 0 ? have : ngpus;
    uint32_t pb = 0;
    while ((1 << pb) < want) ++pb;
    if ((1 << pb) != want || want > have || pb > stop_of(logN))
        return fail(DPF_ERR_PARAM, "dpf: ngpus must be a power of two <= opened devices and 2^(logN-7)");
    auto h = std::make_unique<PirDb>();
    h->logN = logN;
    h->pbits = pb;
    h->nrec = nrec;
    const uint64_t slice = 1ull << (logN - pb);
    for (int g = 0; g < want; ++g) {
        const uint64_t lo = std::min<uint64_t>(nrec, (uint64_t)g * slice);
        const uint64_t hi = std::min<uint64_t>(nrec, lo + slice);
        DeviceGuard gd(g_devs[(size_t)g]->id);
        void* p = nullptr;
        const size_t bytes = std::max<uint64_t>(hi - lo, 1) * 32;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            for (void* q : h->shard) (void)hipFree(q);
            return fail(DPF_ERR_NOMEM, "dpf: DB shard allocation failed");
        }
        if (hi > lo && hipMemcpy(p, db + lo * 32, (hi - lo) * 32, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(p);
            for (void* q : h->shard) (void)hipFree(q);
            return fail(DPF_ERR_HIP, "dpf: DB upload failed");
        }
        h->shard.push_back(p);
        h->shard_n.push_back(hi - lo);
    }
    *handle = h.release();
    return DPF_OK;
}

int dpf_pir_answer(void* handle, const uint8_t* keys, size_t klen, size_t nkeys, uint8_t* ans) {
    PirDb* h = (PirDb*)handle;
    if (!h) return fail(DPF_ERR_PARAM, "dpf: null PIR handle");
    if (int rc = check_key(klen, h->logN)) return rc;
    const int g = (int)h->shard.size();
    std::vector<std::vector<uint8_t>> part((size_t)g, std::vector<uint8_t>(nkeys * 32));
    int rc = shard((size_t)g, g, [&](int dev, size_t lo, size_t hi) {
        (void)hi;
        Dev& d = *g_devs[(size_t)dev];
        std::lock_guard<std::mutex> lk(d.mu);
        DeviceGuard gd(d.id);
        HIP_TRY(hipError_t(d.keys.ensure(std::max<size_t>(1, nkeys * klen))));
        HIP_TRY(hipError_t(d.work.ensure(dpf_pir_workspace_size(nkeys, h->logN, h->pbits))));
        HIP_TRY(hipError_t(d.out.ensure(std::max<size_t>(32, nkeys * 32))));
        HIP_TRY(hipMemcpyAsync(d.keys.p, keys, nkeys * klen, hipMemcpyHostToDevice, d.st));
        int r = dpf_pir_answer_dev(d.id, (const uint8_t*)d.keys.p, klen, nkeys, h->logN, h->pbits, lo,
                                   (const uint8_t*)h->shard[lo], h->shard_n[lo], (uint8_t*)d.out.p, d.work.p, d.st);
        if (r) return r;
        HIP_TRY(hipMemcpyAsync(part[lo].data(), d.out.p, nkeys * 32, hipMemcpyDeviceToHost, d.st));
        HIP_TRY(hipStreamSynchronize(d.st));
        return DPF_OK;
    });
    if (rc) return rc;
    memset(ans, 0, nkeys * 32);
    for (int i = 0; i < g; ++i)
        for (size_t b = 0; b < nkeys * 32; ++b) ans[b] ^= part[(size_t)i][b];
    return DPF_OK;
}

void dpf_pir_db_free(void* handle) {
    PirDb* h = (PirDb*)handle;
    if (!h) return;
    for (size_t i = 0; i < h->shard.size(); ++i) {
        DeviceGuard gd(g_devs[i]->id);
        (void)hipFree(h->shard[i]);
    }
    delete h;
}

}  // extern "C"
