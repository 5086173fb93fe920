// dpf_capi.hip — the C ABI (include/dpf_hip.h) over the gfx950 kernels.
//
// Host-buffer entry points stage keys into HBM, run the kernels on a
// per-device stream under a per-device mutex and copy results back;
// device-resident (_dev) entry points only enqueue on the caller's stream.
// There is no CPU evaluation path: without a usable gfx950 device every
// evaluation call fails with DPF_ERR_NODEV.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dpf_hip.h"
#include "dpf_internal.hpp"
#include "bs_kernels.hpp"
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

// Pinned host staging buffer (hipHostMalloc), grown on demand.
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct Dev {
    int id = 0;
    hipStream_t st = nullptr;    // kernels
    hipStream_t cst = nullptr;   // device -> host copies of the pipelined host-buffer paths
    hipStream_t hst = nullptr;   // host -> device copies (batched Eval's points)
    hipEvent_t ev_k[2] = {nullptr, nullptr}, ev_c[2] = {nullptr, nullptr}, ev_h[2] = {nullptr, nullptr};
    std::mutex mu;
    DevBuf keys, work, out, xs;
    HostBuf pin[2];
    ~Dev();
};

// Parallel host memcpy for the pinned -> caller-buffer leg of the pipelined
// copies (one thread reaches ~10 GB/s; PCIe delivers ~50).  A fixed pool of
// workers takes 2 MiB pieces; the caller works too and waits for the rest.
class CopyPool {
   public:
    static CopyPool& get() {
        static CopyPool pool;
        return pool;
    }
    // memcpy over the pool in 2 MiB pieces.
    void memcpy_par(void* dst, const void* src, size_t n) {
        if (n <= kPiece || workers_.empty()) {
            memcpy(dst, src, n);
            return;
        }
        struct Ctx {
            uint8_t* d;
            const uint8_t* s;
            size_t n;
        } c{static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n};
        parallel_for((n + kPiece - 1) / kPiece, &c, [](void* p, size_t i) {
            const Ctx& x = *static_cast<const Ctx*>(p);
            const size_t off = i * kPiece;
            memcpy(x.d + off, x.s + off, std::min(kPiece, x.n - off));
        });
    }
    // First touch of a (fresh) destination, one write per 4 KiB page, so the
    // page faults -- one per 2 MiB with transparent huge pages -- are taken
    // by all workers at once instead of inside the timed copies.
    void prefault_par(void* dst, size_t n) {
        struct Ctx {
            volatile uint8_t* d;
            size_t n;
        } c{static_cast<volatile uint8_t*>(dst), n};
        parallel_for((n + kPiece - 1) / kPiece, &c, [](void* p, size_t i) {
            const Ctx& x = *static_cast<const Ctx*>(p);
            const size_t off = i * kPiece, end = std::min(off + kPiece, x.n);
            for (size_t o = off; o < end; o += 4096) x.d[o] = 0;
        });
    }

   private:
    static constexpr size_t kPiece = (size_t)2 << 20;
    struct Job {
        void (*fn)(void*, size_t);
        void* ctx;
        size_t npieces;
        size_t active = 0;   // workers inside run(); guarded by mu_
        std::atomic<size_t> next{0}, done{0};
        Job(void (*f)(void*, size_t), void* c, size_t np) : fn(f), ctx(c), npieces(np) {}
    };
    // fn(ctx, i) for i < npieces over the caller and the workers.
    void parallel_for(size_t npieces, void* ctx, void (*fn)(void*, size_t)) {
        Job job{fn, ctx, npieces};
        {
            std::lock_guard<std::mutex> lk(mu_);
            jobs_.push_back(&job);
        }
        cv_.notify_all();
        run(job);
        // Workers that picked the job leave it (active == 0) before it goes out of scope.
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return job.done.load() == job.npieces && job.active == 0; });
        jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &job));
    }
    // Run pieces of `job` until none is left.
    static void run(Job& job) {
        for (size_t i; (i = job.next.fetch_add(1)) < job.npieces;) {
            job.fn(job.ctx, i);
            job.done.fetch_add(1);
        }
    }
    // One worker per CPU this process may use (affinity mask, capped by a
    // cgroup CPU quota), minus the caller, at most 31: first-touch page
    // faults of a fresh caller buffer and the copy itself both scale with
    // threads (one thread copies ~10 GB/s; PCIe delivers ~50).
    CopyPool() {
        const unsigned n = std::min(31u, usable_cpus() > 1 ? usable_cpus() - 1 : 0u);
        for (unsigned i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    static unsigned usable_cpus() {
        unsigned n = std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0) n = (unsigned)CPU_COUNT(&set);
        if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            unsigned long per = 0;
            if (fscanf(f, "%31s %lu", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
                const unsigned long quota = strtoul(q, nullptr, 10) / per;
                if (quota >= 1 && quota < n) n = (unsigned)quota;
            }
            fclose(f);
        }
        return n > 0 ? n : 1;
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            // Take the job the predicate found, under the same lock hold: the
            // piece counter (`next`) moves without the lock, so a second
            // pending() call could find the job already exhausted.
            Job* j = nullptr;
            cv_.wait(lk, [&] { return stop_ || (j = pending()) != nullptr; });
            if (stop_) return;
            ++j->active;
            lk.unlock();
            run(*j);
            lk.lock();
            --j->active;
            done_cv_.notify_all();
        }
    }
    Job* pending() {
        for (Job* j : jobs_)
            if (j->next.load() < j->npieces) return j;
        return nullptr;
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<Job*> jobs_;
    std::vector<std::thread> workers_;
    bool stop_ = false;
};

// Open devices.  Entry points take a snapshot (shared_ptr copies) under
// g_mu, so dpf_gpu_shutdown only drops the registry's references: a call in
// flight, or a PIR handle, keeps its devices alive until it is done with
// them, and the last reference releases the device's buffers and streams.
// The registry is a never-destroyed heap object: a process that exits
// without dpf_gpu_shutdown runs no Dev destructor (so no HIP call) during
// static teardown, whatever the order against the HIP runtime and torch.
std::mutex g_mu;
std::vector<std::shared_ptr<Dev>>& g_devs = *new std::vector<std::shared_ptr<Dev>>();
std::atomic<int> g_ndevs{0};   // g_devs.size(), readable without g_mu (small-call routing)

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

// Streams created by dpf_stream_create_cu_masked and the CUs each may use.
// A _dev entry point launching on one of them sizes its grids to those CUs
// (CuScope); any other stream gets the whole device.
std::mutex g_cus_mu;
std::unordered_map<hipStream_t, int> g_stream_cus;

struct CuScope {
    int prev;
    explicit CuScope(void* stream) : prev(dpfk::cu_budget()) {
        int c = 0;
        if (stream) {
            std::lock_guard<std::mutex> lk(g_cus_mu);
            auto it = g_stream_cus.find((hipStream_t)stream);
            if (it != g_stream_cus.end()) c = it->second;
        }
        dpfk::set_cu_budget(c);
    }
    ~CuScope() { dpfk::set_cu_budget(prev); }
};

Dev::~Dev() {
    std::lock_guard<std::mutex> dl(mu);
    DeviceGuard g(id);
    for (hipStream_t t : {st, cst, hst})
        if (t) (void)hipStreamSynchronize(t);
    keys.release();
    work.release();
    out.release();
    xs.release();
    for (int i = 0; i < 2; ++i) {
        pin[i].release();
        for (hipEvent_t e : {ev_k[i], ev_c[i], ev_h[i]})
            if (e) (void)hipEventDestroy(e);
    }
    for (hipStream_t t : {st, cst, hst})
        if (t) (void)hipStreamDestroy(t);
}

using DevList = std::vector<std::shared_ptr<Dev>>;

int check_gfx950(int ordinal) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, ordinal) != hipSuccess) return fail(DPF_ERR_NODEV, "dpf: device query failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(DPF_ERR_NODEV, std::string("dpf: device is ") + prop.gcnArchName + ", need gfx950");
    return DPF_OK;
}

// Open exactly the HIP ordinals `ids` (caller holds g_mu, registry empty).
int open_list(const std::vector<int>& ids) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return fail(DPF_ERR_NODEV, "dpf: no HIP device visible (gfx950 required)");
    for (int id : ids) {
        if (id < 0 || id >= n) return fail(DPF_ERR_PARAM, "dpf: device ordinal out of range");
        if (int rc = check_gfx950(id)) return rc;
    }
    DevList devs;
    for (int id : ids) {
        auto d = std::make_shared<Dev>();
        d->id = id;
        DeviceGuard g(id);
        if (hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking) != hipSuccess)
            return fail(DPF_ERR_HIP, "dpf: hipStreamCreate failed");
        devs.push_back(std::move(d));
    }
    g_devs = std::move(devs);
    g_ndevs.store((int)g_devs.size());
    return (int)g_devs.size();
}

int open_devices(int ngpus) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_devs.empty()) return (int)g_devs.size();
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return fail(DPF_ERR_NODEV, "dpf: no HIP device visible (gfx950 required)");
    if (ngpus > 0) n = std::min(n, ngpus);
    std::vector<int> ids;
    for (int i = 0; i < n; ++i) ids.push_back(i);
    return open_list(ids);
}

// The opened devices, opening every visible one on first use.  Returns an
// empty list (and sets the error) when none can be opened.
DevList devices(int* rc) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_devs.empty()) {
            *rc = (int)g_devs.size();
            return g_devs;
        }
    }
    *rc = open_devices(0);
    std::lock_guard<std::mutex> lk(g_mu);
    return *rc > 0 ? g_devs : DevList{};
}

// The reference reads k[0:17], the level records k[17+18i : 17+18i+18] for
// i < stop and the final CW at k[len-16 : len] (dpf.go:175-176,186-188,206,
// 219,231-233): any key of at least 17 + 18*stop bytes evaluates without an
// index panic, including keys whose final CW overlaps the last record.
// EvalFull (full) with logN > 63 cannot allocate its 2^(logN-3)-byte output
// (dpf.go:251 panics in makeslice): DPF_ERR_PARAM.  Eval validates no logN
// (dpf.go:171-211): any logN with a long enough key evaluates, its path bits
// above bit 63 read as 0 (path_bit).
int check_key(size_t klen, uint32_t logN, bool full = true) {
    if (full && logN > 63) return fail(DPF_ERR_PARAM, "dpf: logN > 63");
    if (klen < 17 + 18 * (size_t)stop_of(logN)) return fail(DPF_ERR_KEYLEN, "dpf: key shorter than 17+18*(logN-7) bytes");
    return DPF_OK;
}

// ---- AES back end of the tree kernels (configs[1]: bitsliced vs T-table) --
// DPF_AES_IMPL=bitsliced|ttable sets the default; dpf_set_aes_impl switches
// at run time.  Both give bit-identical outputs.
std::atomic<int> g_aes_impl{[] {
    const char* e = getenv("DPF_AES_IMPL");
    return e && (e[0] == 'b' || e[0] == 'B') ? DPF_AES_BITSLICED : DPF_AES_TTABLE;
}()};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Tree workspace for nk expanded keys: [T-table records | byte-sliced CW
// words | byte-sliced frontier for up to `chunk` keys per launch].
size_t tree_ws_bytes(size_t nk, uint32_t stop, uint32_t prefix_bits, size_t chunk) {
    return align256(nk * dpfk::ek_words(stop) * 4) + align256(nk * dpfk::bs_key_words(stop) * 4) +
           dpfk::bs_frontier_bytes(chunk, stop, prefix_bits);
}

struct TreeWs {
    uint32_t* ek;
    uint32_t* ekb;
    void* frontier;
};

TreeWs tree_ws(void* work, size_t nk, uint32_t stop) {
    uint8_t* p = static_cast<uint8_t*>(work);
    TreeWs w;
    w.ek = reinterpret_cast<uint32_t*>(p);
    p += align256(nk * dpfk::ek_words(stop) * 4);
    w.ekb = reinterpret_cast<uint32_t*>(p);
    p += align256(nk * dpfk::bs_key_words(stop) * 4);
    w.frontier = p;
    return w;
}

// The back end a call uses, decided once per call (expansion and launches agree).
bool want_bs() { return g_aes_impl.load(std::memory_order_relaxed) == DPF_AES_BITSLICED; }

// Key records: the T-table's 8-word records always; the byte-sliced planes
// (7.6 MB at configs[1], 2/3 of the unpack time) only for the byte-sliced back end.
hipError_t expand_keys(const uint8_t* d_keys, size_t klen, size_t nk, uint32_t stop, const TreeWs& w, hipStream_t st,
                       bool bs) {
    if (bs) return dpfk::launch_unpack_both(d_keys, klen, nk, stop, w.ek, w.ekb, st);
    return dpfk::launch_unpack(d_keys, klen, nk, stop, w.ek, st);
}

// Leaves of subtree (prefix_bits, prefix) of keys [k0, k0 + n): byte-sliced
// when bs (its records expanded) and the subtree is deep enough, else T-table.
hipError_t run_tree(const TreeWs& w, size_t k0, size_t n, uint32_t stop, uint32_t prefix_bits, uint64_t prefix,
                    uint8_t* out, uint64_t stride, hipStream_t st, bool bs) {
    if (bs && dpfk::bs_applicable(stop, prefix_bits))
        return dpfk::launch_evalfull_bs(w.ek + k0 * dpfk::ek_words(stop), w.ekb + k0 * dpfk::bs_key_words(stop), n, stop,
                                        prefix_bits, prefix, out, stride, w.frontier, st);
    return dpfk::launch_evalfull(w.ek + k0 * dpfk::ek_words(stop), n, stop, prefix_bits, prefix, out, stride, st);
}

// One-shot tree pass from the key bytes in HBM: straight from the bytes when
// the T-table back end runs a wave-uniform shape (dpfk::evalfull_raw_ok: no
// unpack launch, d_work untouched), else expand into d_work and run.
hipError_t tree_from_keys(const uint8_t* d_keys, size_t klen, size_t nk, uint32_t stop, uint32_t prefix_bits,
                          uint64_t prefix, uint8_t* out, uint64_t stride, void* d_work, hipStream_t st, bool bs,
                          bool* expanded) {
    if (!bs && dpfk::evalfull_raw_ok(nk, stop, prefix_bits)) {
        *expanded = false;
        return dpfk::launch_evalfull_raw(d_keys, klen, nk, stop, prefix_bits, prefix, out, stride, st);
    }
    *expanded = true;
    const TreeWs w = tree_ws(d_work, nk, stop);
    hipError_t e = expand_keys(d_keys, klen, nk, stop, w, st, bs);
    return e != hipSuccess ? e : run_tree(w, 0, nk, stop, prefix_bits, prefix, out, stride, st, bs);
}

// Pipelined device -> host output of `nchunks` chunks (<= chunk_cap bytes
// each).  produce(i, dbuf, bytes, host_off) enqueues the kernels writing
// chunk i into device slot dbuf on d.st.  Kernel i, the PCIe copy of chunk
// i-1 (d.cst, into a pinned slot) and the host copy of chunk i-2 (pinned ->
// caller buffer, CopyPool) overlap; two device and two pinned slots.
constexpr size_t kStageBytes = (size_t)32 << 20;
constexpr size_t kSlabMinOut = (size_t)8 << 20;    // one key's output from which it is cut into >= 4 slabs

int ensure_staging(Dev& d, size_t chunk_cap) {
    if (!d.cst) {
        HIP_TRY(hipStreamCreateWithFlags(&d.cst, hipStreamNonBlocking));
        for (int i = 0; i < 2; ++i) {
            HIP_TRY(hipEventCreateWithFlags(&d.ev_k[i], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&d.ev_c[i], hipEventDisableTiming));
        }
    }
    HIP_TRY(hipError_t(d.out.ensure(2 * chunk_cap)));
    for (int i = 0; i < 2; ++i) HIP_TRY(d.pin[i].ensure(chunk_cap));
    return DPF_OK;
}

// Opt-in (DPF_PREFAULT_OUTPUT=1): for large caller buffers (a fresh Go
// slice / numpy array), ask for transparent huge pages and pre-touch the
// pages in parallel while the GPU works, so first touch costs one fault per
// 2 MiB instead of per 4 KiB inside the copy.  Off by default: it changes
// the memory policy of caller-owned memory (a Go heap manages THP itself)
// and zero-writes the buffer before data arrives.
bool prefault_output() {
    static const bool on = [] {
        const char* e = getenv("DPF_PREFAULT_OUTPUT");
        return e && e[0] == '1';
    }();
    return on;
}

void hint_hugepages(uint8_t* p, size_t n) {
    if (n < ((size_t)64 << 20) || !prefault_output()) return;
    const uintptr_t a = ((uintptr_t)p + ((1u << 21) - 1)) & ~(uintptr_t)((1u << 21) - 1);
    const uintptr_t e = ((uintptr_t)p + n) & ~(uintptr_t)((1u << 21) - 1);
    if (e > a) (void)madvise((void*)a, e - a, MADV_HUGEPAGE);
}

template <class Produce>
int pipeline_d2h(Dev& d, size_t nchunks, size_t chunk_cap, Produce produce, uint8_t* out, size_t out_bytes,
                 size_t out_base = 0) {
    // Chunk i lands at out + off_i - out_base; [out, out + out_bytes) is the whole destination.
    if (nchunks == 0) return DPF_OK;
    hint_hugepages(out, out_bytes);
    if (int rc = ensure_staging(d, chunk_cap)) return rc;
    size_t bytes[2] = {0, 0}, off[2] = {0, 0};
    auto drain = [&](size_t i) -> int {              // chunk i: wait for its PCIe copy, then host copy
        const int s = (int)(i & 1);
        HIP_TRY(hipEventSynchronize(d.ev_c[s]));
        CopyPool::get().memcpy_par(out + (off[s] - out_base), d.pin[s].p, bytes[s]);
        return DPF_OK;
    };
    for (size_t i = 0; i < nchunks; ++i) {
        const int s = (int)(i & 1);
        uint8_t* dbuf = (uint8_t*)d.out.p + (size_t)s * chunk_cap;
        if (i >= 2) HIP_TRY(hipStreamWaitEvent(d.st, d.ev_c[s], 0));   // slot's previous PCIe copy done
        if (int rc = produce(i, dbuf, bytes[s], off[s])) return rc;
        HIP_TRY(hipEventRecord(d.ev_k[s], d.st));
        HIP_TRY(hipStreamWaitEvent(d.cst, d.ev_k[s], 0));
        HIP_TRY(hipMemcpyAsync(d.pin[s].p, dbuf, bytes[s], hipMemcpyDeviceToHost, d.cst));
        HIP_TRY(hipEventRecord(d.ev_c[s], d.cst));
        if (i == std::min<size_t>(1, nchunks - 1) && out_bytes >= ((size_t)64 << 20) && prefault_output())
            CopyPool::get().prefault_par(out, out_bytes);   // while the GPU works on chunks 0-1
        if (i >= 1)
            if (int rc = drain(i - 1)) return rc;          // frees pinned slot (i-1)&1 for chunk i+1
    }
    return drain(nchunks - 1);
}

// Host-buffer EvalFull of keys [0, nk) on one device.  Chunks are groups of
// whole keys, or subtree slabs of one key when its output exceeds a chunk.
int full_on_device(Dev& d, const uint8_t* keys, size_t klen, size_t nk, uint32_t logN, uint8_t* out) {
    std::lock_guard<std::mutex> lk(d.mu);
    DeviceGuard g(d.id);
    const uint32_t stop = stop_of(logN);
    const size_t olen = full_len(logN);
    const size_t per = olen <= kStageBytes ? kStageBytes / olen : 1;   // keys per chunk
    HIP_TRY(hipError_t(d.keys.ensure(nk * klen)));
    HIP_TRY(hipError_t(d.work.ensure(tree_ws_bytes(nk, stop, 0, std::min(per, nk)))));
    HIP_TRY(hipMemcpyAsync(d.keys.p, keys, nk * klen, hipMemcpyHostToDevice, d.st));
    const TreeWs w = tree_ws(d.work.p, nk, stop);
    const bool bs = want_bs();
    const uint8_t* dk = (const uint8_t*)d.keys.p;
    uint32_t pb = 0;                                      // one key's output exceeds a chunk: subtree slabs
    while ((olen >> pb) > kStageBytes) ++pb;
    // A key whose output is >= kSlabMinOut goes in >= 4 subtree slabs even
    // when it fits one chunk, so its kernel, PCIe copy and host copy overlap
    // (BenchmarkEvalFull's logN = 28 is one 32 MiB key: as one chunk, the
    // three ran back to back).
    if (olen >= kSlabMinOut && pb < 2) pb = 2;
    // Every chunk straight from the key bytes when each chunk shape allows it
    // (tree_from_keys), else the keys are expanded once for all chunks.
    const bool raw = !bs && (pb == 0 ? dpfk::evalfull_raw_ok(std::min(per, nk), stop, 0) &&
                                                       (nk % per == 0 || dpfk::evalfull_raw_ok(nk % per, stop, 0))
                                                 : dpfk::evalfull_raw_ok(1, stop, pb));
    if (!raw) HIP_TRY(expand_keys(dk, klen, nk, stop, w, d.st, bs));
    if (pb == 0) {
        const size_t nch = (nk + per - 1) / per;
        return pipeline_d2h(d, nch, std::min(per, nk) * olen, [&](size_t i, uint8_t* dbuf, size_t& bytes, size_t& off) {
            const size_t k0 = i * per, n = std::min(per, nk - k0);
            if (raw) HIP_TRY(dpfk::launch_evalfull_raw(dk + k0 * klen, klen, n, stop, 0, 0, dbuf, olen, d.st));
            else HIP_TRY(run_tree(w, k0, n, stop, 0, 0, dbuf, olen, d.st, bs));
            bytes = n * olen;
            off = k0 * olen;
            return DPF_OK;
        }, out, nk * olen);
    }
    const size_t slab = olen >> pb, per_key = (size_t)1 << pb;
    return pipeline_d2h(d, nk * per_key, slab, [&](size_t i, uint8_t* dbuf, size_t& bytes, size_t& off) {
        const size_t k = i / per_key, p = i % per_key;
        if (raw) HIP_TRY(dpfk::launch_evalfull_raw(dk + k * klen, klen, 1, stop, pb, p, dbuf, slab, d.st));
        else HIP_TRY(run_tree(w, k, 1, stop, pb, p, dbuf, slab, d.st, bs));
        bytes = slab;
        off = k * olen + p * slab;
        return DPF_OK;
    }, out, nk * olen);
}

size_t pir_ek_bytes(size_t nkeys, uint32_t logN);
size_t eval_work_bytes(size_t nkeys, size_t ppk, uint32_t logN);

// Host-buffer batched Eval on one device, pipelined over chunks of keys:
// caller xs -> pinned (CopyPool) -> HBM (d.hst) -> k_eval (d.st) -> pinned
// (d.cst) -> caller out, two slots per stage, so chunk i's kernel overlaps
// the PCIe copies of its neighbours.
int eval_on_device(Dev& d, const uint8_t* keys, size_t klen, size_t nk, const uint64_t* xs, size_t ppk,
                   uint32_t logN, uint8_t* out) {
    std::lock_guard<std::mutex> lk(d.mu);
    DeviceGuard g(d.id);
    const uint32_t stop = stop_of(logN);
    const size_t ekw = dpfk::ek_words(stop);
    const size_t per = std::max<size_t>(1, std::min(nk, kStageBytes / (ppk * 8)));   // keys per chunk
    const size_t nch = (nk + per - 1) / per;
    const size_t ekb = pir_ek_bytes(nk, logN);
    const size_t fbytes = dpfk::eval_frontier_bytes(per, stop, ppk);
    const size_t qcap = per * ppk;                        // queries per chunk
    HIP_TRY(hipError_t(d.keys.ensure(std::max<size_t>(1, nk * klen))));
    HIP_TRY(hipError_t(d.work.ensure(std::max<size_t>(16, ekb + fbytes))));
    HIP_TRY(hipError_t(d.xs.ensure(2 * qcap * 8)));
    if (int rc = ensure_staging(d, qcap)) return rc;      // d.out: 2 x qcap result bytes
    for (int i = 0; i < 2; ++i) HIP_TRY(d.pin[i].ensure(qcap * 9));   // [xs qcap*8][results qcap]
    if (!d.hst) {
        HIP_TRY(hipStreamCreateWithFlags(&d.hst, hipStreamNonBlocking));
        for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreateWithFlags(&d.ev_h[i], hipEventDisableTiming));
    }
    HIP_TRY(hipMemcpyAsync(d.keys.p, keys, nk * klen, hipMemcpyHostToDevice, d.st));
    HIP_TRY(dpfk::launch_unpack((const uint8_t*)d.keys.p, klen, nk, stop, (uint32_t*)d.work.p, d.st));
    const uint32_t* ek = (const uint32_t*)d.work.p;
    void* frontier = (uint8_t*)d.work.p + ekb;
    auto drain = [&](size_t i) -> int {
        const int s = (int)(i & 1);
        const size_t k0 = i * per, q = std::min(per, nk - k0) * ppk;
        HIP_TRY(hipEventSynchronize(d.ev_c[s]));
        CopyPool::get().memcpy_par(out + k0 * ppk, (uint8_t*)d.pin[s].p + qcap * 8, q);
        return DPF_OK;
    };
    for (size_t i = 0; i < nch; ++i) {
        const int s = (int)(i & 1);
        const size_t k0 = i * per, n = std::min(per, nk - k0), q = n * ppk;
        uint8_t* pin = (uint8_t*)d.pin[s].p;
        uint64_t* dxs = (uint64_t*)d.xs.p + (size_t)s * qcap;
        uint8_t* dout = (uint8_t*)d.out.p + (size_t)s * qcap;
        CopyPool::get().memcpy_par(pin, xs + k0 * ppk, q * 8);
        if (i >= 2) HIP_TRY(hipStreamWaitEvent(d.hst, d.ev_k[s], 0));   // slot's previous kernel read its xs
        HIP_TRY(hipMemcpyAsync(dxs, pin, q * 8, hipMemcpyHostToDevice, d.hst));
        HIP_TRY(hipEventRecord(d.ev_h[s], d.hst));
        HIP_TRY(hipStreamWaitEvent(d.st, d.ev_h[s], 0));
        if (i >= 2) HIP_TRY(hipStreamWaitEvent(d.st, d.ev_c[s], 0));    // slot's previous results copied out
        HIP_TRY(dpfk::launch_eval(ek + k0 * ekw, stop, logN, dxs, q, ppk, dout, frontier, fbytes, d.st));
        HIP_TRY(hipEventRecord(d.ev_k[s], d.st));
        HIP_TRY(hipStreamWaitEvent(d.cst, d.ev_k[s], 0));
        HIP_TRY(hipMemcpyAsync(pin + qcap * 8, dout, q, hipMemcpyDeviceToHost, d.cst));
        HIP_TRY(hipEventRecord(d.ev_c[s], d.cst));
        if (i >= 1)
            if (int rc = drain(i - 1)) return rc;
    }
    return drain(nch - 1);
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

// The first min(ngpus, opened) devices (ngpus <= 0: all); empty + error set on failure.
DevList pick_devs(int ngpus, int* rc) {
    DevList devs = devices(rc);
    if (*rc <= 0) return {};
    if (ngpus > 0 && (size_t)ngpus < devs.size()) devs.resize((size_t)ngpus);
    *rc = (int)devs.size();
    return devs;
}

// Expanded keys at the start of a PIR workspace, padded to 256 B.
size_t pir_ek_bytes(size_t nkeys, uint32_t logN) {
    return (nkeys * dpfk::ek_words(stop_of(logN)) * 4 + 255) & ~(size_t)255;
}

// Batched-Eval workspace: expanded keys (256-B padded), then the frontier.
size_t eval_work_bytes(size_t nkeys, size_t ppk, uint32_t logN) {
    return pir_ek_bytes(nkeys, logN) + dpfk::eval_frontier_bytes(nkeys, stop_of(logN), ppk);
}

// The expanded form's layout depends on (nkeys, stop) (tree_ws), so each
// expanded workspace is recorded here and dpf_evalfull_expanded_dev refuses
// one expanded for another shape instead of reading misplaced records.
std::mutex g_exp_mu;
// Also records whether the byte-sliced planes were built: the T-table back
// end expands only its own records, and switching to the byte-sliced one
// later derives them from those (launch_bs_from_ek) on first use.
struct Expanded {
    size_t nkeys;
    uint32_t stop;
    bool bs;
};
std::unordered_map<const void*, Expanded>& g_expanded = *new std::unordered_map<const void*, Expanded>();

// Every entry point that expands keys into a caller's d_work records what it
// left there (the same tree_ws layout), so a later dpf_evalfull_expanded_dev
// never reads planes built from other keys; dpf_eval_batch_dev's workspace
// has another layout past the records and is dropped.
void note_expanded(const void* d_work, size_t nkeys, uint32_t stop, bool bs) {
    std::lock_guard<std::mutex> lk(g_exp_mu);
    g_expanded[d_work] = {nkeys, stop, bs};
}
void forget_expanded(const void* d_work) {
    std::lock_guard<std::mutex> lk(g_exp_mu);
    g_expanded.erase(d_work);
}

}  // namespace

extern "C" {

const char* dpf_last_error(void) { return t_err.c_str(); }

size_t dpf_key_len(uint32_t logN) { return key_len(logN); }
size_t dpf_evalfull_len(uint32_t logN) { return full_len(logN); }
size_t dpf_workspace_size(size_t nkeys, uint32_t logN) {
    return std::max<size_t>(16, tree_ws_bytes(nkeys, stop_of(logN), 0, nkeys));
}

int dpf_set_aes_impl(int impl) {
    if (impl != DPF_AES_TTABLE && impl != DPF_AES_BITSLICED) return fail(DPF_ERR_PARAM, "dpf: unknown AES back end");
    return g_aes_impl.exchange(impl);
}

int dpf_get_aes_impl(void) { return g_aes_impl.load(); }

int dpf_set_eval_kernel(int kernel) {
    if (kernel != DPF_EVAL_WALK && kernel != DPF_EVAL_TRIE) return fail(DPF_ERR_PARAM, "dpf: unknown Eval kernel");
    if (kernel == DPF_EVAL_TRIE && !dpfk::eval_trie_built())
        return fail(DPF_ERR_PARAM, "dpf: the trie Eval kernel is not in this build (make -C dpf-go_amd experimental)");
    return dpfk::set_eval_trie(kernel == DPF_EVAL_TRIE) ? DPF_EVAL_TRIE : DPF_EVAL_WALK;
}

int dpf_get_eval_kernel(void) { return dpfk::get_eval_trie() ? DPF_EVAL_TRIE : DPF_EVAL_WALK; }

int dpf_aes_mmo_dev(int device, int impl, int right, const uint8_t* d_in, uint8_t* d_out, size_t nblocks,
                    uint32_t reps, void* stream) {
    if (impl != DPF_AES_TTABLE && impl != DPF_AES_BITSLICED) return fail(DPF_ERR_PARAM, "dpf: unknown AES back end");
    if (nblocks % 8) return fail(DPF_ERR_PARAM, "dpf: nblocks must be a multiple of 8");
    DeviceGuard g(device);
    if (impl == DPF_AES_BITSLICED)
        HIP_TRY(dpfk::launch_mmo_bs(d_in, d_out, nblocks, right ? 1u : 0u, reps, (hipStream_t)stream));
    else
        HIP_TRY(dpfk::launch_mmo_tt(d_in, d_out, nblocks, right ? 1u : 0u, reps, (hipStream_t)stream));
    return DPF_OK;
}

int dpf_gpu_init(int ngpus) { return open_devices(ngpus); }

int dpf_gpu_init_devices(const int* ordinals, int n) {
    if (n <= 0 || ordinals == nullptr) return fail(DPF_ERR_PARAM, "dpf: empty device list");
    std::vector<int> ids(ordinals, ordinals + n);
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_devs.empty()) {
        bool same = g_devs.size() == ids.size();
        for (size_t i = 0; same && i < ids.size(); ++i) same = g_devs[i]->id == ids[i];
        if (!same) return fail(DPF_ERR_PARAM, "dpf: already initialised with other devices (dpf_gpu_shutdown first)");
        return (int)g_devs.size();
    }
    return open_list(ids);
}

void dpf_gpu_shutdown(void) {
    DevList old;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        old.swap(g_devs);
        g_ndevs.store(0);
    }
    // Dropping the registry's references; a device still used by an
    // in-flight call or a PIR handle is released when that lets go.
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

int dpf_keys_pack(const uint8_t* const* keys, const size_t* lens, size_t n, size_t key_len, uint8_t* out) {
    int rc = dpfh::keys_pack(keys, lens, n, key_len, out);
    return rc == DPF_ERR_KEYLEN ? fail(rc, "dpf: key length differs from the batch's key_len")
           : rc                ? fail(rc, "dpf: invalid parameters")
                               : DPF_OK;
}

int dpf_keys_unpack(const uint8_t* packed, size_t key_len, size_t n, uint8_t* const* keys) {
    int rc = dpfh::keys_unpack(packed, key_len, n, keys);
    return rc ? fail(rc, "dpf: invalid parameters") : DPF_OK;
}

int dpf_evalfull_batch(const uint8_t* keys, size_t klen, size_t nkeys, uint32_t logN, uint8_t* out, int ngpus) {
    if (int rc = check_key(klen, logN)) return rc;
    if (nkeys == 0) return DPF_OK;
    int g = 0;
    const DevList devs = pick_devs(ngpus, &g);
    if (g <= 0) return g;
    const size_t olen = full_len(logN);
    return shard(nkeys, g, [&](int dev, size_t lo, size_t hi) {
        return full_on_device(*devs[(size_t)dev], keys + lo * klen, klen, hi - lo, logN, out + lo * olen);
    });
}

// ---- small-call path (host_eval.cpp) ------------------------
std::atomic<int> g_small_mode{[] {
    const char* e = getenv("DPF_SMALL_CALLS");
    if (!e) return DPF_SMALL_AUTO;
    if (e[0] == 'g' || e[0] == 'G') return DPF_SMALL_GPU;
    if (e[0] == 'h' || e[0] == 'H') return DPF_SMALL_HOST;
    return DPF_SMALL_AUTO;
}()};

// Largest logN whose single-key EvalFull goes to the host in AUTO mode: up
// to it, one key's host EvalFull (3*2^(logN-7) AES on VAES) is faster than
// the GPU round trip (key H2D, launch, output D2H, sync) -- measured on the
// GPU box's EPYC (profiles/r03/small_calls; r05: host 69 us vs GPU 89 us at
// 21, 137 vs 105 at 22, profiles/r05/small_calls/small_vaes.json).
constexpr uint32_t kSmallFullMaxLogN = 21;
// Without VAES (DPF_HOST_ISA=aesni: two 128-bit AES-NI chains per node) the
// host path is ~2x slower at these sizes; measured crossover logN = 20: host
// 72 us vs GPU 83 us at 20, 138 vs 100 at 21
// (profiles/r05/small_calls/small_aesni.json; r04's 19 was an estimate).
constexpr uint32_t kSmallFullMaxLogNNoVaes = 20;
// DPF_SMALL_HOST's ceiling: two host-side levels of the full width (~2.1x the
// output) and one core; above it the call goes to the GPU.
constexpr uint32_t kHostFullMaxLogN = 28;
uint32_t small_full_max() { return dpfh::host_eval_vaes() ? kSmallFullMaxLogN : kSmallFullMaxLogNNoVaes; }

int dpf_set_small_call_path(int mode) {
    if (mode != DPF_SMALL_AUTO && mode != DPF_SMALL_GPU && mode != DPF_SMALL_HOST)
        return fail(DPF_ERR_PARAM, "dpf: unknown small-call mode");
    return g_small_mode.exchange(mode);
}
int dpf_get_small_call_path(void) { return g_small_mode.load(); }
uint32_t dpf_small_call_max_logN(void) { return small_full_max(); }

// Route a single call to the host?  Only with a gfx950 device open (so the
// host path is never a stand-in for a missing GPU) and AES-NI present.
// Returns 1 = host, 0 = GPU, < 0 = error (no device).
int route_host(bool full, uint32_t logN) {
    const int mode = g_small_mode.load(std::memory_order_relaxed);
    if (mode == DPF_SMALL_GPU || !dpfh::host_eval_available()) return 0;
    if (g_ndevs.load(std::memory_order_acquire) <= 0) {   // open on first use, as the GPU path would
        int g = 0;
        (void)pick_devs(1, &g);
        if (g <= 0) return g;
    }
    if (mode == DPF_SMALL_HOST) return !full || logN <= kHostFullMaxLogN ? 1 : 0;
    return !full || logN <= small_full_max() ? 1 : 0;
}

int dpf_evalfull(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out) {
    if (int rc = check_key(klen, logN)) return rc;
    const int h = route_host(true, logN);
    if (h < 0) return h;
    if (h) {
        try {
            dpfh::evalfull_host(key, klen, logN, out);
        } catch (const std::bad_alloc&) {
            return fail(DPF_ERR_NOMEM, "dpf: host EvalFull allocation failed");
        }
        return DPF_OK;
    }
    return dpf_evalfull_batch(key, klen, 1, logN, out, 1);
}

int dpf_eval_batch(const uint8_t* keys, size_t klen, size_t nkeys, const uint64_t* xs, size_t ppk, uint32_t logN,
                   uint8_t* out, int ngpus) {
    if (int rc = check_key(klen, logN, false)) return rc;
    if (nkeys == 0 || ppk == 0) return DPF_OK;
    int g = 0;
    const DevList devs = pick_devs(ngpus, &g);
    if (g <= 0) return g;
    return shard(nkeys, g, [&](int dev, size_t lo, size_t hi) {
        return eval_on_device(*devs[(size_t)dev], keys + lo * klen, klen, hi - lo, xs + lo * ppk, ppk, logN,
                              out + lo * ppk);
    });
}

int dpf_eval(const uint8_t* key, size_t klen, uint64_t x, uint32_t logN, uint8_t* out_bit) {
    if (int rc = check_key(klen, logN, false)) return rc;
    const int h = route_host(false, logN);
    if (h < 0) return h;
    if (h) {
        dpfh::eval_batch_host(key, klen, 1, &x, 1, logN, out_bit);
        return DPF_OK;
    }
    return dpf_eval_batch(key, klen, 1, &x, 1, logN, out_bit, 1);
}

int dpf_evalfull_split(const uint8_t* key, size_t klen, uint32_t logN, uint8_t* out, int ngpus) {
    if (int rc = check_key(klen, logN)) return rc;
    int have = 0;
    const DevList devs = pick_devs(0, &have);
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
        Dev& d = *devs[(size_t)dev];
        std::lock_guard<std::mutex> lk(d.mu);
        DeviceGuard gd(d.id);
        HIP_TRY(hipError_t(d.keys.ensure(klen)));
        HIP_TRY(hipError_t(d.work.ensure(tree_ws_bytes(1, stop, pb, 1))));
        HIP_TRY(hipMemcpyAsync(d.keys.p, key, klen, hipMemcpyHostToDevice, d.st));
        const TreeWs w = tree_ws(d.work.p, 1, stop);
        const bool bs = want_bs();
        const uint8_t* dk = (const uint8_t*)d.keys.p;
        // This device's subtree (pb, lo), streamed out in sub-slabs (pb + extra, lo * 2^extra + j).
        uint32_t extra = 0;
        while ((slab >> extra) > kStageBytes && pb + extra < stop) ++extra;
        const size_t sub = slab >> extra;
        const bool raw = !bs && dpfk::evalfull_raw_ok(1, stop, pb + extra);
        if (!raw) HIP_TRY(expand_keys(dk, klen, 1, stop, w, d.st, bs));
        return pipeline_d2h(d, (size_t)1 << extra, sub, [&](size_t j, uint8_t* dbuf, size_t& bytes, size_t& off) {
            const uint64_t p = ((uint64_t)lo << extra) + j;
            if (raw) HIP_TRY(dpfk::launch_evalfull_raw(dk, klen, 1, stop, pb + extra, p, dbuf, sub, d.st));
            else HIP_TRY(run_tree(w, 0, 1, stop, pb + extra, p, dbuf, sub, d.st, bs));
            bytes = sub;
            off = lo * slab + j * sub;
            return DPF_OK;
        }, out + lo * slab, slab, lo * slab);
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
    CuScope cus(stream);
    const bool bs = want_bs();
    bool expanded = false;
    forget_expanded(d_work);
    HIP_TRY(tree_from_keys(d_keys, klen, nkeys, stop, prefix_bits, prefix, d_out, (uint64_t)16 << (stop - prefix_bits),
                           d_work, (hipStream_t)stream, bs, &expanded));
    if (expanded) note_expanded(d_work, nkeys, stop, bs);
    return DPF_OK;
}

int dpf_evalfull_batch_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN,
                           uint8_t* d_out, void* d_work, void* stream) {
    return dpf_evalfull_subtree_dev(device, d_keys, klen, nkeys, logN, 0, 0, d_out, d_work, stream);
}

size_t dpf_eval_workspace_size(size_t nkeys, size_t pts_per_key, uint32_t logN) {
    return std::max<size_t>(16, eval_work_bytes(nkeys, pts_per_key, logN));
}

uint32_t dpf_eval_frontier_level(uint32_t logN, size_t pts_per_key) {
    return logN > 63 ? 0 : dpfk::eval_frontier_level(stop_of(logN), pts_per_key);   // launch_eval: no frontier above 63
}

int dpf_eval_batch_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, const uint64_t* d_xs,
                       size_t ppk, uint32_t logN, uint8_t* d_out, void* d_work, size_t work_bytes, void* stream) {
    if (int rc = check_key(klen, logN, false)) return rc;
    if (nkeys == 0 || ppk == 0) return DPF_OK;
    const uint32_t stop = stop_of(logN);
    const size_t ekb = pir_ek_bytes(nkeys, logN);
    if (work_bytes < nkeys * dpfk::ek_words(stop) * 4) return fail(DPF_ERR_PARAM, "dpf: Eval workspace too small");
    if (d_xs == nullptr || d_out == nullptr || d_keys == nullptr || (reinterpret_cast<uintptr_t>(d_xs) & 7u) != 0)
        return fail(DPF_ERR_PARAM, "dpf: d_keys/d_xs/d_out must be device pointers, d_xs 8-byte aligned");
    DeviceGuard g(device);
    CuScope cus(stream);
    forget_expanded(d_work);
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
    CuScope cus(stream);
    const bool bs = want_bs();
    forget_expanded(d_work);
    HIP_TRY(expand_keys(d_keys, klen, nkeys, stop_of(logN), tree_ws(d_work, nkeys, stop_of(logN)), (hipStream_t)stream,
                        bs));
    note_expanded(d_work, nkeys, stop_of(logN), bs);
    return DPF_OK;
}

int dpf_forget_workspace(const void* d_work) {
    forget_expanded(d_work);
    return DPF_OK;
}

int dpf_evalfull_expanded_dev(int device, void* d_work, size_t nkeys, uint32_t logN, uint32_t prefix_bits,
                              uint64_t prefix, uint8_t* d_out, void* stream) {
    if (logN > 63) return fail(DPF_ERR_PARAM, "dpf: logN > 63");
    const uint32_t stop = stop_of(logN);
    if (prefix_bits > stop || (prefix >> prefix_bits) != 0) return fail(DPF_ERR_PARAM, "dpf: subtree prefix out of range");
    if (nkeys == 0) return DPF_OK;
    const bool bs = want_bs();
    bool build_bs = false;
    {
        std::lock_guard<std::mutex> lk(g_exp_mu);
        const auto it = g_expanded.find(d_work);
        if (it == g_expanded.end() || it->second.nkeys != nkeys || it->second.stop != stop)
            return fail(DPF_ERR_PARAM, "dpf: d_work was not expanded by dpf_expand_keys_dev for this nkeys and logN");
        build_bs = bs && !it->second.bs;
    }
    DeviceGuard g(device);
    CuScope cus(stream);
    const TreeWs w = tree_ws(d_work, nkeys, stop);
    if (build_bs) {
        HIP_TRY(dpfk::launch_bs_from_ek(w.ek, nkeys, stop, w.ekb, (hipStream_t)stream));
        note_expanded(d_work, nkeys, stop, true);   // only once the planes' launch is enqueued
    }
    const uint64_t stride = (uint64_t)16 << (stop - prefix_bits);
    HIP_TRY(run_tree(w, 0, nkeys, stop, prefix_bits, prefix, d_out, stride, (hipStream_t)stream, bs));
    return DPF_OK;
}

// ------------------------------------------------------------------ PIR ---

// Device buffers of the PIR answer entry points: present when there is work
// for them, and aligned as the kernels access them (DB 16 B, answers and
// workspace as u32 words), so a bad buffer is DPF_ERR_PARAM, not a GPU fault.
static int check_pir_bufs(const void* d_keys, size_t nkeys, const void* d_db, uint64_t nrec, const void* d_ans,
                          const void* d_work) {
    if (nkeys > 0 && (!d_keys || !d_ans || !d_work || (nrec > 0 && !d_db)))
        return fail(DPF_ERR_PARAM, "dpf: null device buffer");
    if ((uintptr_t)d_db % 16 != 0 || (uintptr_t)d_ans % 4 != 0 || (uintptr_t)d_work % 16 != 0)
        return fail(DPF_ERR_PARAM, "dpf: misaligned device buffer");
    return DPF_OK;
}

size_t dpf_pir_workspace_size(size_t nkeys, uint32_t logN, uint32_t prefix_bits) {
    const uint32_t stop = stop_of(logN);
    const uint32_t pb = prefix_bits > stop ? stop : prefix_bits;
    return align256(tree_ws_bytes(nkeys, stop, pb, nkeys)) + align256(nkeys * ((size_t)16 << (stop - pb))) +
           dpfk::pir_fold_parts_bytes();
}

int dpf_pir_answer_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN,
                       uint32_t prefix_bits, uint64_t prefix, const uint8_t* d_db, uint64_t nrec, uint8_t* d_ans,
                       void* d_work, void* stream) {
    if (int rc = check_key(klen, logN)) return rc;
    const uint32_t stop = stop_of(logN);
    if (prefix_bits > stop || (prefix >> prefix_bits) != 0) return fail(DPF_ERR_PARAM, "dpf: subtree prefix out of range");
    const uint64_t slice = logN - prefix_bits >= 64 ? ~0ull : (1ull << (logN - prefix_bits));
    if (nrec > slice) return fail(DPF_ERR_PARAM, "dpf: more DB records than the subtree's domain");
    if (int rc = check_pir_bufs(d_keys, nkeys, d_db, nrec, d_ans, d_work)) return rc;
    DeviceGuard g(device);
    CuScope cus(stream);
    hipStream_t st = (hipStream_t)stream;
    if (nkeys == 0) return DPF_OK;
    if (nrec == 0) {
        HIP_TRY(hipMemsetAsync(d_ans, 0, nkeys * 32, st));
        return DPF_OK;
    }
    // [tree workspace | selection bits = EvalFull bytes of the subtree | fold partials]
    uint8_t* bits = (uint8_t*)d_work + align256(tree_ws_bytes(nkeys, stop, prefix_bits, nkeys));
    const uint64_t per_key = (uint64_t)16 << (stop - prefix_bits);
    const bool bs = want_bs();
    bool expanded = false;
    forget_expanded(d_work);
    HIP_TRY(tree_from_keys(d_keys, klen, nkeys, stop, prefix_bits, prefix, bits, per_key, d_work, st, bs, &expanded));
    if (expanded) note_expanded(d_work, nkeys, stop, bs);
    uint32_t* parts = (uint32_t*)(bits + align256(nkeys * per_key));
    HIP_TRY(dpfk::launch_pir_fold((const uint32_t*)bits, per_key / 4, d_db, nrec, 32, (uint32_t)nkeys, (uint32_t*)d_ans,
                                  parts, st));
    return DPF_OK;
}

// PIR kernel over the sliced DB: the tree launch then the fold launch
// (DPF_PIR_SPLIT, the default: measured faster), or both in one launch
// where it applies (DPF_PIR_FUSED, k_pir_fused).  DPF_PIR_KERNEL=split|
// fused|fused-any sets the start value; in a build without k_pir_fused the
// environment value falls back to split, as dpf_set_pir_kernel refuses it.
std::atomic<int> g_pir_kernel{[] {
    const char* e = getenv("DPF_PIR_KERNEL");
    if (!dpfk::pir_fused_built()) return DPF_PIR_SPLIT;
    if (e && strcmp(e, "fused-any") == 0) return DPF_PIR_FUSED_ANY;
    if (e && e[0] == 'f') return DPF_PIR_FUSED;
    return DPF_PIR_SPLIT;
}()};

int dpf_set_pir_kernel(int kernel) {
    if (kernel != DPF_PIR_SPLIT && kernel != DPF_PIR_FUSED && kernel != DPF_PIR_FUSED_ANY)
        return fail(DPF_ERR_PARAM, "dpf: unknown PIR kernel");
    if (kernel != DPF_PIR_SPLIT && !dpfk::pir_fused_built())
        return fail(DPF_ERR_PARAM, "dpf: the fused PIR kernel is not in this build (make -C dpf-go_amd experimental)");
    return g_pir_kernel.exchange(kernel);
}
int dpf_get_pir_kernel(void) { return g_pir_kernel.load(); }

int dpf_pir_kernel_for(size_t nkeys, uint32_t logN, uint32_t prefix_bits) {
    const uint32_t stop = stop_of(logN);
    const int k = g_pir_kernel.load(std::memory_order_relaxed);
    return !want_bs() && k != DPF_PIR_SPLIT && prefix_bits <= stop &&
                   dpfk::pir_fused_ok(nkeys, stop, prefix_bits, k == DPF_PIR_FUSED_ANY)
               ? DPF_PIR_FUSED
               : DPF_PIR_SPLIT;
}

size_t dpf_pir_db_sliced_size(uint64_t nrec) { return std::max<size_t>(16, dpfk::pir_sliced_bytes(nrec)); }

int dpf_pir_db_slice_dev(int device, const uint8_t* d_db, uint64_t nrec, uint8_t* d_dbs, void* stream) {
    if (nrec > 0 && (!d_db || !d_dbs)) return fail(DPF_ERR_PARAM, "dpf: null device buffer");
    if (((uintptr_t)d_db | (uintptr_t)d_dbs) % 16 != 0) return fail(DPF_ERR_PARAM, "dpf: misaligned device buffer");
    DeviceGuard g(device);
    HIP_TRY(dpfk::launch_slice_db(d_db, nrec, d_dbs, (hipStream_t)stream));
    return DPF_OK;
}

int dpf_pir_answer_sliced_dev(int device, const uint8_t* d_keys, size_t klen, size_t nkeys, uint32_t logN,
                              uint32_t prefix_bits, uint64_t prefix, const uint8_t* d_dbs, uint64_t nrec,
                              uint8_t* d_ans, void* d_work, void* stream) {
    if (int rc = check_key(klen, logN)) return rc;
    const uint32_t stop = stop_of(logN);
    if (prefix_bits > stop || (prefix >> prefix_bits) != 0) return fail(DPF_ERR_PARAM, "dpf: subtree prefix out of range");
    const uint64_t slice = logN - prefix_bits >= 64 ? ~0ull : (1ull << (logN - prefix_bits));
    if (nrec > slice) return fail(DPF_ERR_PARAM, "dpf: more DB records than the subtree's domain");
    if (int rc = check_pir_bufs(d_keys, nkeys, d_dbs, nrec, d_ans, d_work)) return rc;
    DeviceGuard g(device);
    CuScope cus(stream);
    hipStream_t st = (hipStream_t)stream;
    if (nkeys == 0) return DPF_OK;
    if (nrec == 0) {
        HIP_TRY(hipMemsetAsync(d_ans, 0, nkeys * 32, st));
        return DPF_OK;
    }
    // The same workspace and tree pass as dpf_pir_answer_dev; the fold reads the sliced DB.
    uint8_t* bits = (uint8_t*)d_work + align256(tree_ws_bytes(nkeys, stop, prefix_bits, nkeys));
    const uint64_t per_key = (uint64_t)16 << (stop - prefix_bits);
    const bool bs = want_bs();
    const int fz = g_pir_kernel.load(std::memory_order_relaxed);
    if (!bs && fz != DPF_PIR_SPLIT && dpfk::pir_fused_ok(nkeys, stop, prefix_bits, fz == DPF_PIR_FUSED_ANY)) {
        // One launch: tree + matrix-core fold (k_pir_fused) from the expanded records.
        const TreeWs w = tree_ws(d_work, nkeys, stop);
        forget_expanded(d_work);
        HIP_TRY(dpfk::launch_unpack(d_keys, klen, nkeys, stop, w.ek, st));
        note_expanded(d_work, nkeys, stop, false);
        uint32_t* parts = (uint32_t*)(bits + align256(nkeys * per_key));
        HIP_TRY(dpfk::launch_pir_fused(w.ek, (uint32_t)nkeys, stop, prefix_bits, prefix, d_dbs, nrec, (uint32_t*)d_ans,
                                       parts, st));
        return DPF_OK;
    }
    bool expanded = false;
    forget_expanded(d_work);
    HIP_TRY(tree_from_keys(d_keys, klen, nkeys, stop, prefix_bits, prefix, bits, per_key, d_work, st, bs, &expanded));
    if (expanded) note_expanded(d_work, nkeys, stop, bs);
    uint32_t* parts = (uint32_t*)(bits + align256(nkeys * per_key));
    HIP_TRY(dpfk::launch_pir_fold_sliced((const uint32_t*)bits, per_key / 4, d_dbs, nrec, (uint32_t)nkeys,
                                         (uint32_t*)d_ans, parts, st));
    return DPF_OK;
}

int dpf_xor_fold_sliced_dev(int device, const uint8_t* d_bits, size_t bits_stride, size_t nkeys, const uint8_t* d_dbs,
                            uint64_t nrec, uint8_t* d_ans, void* d_work, void* stream) {
    if (bits_stride % 16 != 0) return fail(DPF_ERR_PARAM, "dpf: bits_stride must be a multiple of 16");
    if (nrec > (uint64_t)bits_stride * 8) return fail(DPF_ERR_PARAM, "dpf: more records than selection bits per key");
    if (((uintptr_t)d_bits | (uintptr_t)d_dbs) % 16 != 0 || (uintptr_t)d_ans % 4 != 0)
        return fail(DPF_ERR_PARAM, "dpf: misaligned device buffer");
    if (nkeys > 0 && (!d_ans || !d_work || (nrec > 0 && (!d_bits || !d_dbs))))
        return fail(DPF_ERR_PARAM, "dpf: null device buffer");
    DeviceGuard g(device);
    CuScope cus(stream);
    if (nkeys == 0) return DPF_OK;
    HIP_TRY(dpfk::launch_pir_fold_sliced((const uint32_t*)d_bits, bits_stride / 4, d_dbs, nrec, (uint32_t)nkeys,
                                         (uint32_t*)d_ans, (uint32_t*)d_work, (hipStream_t)stream));
    return DPF_OK;
}

size_t dpf_xor_fold_workspace_size(void) { return dpfk::pir_fold_parts_bytes(); }

int dpf_set_fold_limits(uint32_t max_blocks, uint32_t max_sg_per_block) {
    dpfk::set_fold_limits(max_blocks, max_sg_per_block);
    return DPF_OK;
}

int dpf_xor_fold_dev(int device, const uint8_t* d_bits, size_t bits_stride, size_t nkeys, const uint8_t* d_payload,
                     uint64_t nrec, size_t rec_bytes, uint8_t* d_ans, void* d_work, void* stream) {
    if (rec_bytes == 0 || rec_bytes % 32 != 0) return fail(DPF_ERR_PARAM, "dpf: rec_bytes must be a positive multiple of 32");
    if (bits_stride % 16 != 0) return fail(DPF_ERR_PARAM, "dpf: bits_stride must be a multiple of 16");
    if (nrec > (uint64_t)bits_stride * 8) return fail(DPF_ERR_PARAM, "dpf: more records than selection bits per key");
    if (((uintptr_t)d_bits | (uintptr_t)d_payload) % 16 != 0 || (uintptr_t)d_ans % 4 != 0)
        return fail(DPF_ERR_PARAM, "dpf: misaligned device buffer");
    if (nkeys > 0 && (!d_ans || !d_work || (nrec > 0 && (!d_bits || !d_payload))))
        return fail(DPF_ERR_PARAM, "dpf: null device buffer");
    DeviceGuard g(device);
    CuScope cus(stream);
    hipStream_t st = (hipStream_t)stream;
    if (nkeys == 0) return DPF_OK;
    HIP_TRY(dpfk::launch_pir_fold((const uint32_t*)d_bits, bits_stride / 4, d_payload, nrec, rec_bytes, (uint32_t)nkeys,
                                  (uint32_t*)d_ans, (uint32_t*)d_work, st));
    return DPF_OK;
}

// A PIR handle owns references to the devices its shards live on, so it
// stays usable (and freeable) after dpf_gpu_shutdown.
struct PirDb {
    uint32_t logN = 0, pbits = 0;
    uint64_t nrec = 0;
    bool sliced = true;            // shards in the bit-sliced layout (the matrix-core fold)
    DevList devs;                  // per shard: its device
    std::vector<void*> shard;      // per device: its DB slice
    std::vector<uint64_t> shard_n; // records in that slice
    ~PirDb() {
        for (size_t i = 0; i < shard.size(); ++i) {
            DeviceGuard gd(devs[i]->id);
            (void)hipFree(shard[i]);
        }
    }
};

int dpf_pir_db_create(const uint8_t* db, uint64_t nrec, uint32_t logN, int ngpus, void** handle) {
    if (!handle) return fail(DPF_ERR_PARAM, "dpf: null handle");
    *handle = nullptr;
    if (logN > 63 || (logN < 64 && nrec > (1ull << logN))) return fail(DPF_ERR_PARAM, "dpf: DB larger than 2^logN");
    int have = 0;
    const DevList devs = pick_devs(0, &have);
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
    // DPF_PIR_FOLD=lds keeps the row-major shards and the LDS fold (A/B runs).
    static const bool lds = [] {
        const char* e = getenv("DPF_PIR_FOLD");
        return e && e[0] == 'l';
    }();
    h->sliced = !lds;
    const uint64_t slice = 1ull << (logN - pb);
    for (int g = 0; g < want; ++g) {
        const uint64_t lo = std::min<uint64_t>(nrec, (uint64_t)g * slice);
        const uint64_t hi = std::min<uint64_t>(nrec, lo + slice);
        DeviceGuard gd(devs[(size_t)g]->id);
        void* p = nullptr;
        const size_t bytes = h->sliced ? dpf_pir_db_sliced_size(hi - lo) : std::max<uint64_t>(hi - lo, 1) * 32;
        if (hipMalloc(&p, bytes) != hipSuccess) return fail(DPF_ERR_NOMEM, "dpf: DB shard allocation failed");
        h->devs.push_back(devs[(size_t)g]);     // ~PirDb frees what was allocated so far
        h->shard.push_back(p);
        h->shard_n.push_back(hi - lo);
        if (hi <= lo) continue;
        if (!h->sliced) {
            if (hipMemcpy(p, db + lo * 32, (hi - lo) * 32, hipMemcpyHostToDevice) != hipSuccess)
                return fail(DPF_ERR_HIP, "dpf: DB upload failed");
            continue;
        }
        // Row-major records up through a staging buffer, sliced once on the device.
        void* tmp = nullptr;
        if (hipMalloc(&tmp, (hi - lo) * 32) != hipSuccess) return fail(DPF_ERR_NOMEM, "dpf: DB staging allocation failed");
        const bool ok = hipMemcpy(tmp, db + lo * 32, (hi - lo) * 32, hipMemcpyHostToDevice) == hipSuccess &&
                        dpfk::launch_slice_db((const uint8_t*)tmp, hi - lo, (uint8_t*)p, nullptr) == hipSuccess &&
                        hipDeviceSynchronize() == hipSuccess;
        (void)hipFree(tmp);
        if (!ok) return fail(DPF_ERR_HIP, "dpf: DB upload failed");
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
        Dev& d = *h->devs[(size_t)dev];
        std::lock_guard<std::mutex> lk(d.mu);
        DeviceGuard gd(d.id);
        HIP_TRY(hipError_t(d.keys.ensure(std::max<size_t>(1, nkeys * klen))));
        HIP_TRY(hipError_t(d.work.ensure(dpf_pir_workspace_size(nkeys, h->logN, h->pbits))));
        HIP_TRY(hipError_t(d.out.ensure(std::max<size_t>(32, nkeys * 32))));
        HIP_TRY(hipMemcpyAsync(d.keys.p, keys, nkeys * klen, hipMemcpyHostToDevice, d.st));
        int r = (h->sliced ? dpf_pir_answer_sliced_dev : dpf_pir_answer_dev)(
            d.id, (const uint8_t*)d.keys.p, klen, nkeys, h->logN, h->pbits, lo, (const uint8_t*)h->shard[lo],
            h->shard_n[lo], (uint8_t*)d.out.p, d.work.p, d.st);
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

void dpf_pir_db_free(void* handle) { delete (PirDb*)handle; }

int dpf_stream_create_cu_masked(int device, uint32_t cu_first, uint32_t cu_count, void** stream) {
    if (!stream) return fail(DPF_ERR_PARAM, "dpf: null stream out-pointer");
    *stream = nullptr;
    DeviceGuard g(device);
    int ncu = 0;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
    if (cu_count == 0 || (uint64_t)cu_first + cu_count > (uint64_t)ncu)
        return fail(DPF_ERR_PARAM, "dpf: CU range outside the device");
    std::vector<uint32_t> mask(((size_t)ncu + 31) / 32, 0u);
    for (uint32_t b = cu_first; b < cu_first + cu_count; ++b) mask[b / 32] |= 1u << (b % 32);
    hipStream_t st = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
    {
        std::lock_guard<std::mutex> lk(g_cus_mu);
        g_stream_cus[st] = (int)cu_count;
    }
    *stream = st;
    return DPF_OK;
}

int dpf_stream_destroy(void* stream) {
    if (!stream) return DPF_OK;
    {
        std::lock_guard<std::mutex> lk(g_cus_mu);
        g_stream_cus.erase((hipStream_t)stream);
    }
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return DPF_OK;
}

}  // extern "C"
