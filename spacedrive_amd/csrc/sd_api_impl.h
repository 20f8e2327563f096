// sd_api_impl.h -- the host-side types shared by the C ABI's translation units
// (sd_cas_api.cpp: context, batches, dedup; sd_files.cpp: the file readers' pipelines and
// streaming): device / pinned buffers, stream slots, the opaque ABI structs.
#pragma once
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "sd_host.h"
#include "sd_internal.h"
#include "stage_pool.h"

#define HIP_CHECK(expr)                                                                              \
    do {                                                                                             \
        hip_thread_check(#expr); /* never on a private-fd-table thread (sd_host.h) */                \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            throw sd_failure(e_ == hipErrorOutOfMemory ? SD_ERR_NOMEM : SD_ERR_DEVICE,              \
                             std::string(#expr) + ": " + hipGetErrorString(e_));                    \
    } while (0)

namespace sdi {

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
inline void to_hex(const uint8_t* h, int nbytes, char* out) { hex_lower(h, nbytes, out); }

// RAII device buffer
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void alloc(size_t n) {
        reset();
        if (n == 0) n = 16;
        HIP_CHECK(hipMalloc(&p, n));
        bytes = n;
    }
    // grow-only (never frees a buffer that is large enough: hipFree synchronises the device)
    void ensure(size_t n) {
        if (n > bytes) alloc(n);
    }
    // grow keeping the contents (the caller has synchronised every stream writing it)
    void grow_preserve(size_t n) {
        if (n <= bytes) return;
        void* q = nullptr;
        HIP_CHECK(hipMalloc(&q, n));
        if (p) {
            const hipError_t e = hipMemcpy(q, p, bytes, hipMemcpyDeviceToDevice);
            if (e != hipSuccess) {
                (void)hipFree(q);
                HIP_CHECK(e);
            }
            (void)hipFree(p);
        }
        p = q;
        bytes = n;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
    template <class T>
    void upload(const std::vector<T>& v, hipStream_t s = nullptr) {
        ensure(v.size() * sizeof(T));
        if (v.empty()) return;
        if (s) HIP_CHECK(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
        else HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    }
};

struct PinnedBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~PinnedBuf() { reset(); }
    void reset() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t n) {
        if (n <= bytes) return;
        reset();
        HIP_CHECK(hipHostMalloc(&p, n, hipHostMallocDefault));
        bytes = n;
    }
    uint8_t* u8() const { return reinterpret_cast<uint8_t*>(p); }
};

// A plan's host tables packed into one pinned buffer and copied to one device buffer with
// a single H2D: one DMA the host does not wait on, instead of an allocation and a staged
// pageable copy per table (those cost ~12 us each, most of a small batch's host time).
// add() queues a table at a 16-byte aligned offset; upload() packs and copies.  The pinned
// buffer is read by the async copy: the caller syncs the stream before the next upload
// (every plan is rebuilt only after its previous run has drained).
struct Tables {
    PinnedBuf host;
    DevBuf dev;
    std::vector<std::pair<const void*, size_t>> parts;
    std::vector<size_t> offs;
    size_t bytes = 0;
    void begin() {
        parts.clear();
        offs.clear();
        bytes = 0;
    }
    template <class T>
    size_t add(const std::vector<T>& v) {
        const size_t o = bytes;
        parts.emplace_back(v.data(), v.size() * sizeof(T));
        offs.push_back(o);
        bytes = align_up(o + v.size() * sizeof(T), 16);
        return o;
    }
    void upload(hipStream_t s) {
        if (bytes == 0) return;
        host.ensure(bytes);
        dev.ensure(bytes);
        for (size_t k = 0; k < parts.size(); k++)
            if (parts[k].second) memcpy(host.u8() + offs[k], parts[k].first, parts[k].second);
        if (s) HIP_CHECK(hipMemcpyAsync(dev.p, host.p, bytes, hipMemcpyHostToDevice, s));
        else HIP_CHECK(hipMemcpy(dev.p, host.p, bytes, hipMemcpyHostToDevice));
    }
    template <class T>
    T* at(size_t off) const { return reinterpret_cast<T*>(reinterpret_cast<uint8_t*>(dev.p) + off); }
};

}  // namespace sdi

struct sd_checksum_batch {
    size_t n = 0;
    CkPlan plan;
    sdi::Tables tab;  // files, wg_map, then one table per reduce pass
    size_t o_files = 0, o_map = 0;
    std::vector<size_t> o_pass;
    sdi::DevBuf lvl[2];
    const ck_file* d_files() const { return tab.at<ck_file>(o_files); }
    const uint2* d_map() const { return tab.at<uint2>(o_map); }
    const ck_reduce_wg* d_pass(size_t k) const { return tab.at<ck_reduce_wg>(o_pass[k]); }
};

// one file over the ranks of a communicator (include/sd_cas.h, sd_split_range)
struct sd_split_checksum {
    SplitPlan sp;
    sd_checksum_batch plan;  // the whole file as one message: leaf table + reduce passes
};

struct sd_cas_batch {
    size_t n = 0;
    uint32_t n_sampled = 0, n_whole = 0, n_long = 0;
    uint64_t compressions = 0, msg_bytes = 0, staged_bytes = 0, whole_chunks = 0;
    WholePlan whole;  // work lists (kernel formats in cas_kernels.hip, k_whole_items / _merge8)
    sdi::Tables tab;  // the sampled files' rows and offsets, the work lists, the long-message rows
    size_t o_sidx = 0, o_soff = 0, o_full = 0, o_tail = 0, o_ma = 0, o_mb = 0, o_lidx = 0, o_wrows = 0;
    bool whole_wave = false;  // n_whole <= "whole_wave_max" at plan time: one workgroup per file
    sdi::DevBuf cvbuf, cv2;
    bool sampled_wave = false;  // n_sampled <= "sampled_wave_max" at plan time: one wave per file
    sdi::DevBuf srows;          // otherwise the sampled files' node CVs between the two kernels
    // whole-file messages longer than SD_WHOLE_ITEMS_MAX: a checksum sub-batch over their
    // byte ranges, its hashes scattered to out[long_idx[i]]
    sd_checksum_batch lng;
    sdi::DevBuf long_out;
    // host tables (packed into tab by the plan)
    std::vector<uint32_t> h_sidx, h_long_idx;
    std::vector<sd_u32x4> h_wrows;  // whole_wave: (u64 message offset, length, output row)
    std::vector<uint64_t> h_soff;
    const uint32_t* d_sidx() const { return tab.at<uint32_t>(o_sidx); }
    const uint64_t* d_soff() const { return tab.at<uint64_t>(o_soff); }
    const uint4* d_full() const { return tab.at<uint4>(o_full); }
    const uint4* d_tail() const { return tab.at<uint4>(o_tail); }
    const uint4* d_ma() const { return tab.at<uint4>(o_ma); }
    const uint4* d_mb() const { return tab.at<uint4>(o_mb); }
    const uint32_t* d_lidx() const { return tab.at<uint32_t>(o_lidx); }
    const uint4* d_wrows() const { return tab.at<uint4>(o_wrows); }
};

namespace sdi {

// per-call working set of the host drop-in entry points; its batches persist with the slot
// in the context's pool, so a call reuses their device and pinned tables
struct Slot {
    hipStream_t stream = nullptr;
    DevBuf staged, hashes;
    PinnedBuf host_hashes, window;
    Tables aux;  // a call's own tables (the split checksum's block map), grown with the slot
    sd_cas_batch cas;
    sd_checksum_batch ck;
    hipEvent_t drained = nullptr;  // sync()'s blocking-sync event
    Slot() = default;
    Slot(const Slot&) = delete;
    Slot& operator=(const Slot&) = delete;
    ~Slot() {
        if (drained) (void)hipEventDestroy(drained);
    }
    // Waits for the stream's queued work with the thread asleep (a blocking-sync event), as
    // the file stager's waits do: the reader and co-hash threads beside it share the host
    // budget.  (A/B against hipStreamSynchronize, profiles/r4/r4l_sync_ab/: no difference
    // beyond the box's noise -- the runtime's own wait already sleeps after a short poll.)
    void sync() {
        if (!drained) HIP_CHECK(hipEventCreateWithFlags(&drained, hipEventDisableTiming | hipEventBlockingSync));
        HIP_CHECK(hipEventRecord(drained, stream));
        HIP_CHECK(hipEventSynchronize(drained));
    }
};

}  // namespace sdi

struct sd_cas_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::mutex coal_mu;
    sd_coalescer* coal = nullptr;  // latency path, created on the first single-file call
    std::atomic<uint64_t> files_calls_cpu{0}, files_calls_gpu{0};  // sd_cas_ids_files routes
    std::atomic<uint64_t> checksum_calls_cpu{0}, checksum_calls_gpu{0},  // sd_file_checksums routes
        checksum_calls_hybrid{0};
    // bytes (stat lengths) of the files sd_file_checksums gave the GPU route, and the CPU path
    // in split calls
    std::atomic<uint64_t> checksum_bytes_gpu{0}, checksum_bytes_cpu_split{0};
    std::atomic<uint64_t> cas_ids_gpu_files{0}, cas_ids_host_files{0};  // sd_cas_ids: who hashed
    std::atomic<uint64_t> checksums_gpu_bytes{0}, checksums_host_bytes{0};  // sd_checksums: who hashed
    std::mutex split_mu;
    SplitRoutes split_routes;  // sd_file_checksums: the split or the CPU path, learned (sd_host.h)
    uint64_t split_routes_gen = 0;  // split_route_tuning_gen() the rates were learned under
    // sd_checksums' co-hashed calls: the GPU + host threads, or the CPU path alone, learned
    // the same way (route 0 = co-hash, 1 = CPU path; under split_mu)
    SplitRoutes cohash_routes;
    uint64_t cohash_routes_gen = 0;
    std::mutex pool_mu;
    // Reader threads.  stage_pool: tasks that open and close their own files (the cas
    // stager, checksum packs), on private fd tables (stage_pool.h); io_pool: parallel preads
    // of a descriptor the caller opened (a streamed checksum), on the shared table.  One of
    // each per context, grown to the largest thread count any call asked for; a caller holds
    // its shared_ptr while it runs, so a concurrent call that grows a pool never destroys
    // one in use.
    std::shared_ptr<StagePool> pool, iopool;
    std::shared_ptr<StagePool> stage_pool(int nthreads) {
        std::lock_guard<std::mutex> g(pool_mu);
        if (!pool || pool->threads() < nthreads) pool = std::make_shared<StagePool>(nthreads, true);
        return pool;
    }
    std::shared_ptr<StagePool> io_pool(int nthreads) {
        std::lock_guard<std::mutex> g(pool_mu);
        if (!iopool || iopool->threads() < nthreads) iopool = std::make_shared<StagePool>(nthreads, false);
        return iopool;
    }
    sd_coalescer* coalescer() {
        std::lock_guard<std::mutex> g(coal_mu);
        if (!coal) coal = coalescer_create(this);
        return coal;
    }
    std::vector<std::unique_ptr<sdi::Slot>> free_slots;

    std::unique_ptr<sdi::Slot> acquire() {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_slots.empty()) {
                auto s = std::move(free_slots.back());
                free_slots.pop_back();
                return s;
            }
        }
        auto s = std::make_unique<sdi::Slot>();
        HIP_CHECK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        return s;
    }
    void release(std::unique_ptr<sdi::Slot> s) {
        std::lock_guard<std::mutex> g(mu);
        free_slots.push_back(std::move(s));
    }
    void bind() { HIP_CHECK(hipSetDevice(device)); }
    static hipStream_t pick(void* s) { return reinterpret_cast<hipStream_t>(s); }  // NULL = null stream
};

namespace sdi {

// Two slots held for one call; released (after their streams drain) on scope exit.
struct SlotPair {
    sd_cas_ctx* c;
    std::unique_ptr<Slot> s[2];
    std::unique_ptr<Slot> cp;  // a third queue, for H2D copies issued back to back (copy_stream)
    explicit SlotPair(sd_cas_ctx* ctx) : c(ctx) {
        s[0] = c->acquire();
        s[1] = c->acquire();
    }
    ~SlotPair() {
        for (auto* x : {&s[0], &s[1], &cp})
            if (*x) {
                (void)hipStreamSynchronize((*x)->stream);
                c->release(std::move(*x));
            }
    }
    // One stream for all of a call's host-to-device copies: they run one after the other on
    // one DMA queue (two copies in flight on two streams measured 46 instead of 56 GB/s on
    // some boxes), while the kernels of the two slots overlap them.
    hipStream_t copy_stream() {
        if (!cp) cp = c->acquire();
        return cp->stream;
    }
    Slot& operator[](int k) { return *s[k]; }
    void sync_all() {
        s[0]->sync();
        s[1]->sync();
    }
};

}  // namespace sdi

namespace sdi {
// checksum batches (device): (re)plan reusing the batch's buffers; the reduce passes; leaf + reduce
void plan_checksum_batch(sd_checksum_batch* b, const uint64_t* offsets, const uint64_t* lens, size_t n,
                         hipStream_t stream);
void run_checksum_reduce(const sd_checksum_batch* b, uint32_t* out, hipStream_t s);
void run_checksum_batch(const sd_checksum_batch* b, const uint8_t* d_data, uint8_t* d_hash32, hipStream_t s);
// cas batches (device)
void plan_cas_batch(sd_cas_batch* b, const sd_extent* ext, size_t n, hipStream_t stream);
void run_cas_batch(const sd_cas_batch* b, const uint8_t* d_staged, uint8_t* d_hash32, hipStream_t s,
                   int parts = SD_PART_SAMPLED | SD_PART_WHOLE);
}  // namespace sdi
