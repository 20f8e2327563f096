// sd_cas_api.cpp -- host side of the C ABI declared in include/sd_cas.h.
//
// Replaces, behind `extern "C"`, the per-file calls
//   generate_cas_id   /root/reference/core/src/object/cas.rs:23-62
//   file_checksum     /root/reference/core/src/object/validation/hash.rs:10-24
// with batched calls that stage messages on the host and hash them with the gfx950
// kernels of cas_kernels.hip.  Thread-safety: a context owns a mutex-protected pool of
// streams; prepared batches own their scratch (one run of a batch at a time).  Every
// entry point catches all C++ exceptions (the reference FFI fences panics with
// catch_unwind, apps/mobile/modules/sd-core/ios/crate/src/lib.rs:41,60).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "sd_internal.h"
#include "stage_pool.h"

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

struct sd_failure : std::runtime_error {
    int rc;
    sd_failure(int r, const std::string& m) : std::runtime_error(m), rc(r) {}
};

#define HIP_CHECK(expr)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            throw sd_failure(e_ == hipErrorOutOfMemory ? SD_ERR_NOMEM : SD_ERR_DEVICE,              \
                             std::string(#expr) + ": " + hipGetErrorString(e_));                    \
    } while (0)

#define SD_GUARD_BEGIN try {
#define SD_GUARD_END                                   \
    }                                                  \
    catch (const sd_failure& f) {                      \
        set_err("%s", f.what());                       \
        return f.rc;                                   \
    }                                                  \
    catch (const std::bad_alloc&) {                    \
        set_err("host allocation failed");             \
        return SD_ERR_NOMEM;                           \
    }                                                  \
    catch (const std::exception& ex) {                 \
        set_err("internal error: %s", ex.what());      \
        return SD_ERR_INTERNAL;                        \
    }                                                  \
    catch (...) {                                      \
        set_err("internal error");                     \
        return SD_ERR_INTERNAL;                        \
    }

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

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
    void ensure(size_t n) {
        if (n > bytes) alloc(n);
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
    // grow-only (never frees a buffer that is large enough: hipFree synchronises the device)
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
};

// per-call working set of the host drop-in entry points
struct Slot {
    hipStream_t stream = nullptr;
    DevBuf staged, hashes;
    PinnedBuf host_hashes, window;
};

}  // namespace

struct sd_cas_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::mutex coal_mu;
    sd_coalescer* coal = nullptr;  // latency path, created on the first single-file call
    std::mutex pool_mu;
    std::unique_ptr<StagePool> pool;  // file stager threads (sd_cas_ids_files)
    StagePool& stage_pool(int nthreads) {
        std::lock_guard<std::mutex> g(pool_mu);
        if (!pool || pool->threads() != nthreads) pool = std::make_unique<StagePool>(nthreads);
        return *pool;
    }
    sd_coalescer* coalescer() {
        std::lock_guard<std::mutex> g(coal_mu);
        if (!coal) coal = coalescer_create(this);
        return coal;
    }
    std::vector<std::unique_ptr<Slot>> free_slots;

    std::unique_ptr<Slot> acquire() {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_slots.empty()) {
                auto s = std::move(free_slots.back());
                free_slots.pop_back();
                return s;
            }
        }
        auto s = std::make_unique<Slot>();
        HIP_CHECK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        return s;
    }
    void release(std::unique_ptr<Slot> s) {
        std::lock_guard<std::mutex> g(mu);
        free_slots.push_back(std::move(s));
    }
    void bind() { HIP_CHECK(hipSetDevice(device)); }
    static hipStream_t pick(void* s) { return reinterpret_cast<hipStream_t>(s); }  // NULL = null stream
};

struct sd_cas_batch {
    size_t n = 0;
    uint32_t n_sampled = 0, n_whole = 0, n_multi = 0;
    uint32_t total_chunks = 0;
    uint64_t compressions = 0, msg_bytes = 0, staged_bytes = 0;
    uint32_t n_groups = 0;  // whole-file groups of the fused kernel
    uint32_t total_pairs = 0, n_multi2 = 0;  // pair leaf: chunk pairs; files with >= 3 chunks
    uint32_t n_groups2 = 0;                  // forest groups over the multi-pair files
    // variant 6 item lists (kernel formats in cas_kernels.hip, k_whole_full / _tail / _merge8)
    uint32_t n_full = 0, n_tail = 0, n_merge_a = 0, n_merge_b = 0, n_cv2 = 0;
    DevBuf ext, sidx, order, prefix, hint, cvbuf, groups, prefix2, hint2, groups2;
    DevBuf full_items, tail_items, merge_a, merge_b, cv2;
    std::vector<uint4> h_full, h_tail, h_merge_a, h_merge_b;
    // variant 2: the whole-file tree kernel runs on a side stream beside the sampled kernel
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    ~sd_cas_batch() {
        if (side) (void)hipStreamDestroy(side);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
    }
    std::vector<sd_extent> h_ext;  // host copies backing async uploads
    std::vector<uint32_t> h_sidx, h_order, h_prefix, h_hint, h_prefix2, h_hint2;
    std::vector<uint2> h_groups, h_groups2;
};

struct ck_pass {
    DevBuf wgs;
    std::vector<ck_reduce_wg> h_wgs;  // host copy backing the async upload
    uint32_t n_wg = 0;
    int src = 0, dst = 1;  // which CV level buffer
};

struct sd_checksum_batch {
    size_t n = 0;
    uint64_t total_bytes = 0, compressions = 0, blocks = 0;
    std::vector<ck_file> files_h;
    std::vector<uint2> wg_map_h;
    DevBuf files, wg_map;
    DevBuf lvl[2];
    std::vector<std::unique_ptr<ck_pass>> passes;  // capacity reused across replans
    size_t n_passes = 0;
};

namespace {

// ----------------------------------------------------------------- cas batch planning
uint32_t msg_chunks(uint32_t msg_len) { return msg_len == 0 ? 1u : (msg_len + 1023u) / 1024u; }

uint64_t msg_compressions(uint64_t msg_len) {  // blocks in all chunks + parents
    const uint64_t C = msg_len == 0 ? 1 : (msg_len + 1023) / 1024;
    uint64_t blocks = 0;
    for (uint64_t c = 0; c < C; c++) {
        const uint64_t len = std::min<uint64_t>(1024, msg_len - c * 1024);
        blocks += len == 0 ? 1 : (len + 63) / 64;
    }
    return blocks + (C - 1);
}

uint64_t file_compressions(uint64_t len) {  // same, closed form for large inputs
    const uint64_t C = len == 0 ? 1 : (len + 1023) / 1024;
    const uint64_t last = len - (C - 1) * 1024;
    return (C - 1) * 16 + (last == 0 ? 1 : (last + 63) / 64) + (C - 1);
}

void validate_extent(const sd_extent& e, size_t i) {
    const bool whole = e.size <= SD_MINIMUM_FILE_SIZE;
    const uint64_t want = whole ? 8 + e.size : SD_SAMPLED_MSG_LEN;
    if (e.kind != (whole ? SD_KIND_WHOLE : SD_KIND_SAMPLED) || e.msg_len != want)
        throw sd_failure(SD_ERR_INVALID, "extent " + std::to_string(i) + ": kind/msg_len do not match size");
    if (e.msg_offset % 16)
        throw sd_failure(SD_ERR_INVALID, "extent " + std::to_string(i) + ": msg_offset not 16-byte aligned");
}

// compressions of aligned chunk pair (c0, c0 + 1) holding glen (1..2048) message bytes
uint32_t pair_compressions(uint32_t glen) {
    const uint32_t l0 = std::min<uint32_t>(glen, 1024), l1 = glen - l0;
    return (l0 + 63) / 64 + (l1 ? (l1 + 63) / 64 + 1 : 0);
}

// Variant-6 work lists over the length-sorted whole files (b->h_order, pair prefix
// b->h_prefix2): full-pair items in (file, pair) order; tail items counting-sorted by
// compressions, descending; merge8 items -- pass A over aligned groups of <= 8 pair nodes
// (the whole tree when a file has <= 8 nodes), pass B over the pass-A nodes of files with
// more than 8.
void plan_whole_items(sd_cas_batch* b, const sd_extent* ext) {
    auto& full = b->h_full;
    auto& tail = b->h_tail;
    auto& ma = b->h_merge_a;
    auto& mb = b->h_merge_b;
    full.clear();
    tail.clear();
    ma.clear();
    mb.clear();
    std::vector<uint32_t> tail_cost;
    const auto& p2 = b->h_prefix2;
    // items are emitted in file (= staged address) order, so the full-pair waves sweep the
    // staged buffer front to back as the sampled kernel does, instead of hopping between
    // the length-sorted files' scattered messages; the cv slot still follows the sorted order
    std::vector<uint32_t> rank(b->n, 0);
    for (uint32_t k = 0; k < b->n_whole; k++) rank[b->h_order[k]] = k;
    for (uint32_t file = 0; file < b->n; file++) {
        const sd_extent& e = ext[file];
        if (e.kind != SD_KIND_WHOLE) continue;
        const uint32_t k = rank[file];
        const uint32_t C = msg_chunks(e.msg_len), P = (C + 1) / 2;
        const bool multi = C >= 3;
        for (uint32_t j = 0; j < P; j++) {
            const uint64_t off = e.msg_offset + 2048ull * j;
            const uint32_t glen = std::min<uint32_t>(2048, e.msg_len - 2048 * j);
            const uint32_t lo = (uint32_t)off, hi = (uint32_t)(off >> 32);
            if (multi && glen == 2048) {
                full.push_back(make_uint4(lo, hi, p2[k] + j, 2 * j));
            } else {
                const uint32_t w = glen | ((2 * j) << 12) | (multi ? 0u : 0x80000000u);
                tail.push_back(make_uint4(lo, hi, multi ? p2[k] + j : file, w));
                tail_cost.push_back(pair_compressions(glen));
            }
        }
    }
    // stable counting sort of the tail items by cost, descending (cost 1..33)
    {
        std::vector<uint32_t> start(35, 0);
        for (uint32_t c : tail_cost) start[34 - c]++;
        uint32_t acc = 0;
        for (auto& s : start) {
            const uint32_t t = s;
            s = acc;
            acc += t;
        }
        std::vector<uint4> sorted(tail.size());
        for (size_t i = 0; i < tail.size(); i++) sorted[start[34 - tail_cost[i]]++] = tail[i];
        tail.swap(sorted);
    }
    uint32_t cv2 = 0;
    for (uint32_t k = 0; k < b->n_multi2; k++) {
        const uint32_t P = p2[k + 1] - p2[k], file = b->h_order[k];
        if (P <= 8) {
            ma.push_back(make_uint4(p2[k], P | 0x80000000u, file, 0));
            continue;
        }
        const uint32_t G = (P + 7) / 8;
        for (uint32_t a = 0; a < G; a++) ma.push_back(make_uint4(p2[k] + 8 * a, std::min<uint32_t>(8, P - 8 * a), cv2 + a, 0));
        if (G > 8) throw sd_failure(SD_ERR_INTERNAL, "whole-file message with more than 64 pair nodes");
        mb.push_back(make_uint4(cv2, G | 0x80000000u, file, 0));
        cv2 += G;
    }
    b->n_full = (uint32_t)full.size();
    b->n_tail = (uint32_t)tail.size();
    b->n_merge_a = (uint32_t)ma.size();
    b->n_merge_b = (uint32_t)mb.size();
    b->n_cv2 = cv2;
}

// (Re)plans `b` for these extents, reusing its device buffers.  With a stream, the small
// metadata uploads are async on it and read from b's host copies, which stay valid until
// the next rebuild of `b` (the caller syncs the stream before that).
void plan_cas_batch(sd_cas_batch* b, const sd_extent* ext, size_t n, hipStream_t stream) {
    if (n >= (1ull << 31)) throw sd_failure(SD_ERR_INVALID, "batch too large");
    b->n = n;
    b->n_sampled = b->n_whole = b->n_multi = 0;
    b->compressions = b->msg_bytes = 0;
    std::vector<uint32_t>& sidx = b->h_sidx;
    sidx.clear();
    std::vector<uint32_t> count(SD_MINIMUM_FILE_SIZE + 9 + 1, 0);
    uint64_t end = 0;
    for (size_t i = 0; i < n; i++) {
        validate_extent(ext[i], i);
        end = std::max<uint64_t>(end, align_up(ext[i].msg_offset + ext[i].msg_len, SD_STAGE_PAD));
        b->msg_bytes += ext[i].msg_len;
        if (ext[i].kind == SD_KIND_SAMPLED) {
            sidx.push_back((uint32_t)i);
            b->compressions += 953;  // 56 x 16 + 1 blocks, 56 parents
        } else {
            count[ext[i].msg_len]++;
            b->compressions += msg_compressions(ext[i].msg_len);
        }
    }
    b->staged_bytes = end;
    b->n_sampled = (uint32_t)sidx.size();
    b->n_whole = (uint32_t)(n - sidx.size());
    // counting sort of whole files by msg_len, descending (uniform lanes in both kernels)
    std::vector<uint32_t> start(count.size() + 1, 0);
    for (size_t L = count.size(); L-- > 0;) start[L] = start[L + 1] + count[L];
    std::vector<uint32_t>& order = b->h_order;
    order.assign(b->n_whole, 0);
    for (size_t i = 0; i < n; i++)
        if (ext[i].kind == SD_KIND_WHOLE) order[start[ext[i].msg_len + 1]++] = (uint32_t)i;
    std::vector<uint32_t>& prefix = b->h_prefix;
    prefix.assign(b->n_whole + 1, 0);
    uint64_t total = 0;
    for (uint32_t k = 0; k < b->n_whole; k++) {
        prefix[k] = (uint32_t)total;
        const uint32_t C = msg_chunks(ext[order[k]].msg_len);
        total += C;
        if (C >= 2) b->n_multi = k + 1;
    }
    if (total >= (1ull << 32)) throw sd_failure(SD_ERR_INVALID, "too many chunks in one batch");
    prefix[b->n_whole] = (uint32_t)total;
    b->total_chunks = (uint32_t)total;
    const uint32_t W = (b->total_chunks + 63) / 64;
    std::vector<uint32_t>& hint = b->h_hint;
    hint.assign(W + 1, 0);
    {
        uint32_t k = 0;
        for (uint32_t w = 0; w <= W; w++) {
            const uint64_t c = std::min<uint64_t>((uint64_t)w * 64, total ? total - 1 : 0);
            while (k + 1 < b->n_whole && prefix[k + 1] <= c) k++;
            hint[w] = k;
        }
    }
    // the same in units of aligned chunk pairs (pair leaf kernel)
    {
        std::vector<uint32_t>& p2 = b->h_prefix2;
        p2.assign(b->n_whole + 1, 0);
        uint32_t tp = 0;
        b->n_multi2 = 0;
        for (uint32_t k = 0; k < b->n_whole; k++) {
            p2[k] = tp;
            const uint32_t C = msg_chunks(ext[order[k]].msg_len);
            tp += (C + 1) / 2;
            if (C >= 3) b->n_multi2 = k + 1;
        }
        p2[b->n_whole] = tp;
        b->total_pairs = tp;
        // forest groups: consecutive multi-pair files whose pair nodes fit 448 lanes
        b->h_groups2.clear();
        uint32_t first = 0, lanes = 0;
        for (uint32_t k = 0; k < b->n_multi2; k++) {
            const uint32_t L = p2[k + 1] - p2[k];
            if (lanes + L > 448) {
                b->h_groups2.push_back(make_uint2(first, k - first));
                first = k;
                lanes = 0;
            }
            lanes += L;
        }
        if (b->n_multi2) b->h_groups2.push_back(make_uint2(first, b->n_multi2 - first));
        b->n_groups2 = (uint32_t)b->h_groups2.size();
        const uint32_t W2 = (tp + 63) / 64;
        std::vector<uint32_t>& h2 = b->h_hint2;
        h2.assign(W2 + 1, 0);
        uint32_t k = 0;
        for (uint32_t w = 0; w <= W2; w++) {
            const uint64_t c = std::min<uint64_t>((uint64_t)w * 64, tp ? tp - 1 : 0);
            while (k + 1 < b->n_whole && p2[k + 1] <= c) k++;
            h2[w] = k;
        }
    }
    plan_whole_items(b, ext);
    // whole-file groups for the fused kernel: consecutive (length-sorted) files whose
    // chunk pairs fit one 448-lane workgroup
    b->h_groups.clear();
    {
        uint32_t first = 0, lanes = 0;
        for (uint32_t k = 0; k < b->n_whole; k++) {
            const uint32_t L = (msg_chunks(ext[order[k]].msg_len) + 1) / 2;
            if (lanes + L > 448) {
                b->h_groups.push_back(make_uint2(first, k - first));
                first = k;
                lanes = 0;
            }
            lanes += L;
        }
        if (b->n_whole) b->h_groups.push_back(make_uint2(first, b->n_whole - first));
    }
    b->n_groups = (uint32_t)b->h_groups.size();
    b->groups.upload(b->h_groups, stream);
    b->h_ext.assign(ext, ext + n);
    b->ext.upload(b->h_ext, stream);
    b->sidx.upload(sidx, stream);
    b->order.upload(order, stream);
    b->prefix.upload(prefix, stream);
    b->hint.upload(hint, stream);
    b->prefix2.upload(b->h_prefix2, stream);
    b->hint2.upload(b->h_hint2, stream);
    b->groups2.upload(b->h_groups2, stream);
    b->full_items.upload(b->h_full, stream);
    b->tail_items.upload(b->h_tail, stream);
    b->merge_a.upload(b->h_merge_a, stream);
    b->merge_b.upload(b->h_merge_b, stream);
    b->cv2.ensure((size_t)b->n_cv2 * 32);
    b->cvbuf.ensure((size_t)b->total_chunks * 32);
}

sd_cas_batch* build_cas_batch(const sd_extent* ext, size_t n) {
    auto b = std::make_unique<sd_cas_batch>();
    plan_cas_batch(b.get(), ext, n, nullptr);
    return b.release();
}

void run_cas_batch(const sd_cas_batch* b, const uint8_t* d_staged, uint8_t* d_hash32, hipStream_t s,
                   int parts = SD_PART_SAMPLED | SD_PART_WHOLE) {
    uint32_t* out = reinterpret_cast<uint32_t*>(d_hash32);
    const int wv = tuning_get(SD_TUNE_WHOLE_VARIANT);
    if (wv == 0 || wv == 4) {  // one fused launch (4: prefetching pair leaves)
        HIP_CHECK(sdk::launch_cas_mixed(d_staged, b->ext.as<sd_extent>(), b->sidx.as<uint32_t>(),
                                        (parts & SD_PART_SAMPLED) ? b->n_sampled : 0, b->order.as<uint32_t>(),
                                        b->groups.as<uint2>(), (parts & SD_PART_WHOLE) ? b->n_groups : 0, out, s,
                                        wv == 4));
        return;
    }
    if (wv == 6 || wv == 7 || wv == 8) {  // sampled kernel; full-pair / cost-sorted tail-pair items (7, 8: one
                                          // launch; 8: line-pair loads); two merge8 passes
        if (parts & SD_PART_SAMPLED)
            HIP_CHECK(sdk::launch_cas_sampled(d_staged, b->ext.as<sd_extent>(), b->sidx.as<uint32_t>(), b->n_sampled,
                                              out, s));
        if (parts & SD_PART_WHOLE)
            HIP_CHECK(sdk::launch_whole_items(d_staged, b->full_items.as<uint4>(), b->n_full, b->tail_items.as<uint4>(),
                                              b->n_tail, b->merge_a.as<uint4>(), b->n_merge_a, b->merge_b.as<uint4>(),
                                              b->n_merge_b, b->cvbuf.as<uint32_t>(), b->cv2.as<uint32_t>(), out, s,
                                              wv >= 7, wv == 8 ? 2 : 1));
        return;
    }
    if (wv == 3 || wv == 5) {  // sampled kernel; prefetching pair leaf + tree (3) / LDS forest (5) over pair nodes
        if (parts & SD_PART_SAMPLED)
            HIP_CHECK(sdk::launch_cas_sampled(d_staged, b->ext.as<sd_extent>(), b->sidx.as<uint32_t>(), b->n_sampled,
                                              out, s));
        if (parts & SD_PART_WHOLE) {
            HIP_CHECK(sdk::launch_whole_pair_leaf(d_staged, b->ext.as<sd_extent>(), b->order.as<uint32_t>(),
                                                  b->prefix2.as<uint32_t>(), b->hint2.as<uint32_t>(), b->n_whole,
                                                  b->total_pairs, b->cvbuf.as<uint32_t>(), out, s));
            if (wv == 3)
                HIP_CHECK(sdk::launch_whole_tree(b->order.as<uint32_t>(), b->prefix2.as<uint32_t>(), b->n_multi2,
                                                 b->cvbuf.as<uint32_t>(), out, s));
            else
                HIP_CHECK(sdk::launch_whole_forest(b->order.as<uint32_t>(), b->prefix2.as<uint32_t>(),
                                                   b->groups2.as<uint2>(), b->n_groups2, b->cvbuf.as<uint32_t>(), out,
                                                   s));
        }
        return;
    }
    if (tuning_get(SD_TUNE_WHOLE_VARIANT) == 2 && (parts & SD_PART_WHOLE) && (parts & SD_PART_SAMPLED) && b->n_multi) {
        // whole-file leaf, then the sampled kernel on `s` beside the whole-file tree on a
        // side stream (the tree's long single-lane chains leave most issue slots idle)
        auto* mb = const_cast<sd_cas_batch*>(b);
        if (!mb->side) {
            HIP_CHECK(hipStreamCreateWithFlags(&mb->side, hipStreamNonBlocking));
            HIP_CHECK(hipEventCreateWithFlags(&mb->fork, hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&mb->join, hipEventDisableTiming));
        }
        HIP_CHECK(sdk::launch_whole_leaf(d_staged, b->ext.as<sd_extent>(), b->order.as<uint32_t>(),
                                         b->prefix.as<uint32_t>(), b->hint.as<uint32_t>(), b->n_whole,
                                         b->total_chunks, b->cvbuf.as<uint32_t>(), out, s));
        HIP_CHECK(hipEventRecord(mb->fork, s));
        HIP_CHECK(hipStreamWaitEvent(mb->side, mb->fork, 0));
        HIP_CHECK(sdk::launch_whole_tree(b->order.as<uint32_t>(), b->prefix.as<uint32_t>(), b->n_multi,
                                         b->cvbuf.as<uint32_t>(), out, mb->side));
        HIP_CHECK(hipEventRecord(mb->join, mb->side));
        HIP_CHECK(sdk::launch_cas_sampled(d_staged, b->ext.as<sd_extent>(), b->sidx.as<uint32_t>(), b->n_sampled, out,
                                          s));
        HIP_CHECK(hipStreamWaitEvent(s, mb->join, 0));
        return;
    }
    // variant 1 (default): separate sampled kernel, whole-file leaf kernel, whole-file tree
    // kernel -- 1.5% faster than the fused launch in a same-process A/B
    if (parts & SD_PART_SAMPLED)
        HIP_CHECK(sdk::launch_cas_sampled(d_staged, b->ext.as<sd_extent>(), b->sidx.as<uint32_t>(), b->n_sampled, out,
                                          s));
    if (parts & SD_PART_WHOLE)
        HIP_CHECK(sdk::launch_whole(d_staged, b->ext.as<sd_extent>(), b->order.as<uint32_t>(), b->prefix.as<uint32_t>(),
                                    b->hint.as<uint32_t>(), b->n_whole, b->total_chunks, b->n_multi,
                                    b->cvbuf.as<uint32_t>(), out, s));
}

// -------------------------------------------------------------- checksum planning
constexpr uint64_t CK_BLOCK_BYTES = 1024ull * 1024ull;  // 1024 chunks per leaf workgroup

// (Re)plans `b` for these byte ranges reusing its device buffers (grow-only; see
// plan_cas_batch for the stream / host-copy lifetime rule).
void plan_checksum_batch(sd_checksum_batch* b, const uint64_t* offsets, const uint64_t* lens, size_t n,
                         hipStream_t stream) {
    if (n >= (1ull << 31)) throw sd_failure(SD_ERR_INVALID, "batch too large");
    b->n = n;
    b->total_bytes = b->compressions = b->blocks = 0;
    b->files_h.resize(n);
    b->wg_map_h.clear();
    std::vector<uint64_t> level_n(n);  // current level size per file
    uint64_t cv0 = 0;
    for (size_t i = 0; i < n; i++) {
        if (offsets[i] % 16) throw sd_failure(SD_ERR_INVALID, "checksum range " + std::to_string(i) + " not 16-byte aligned");
        const uint64_t nb = lens[i] == 0 ? 1 : (lens[i] + CK_BLOCK_BYTES - 1) / CK_BLOCK_BYTES;
        if (nb >= (1ull << 32)) throw sd_failure(SD_ERR_INVALID, "file too large");
        b->files_h[i] = ck_file{offsets[i], lens[i], nb > 1 ? cv0 : 0};
        for (uint64_t k = 0; k < nb; k++) b->wg_map_h.push_back(make_uint2((uint32_t)i, (uint32_t)k));
        if (nb > 1) cv0 += nb;
        level_n[i] = nb;
        b->total_bytes += lens[i];
        b->compressions += file_compressions(lens[i]);
        b->blocks += nb;
    }
    b->files.upload(b->files_h, stream);
    b->wg_map.upload(b->wg_map_h, stream);
    // reduce passes: groups of 256 CVs per workgroup until every file has its root
    std::vector<uint64_t> base(n, 0);
    for (size_t i = 0; i < n; i++) base[i] = b->files_h[i].cv_base;
    size_t lvl_cap[2] = {cv0, 0};
    int src = 0;
    b->n_passes = 0;
    for (;;) {
        if (b->n_passes == b->passes.size()) b->passes.push_back(std::make_unique<ck_pass>());
        ck_pass& p = *b->passes[b->n_passes];
        p.h_wgs.clear();
        uint64_t dst_total = 0;
        std::vector<uint64_t> nbase(n, 0);
        for (size_t i = 0; i < n; i++) {
            const uint64_t cnt = level_n[i];
            if (cnt <= 1) continue;
            const uint64_t groups = (cnt + 255) / 256;
            nbase[i] = dst_total;
            for (uint64_t g = 0; g < groups; g++) {
                ck_reduce_wg w{};
                w.src_base = base[i] + g * 256;
                w.dst_index = dst_total + g;
                w.count = (uint32_t)std::min<uint64_t>(256, cnt - g * 256);
                w.file = (uint32_t)i;
                w.is_root = groups == 1;
                p.h_wgs.push_back(w);
            }
            dst_total += groups == 1 ? 0 : groups;
            level_n[i] = groups == 1 ? 1 : groups;
        }
        if (p.h_wgs.empty()) break;
        p.wgs.upload(p.h_wgs, stream);
        p.n_wg = (uint32_t)p.h_wgs.size();
        p.src = src;
        p.dst = 1 - src;
        lvl_cap[1 - src] = std::max<size_t>(lvl_cap[1 - src], dst_total);
        b->n_passes++;
        base = nbase;
        src = 1 - src;
    }
    b->lvl[0].ensure(lvl_cap[0] * 32);
    b->lvl[1].ensure(lvl_cap[1] * 32);
}

sd_checksum_batch* build_checksum_batch(const uint64_t* offsets, const uint64_t* lens, size_t n) {
    auto b = std::make_unique<sd_checksum_batch>();
    plan_checksum_batch(b.get(), offsets, lens, n, nullptr);
    return b.release();
}

void run_checksum_leaf(const sd_checksum_batch* b, const uint8_t* d_data, uint64_t shift, uint32_t wg0, uint32_t wg1,
                       uint32_t* out, hipStream_t s);

void run_checksum_reduce(const sd_checksum_batch* b, uint32_t* out, hipStream_t s) {
    for (size_t k = 0; k < b->n_passes; k++) {
        const ck_pass& p = *b->passes[k];
        HIP_CHECK(sdk::launch_ck_reduce(b->lvl[p.src].as<uint32_t>(), b->lvl[p.dst].as<uint32_t>(),
                                        p.wgs.as<ck_reduce_wg>(), p.n_wg, out, s));
    }
}

void run_checksum_batch(const sd_checksum_batch* b, const uint8_t* d_data, uint8_t* d_hash32, hipStream_t s) {
    uint32_t* out = reinterpret_cast<uint32_t*>(d_hash32);
    run_checksum_leaf(b, d_data, 0, 0, (uint32_t)b->wg_map_h.size(), out, s);
    run_checksum_reduce(b, out, s);
}

const char HEX[] = "0123456789abcdef";
void to_hex(const uint8_t* h, int nbytes, char* out) {
    for (int i = 0; i < nbytes; i++) {
        out[2 * i] = HEX[h[i] >> 4];
        out[2 * i + 1] = HEX[h[i] & 15];
    }
    out[2 * nbytes] = 0;
}

int32_t io_status(int err) { return (int32_t)(SD_FILE_IO_ERROR | ((uint32_t)(err & 0xFFFF) << 16)); }

// read exactly n bytes at off; returns 0, or an sd_file_status code
int32_t pread_exact(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
    while (n) {
        const ssize_t r = pread(fd, dst, n, (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return io_status(errno);
        }
        if (r == 0) return SD_FILE_SHORT_READ;
        dst += r;
        n -= (uint64_t)r;
        off += (uint64_t)r;
    }
    return SD_FILE_OK;
}

// Reads one file into its extent exactly as generate_cas_id does (cas.rs:25-58) and
// zero-pads the message to SD_STAGE_PAD.  Returns an sd_file_status.
int32_t stage_one(const char* path, const sd_extent& e, uint8_t* staged) {
    uint8_t* dst = staged + e.msg_offset;
    const uint64_t size = e.size;
    for (int i = 0; i < 8; i++) dst[i] = (uint8_t)(size >> (8 * i));  // cas.rs:25 le64
    const uint64_t padded = align_up(e.msg_len, SD_STAGE_PAD);
    memset(dst + e.msg_len, 0, padded - e.msg_len);
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return io_status(errno);
    int32_t st = SD_FILE_OK;
    if (e.kind == SD_KIND_WHOLE) {  // cas.rs:29 fs::read -- requires len == size
        st = pread_exact(fd, dst + 8, size, 0);
        if (st == SD_FILE_OK) {
            uint8_t extra;
            if (pread(fd, &extra, 1, (off_t)size) == 1) st = SD_FILE_SHORT_READ;  // file grew since stat
        }
    } else {  // cas.rs:31-58: header, 4 samples at 8192 + k*seek_jump, footer
        const uint64_t H = SD_HEADER_OR_FOOTER_SIZE, S = SD_SAMPLE_SIZE;
        const uint64_t jump = (size - 2 * H) / SD_SAMPLE_COUNT;
        uint8_t* p = dst + 8;
        st = pread_exact(fd, p, H, 0);
        p += H;
        uint64_t current_pos = H;
        while (st == SD_FILE_OK) {
            st = pread_exact(fd, p, S, current_pos);
            p += S;
            if (current_pos >= H + jump * (SD_SAMPLE_COUNT - 1)) break;
            current_pos += jump;
        }
        if (st == SD_FILE_OK) st = pread_exact(fd, p, H, size - H);
    }
    close(fd);
    return st;
}

}  // namespace

// ------------------------------------------------------------------ tuning knobs
#include <atomic>
// defaults: sampled U = 2 with line-pair loads (22), whole-file work lists in one launch
// with line-pair loads (8), checksum leaf with line-pair loads (1), LDS-bucket dedup
// grouping (1) -- DESIGN.md §7
static std::atomic<int> g_tune[SD_TUNE_NKEYS] = {{22}, {8}, {1}, {200}, {4096}, {32}, {0}, {1}};
int tuning_get(int key) { return (key >= 0 && key < SD_TUNE_NKEYS) ? g_tune[key].load(std::memory_order_relaxed) : 0; }

// ============================================================================ C ABI
extern "C" {

int sd_cas_set_tuning(const char* key, int value) {
    SD_GUARD_BEGIN
    if (!key) throw sd_failure(SD_ERR_INVALID, "null key");
    static const char* names[SD_TUNE_NKEYS] = {"sampled_variant", "whole_variant", "checksum_variant",
                                               "coalesce_window_us", "coalesce_max", "files_window_mb",
                                               "whole_lds_kb", "dedup_variant"};
    for (int k = 0; k < SD_TUNE_NKEYS; k++)
        if (strcmp(key, names[k]) == 0) {
            g_tune[k].store(value, std::memory_order_relaxed);
            return SD_OK;
        }
    throw sd_failure(SD_ERR_INVALID, std::string("unknown tuning key ") + key);
    SD_GUARD_END
}

int sd_cas_abi_version(void) { return SD_CAS_ABI_VERSION; }

const char* sd_cas_last_error(void) { return g_err.c_str(); }

int sd_cas_ctx_create(int device, sd_cas_ctx** out) {
    SD_GUARD_BEGIN
    if (!out) throw sd_failure(SD_ERR_INVALID, "out is null");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        throw sd_failure(SD_ERR_DEVICE, "no HIP device available (libsdcas has no CPU fallback)");
    if (device < 0 || device >= count) throw sd_failure(SD_ERR_INVALID, "device index out of range");
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        throw sd_failure(SD_ERR_DEVICE, std::string("libsdcas is built for gfx950, device is ") + prop.gcnArchName);
    auto c = std::make_unique<sd_cas_ctx>();
    c->device = device;
    c->bind();
    HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    *out = c.release();
    return SD_OK;
    SD_GUARD_END
}

void sd_cas_ctx_destroy(sd_cas_ctx* ctx) {
    if (!ctx) return;
    try {
        if (ctx->coal) coalescer_destroy(ctx->coal);  // drains its queue, joins the dispatcher
        ctx->coal = nullptr;
        ctx->bind();
        (void)hipDeviceSynchronize();
        for (auto& s : ctx->free_slots)
            if (s->stream) (void)hipStreamDestroy(s->stream);
        ctx->free_slots.clear();
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    } catch (...) {
    }
    delete ctx;
}

int sd_cas_host_alloc(sd_cas_ctx* ctx, uint64_t bytes, void** out) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    HIP_CHECK(hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault));
    return SD_OK;
    SD_GUARD_END
}

void sd_cas_host_free(sd_cas_ctx* ctx, void* p) {
    if (p) (void)hipHostFree(p);
}

int sd_cas_stage_plan(const uint64_t* sizes, size_t n, sd_extent* extents_out, uint64_t* total_bytes_out) {
    SD_GUARD_BEGIN
    if ((!sizes || !extents_out) && n) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (!total_bytes_out) throw sd_failure(SD_ERR_INVALID, "total_bytes_out is null");
    uint64_t off = 0;
    for (size_t i = 0; i < n; i++) {
        sd_extent& e = extents_out[i];
        e.size = sizes[i];
        const bool whole = sizes[i] <= SD_MINIMUM_FILE_SIZE;  // cas.rs:27 (<=)
        e.kind = whole ? SD_KIND_WHOLE : SD_KIND_SAMPLED;
        e.msg_len = whole ? (uint32_t)(8 + sizes[i]) : SD_SAMPLED_MSG_LEN;
        e.msg_offset = off;
        off = align_up(off + e.msg_len, SD_STAGE_ALIGN);
    }
    *total_bytes_out = off;
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_stage_file(const char* path, const sd_extent* ext, uint8_t* staged, int32_t* status) {
    SD_GUARD_BEGIN
    if (!path || !ext || !staged || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    validate_extent(*ext, 0);
    *status = stage_one(path, *ext, staged);
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_stage_files(const char* const* paths, const sd_extent* extents, size_t n, uint8_t* staged,
                       int32_t* status, int nthreads) {
    SD_GUARD_BEGIN
    if (n && (!paths || !extents || !staged || !status)) throw sd_failure(SD_ERR_INVALID, "null argument");
    for (size_t i = 0; i < n; i++) validate_extent(extents[i], i);
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    std::atomic<size_t> cursor{0};
    auto work = [&]() {
        for (;;) {
            const size_t i = cursor.fetch_add(1, std::memory_order_relaxed);
            if (i >= n) break;
            status[i] = stage_one(paths[i], extents[i], staged);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; t++) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_batch_create(sd_cas_ctx* ctx, const sd_extent* extents, size_t n, sd_cas_batch** out) {
    SD_GUARD_BEGIN
    if (!ctx || !out || (!extents && n)) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    *out = build_cas_batch(extents, n);
    return SD_OK;
    SD_GUARD_END
}

void sd_cas_batch_destroy(sd_cas_batch* batch) {
    try {
        delete batch;
    } catch (...) {
    }
}

int sd_cas_batch_run(sd_cas_ctx* ctx, const sd_cas_batch* batch, const uint8_t* d_staged, uint8_t* d_hash32,
                     void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !batch || (batch->n && (!d_staged || !d_hash32))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    run_cas_batch(batch, d_staged, d_hash32, ctx->pick(stream));
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_batch_run_part(sd_cas_ctx* ctx, const sd_cas_batch* batch, int parts, const uint8_t* d_staged,
                          uint8_t* d_hash32, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !batch || (batch->n && (!d_staged || !d_hash32))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    run_cas_batch(batch, d_staged, d_hash32, ctx->pick(stream), parts);
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_batch_stats(const sd_cas_batch* b, uint64_t out[6]) {
    SD_GUARD_BEGIN
    if (!b || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = b->n; out[1] = b->n_sampled; out[2] = b->n_whole; out[3] = b->total_chunks;
    out[4] = b->compressions; out[5] = b->msg_bytes;
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_ids(sd_cas_ctx* ctx, const uint8_t* staged, uint64_t staged_bytes, const sd_extent* extents, size_t n,
               char* out_hex17, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!staged || !extents || !out_hex17))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    // files whose staging failed keep their status and are not hashed
    std::vector<size_t> live;
    live.reserve(n);
    for (size_t i = 0; i < n; i++)
        if (!status || status[i] == SD_FILE_OK) live.push_back(i);
    // windows of files (index order) whose staged span fits WINDOW bytes; two slots
    // alternate so window k+1's H2D copy overlaps window k's kernels
    const uint64_t WINDOW = 512ull << 20;
    struct Win {
        size_t gi = 0, gj = 0;
        bool busy = false;
    };
    std::unique_ptr<Slot> slots[2] = {ctx->acquire(), ctx->acquire()};
    struct Rel {
        sd_cas_ctx* c;
        std::unique_ptr<Slot>* s;
        ~Rel() {
            for (int k = 0; k < 2; k++)
                if (s[k]) {
                    (void)hipStreamSynchronize(s[k]->stream);
                    c->release(std::move(s[k]));
                }
        }
    } rel{ctx, slots};
    sd_cas_batch batches[2];
    Win wins[2];
    auto harvest = [&](int k) {
        if (!wins[k].busy) return;
        HIP_CHECK(hipStreamSynchronize(slots[k]->stream));
        const uint8_t* h = reinterpret_cast<const uint8_t*>(slots[k]->host_hashes.p);
        for (size_t q = wins[k].gi; q < wins[k].gj; q++) {
            to_hex(h + (q - wins[k].gi) * 32, 8, out_hex17 + live[q] * 17);  // cas.rs:61 to_hex()[..16]
            if (status) status[live[q]] = SD_FILE_OK;
        }
        wins[k].busy = false;
    };
    std::vector<sd_extent> ext;
    size_t gi = 0;
    for (int w = 0; gi < live.size(); w ^= 1) {
        harvest(w);  // frees slot w (its previous window is done)
        uint64_t lo = UINT64_MAX, hi = 0;
        size_t gj = gi;
        while (gj < live.size()) {
            const sd_extent& e = extents[live[gj]];
            const uint64_t nlo = std::min(lo, e.msg_offset);
            const uint64_t nhi = std::max(hi, align_up(e.msg_offset + e.msg_len, SD_STAGE_PAD));
            if (gj > gi && nhi - nlo > WINDOW) break;
            lo = nlo;
            hi = nhi;
            gj++;
        }
        if (hi > staged_bytes) throw sd_failure(SD_ERR_INVALID, "extent beyond staged_bytes");
        ext.clear();
        for (size_t q = gi; q < gj; q++) {
            sd_extent e = extents[live[q]];
            e.msg_offset -= lo;
            ext.push_back(e);
        }
        Slot& sl = *slots[w];
        plan_cas_batch(&batches[w], ext.data(), ext.size(), sl.stream);
        sl.staged.ensure(hi - lo);
        sl.hashes.ensure(ext.size() * 32);
        sl.host_hashes.ensure(ext.size() * 32);
        HIP_CHECK(hipMemcpyAsync(sl.staged.p, staged + lo, hi - lo, hipMemcpyHostToDevice, sl.stream));
        run_cas_batch(&batches[w], sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, ext.size() * 32, hipMemcpyDeviceToHost, sl.stream));
        wins[w] = Win{gi, gj, true};
        gi = gj;
    }
    harvest(0);
    harvest(1);
    return SD_OK;
    SD_GUARD_END
}

// Path-based drop-in batch: generate_cas_id (cas.rs:23-62) for n (path, size) pairs,
// the sizes being the ones the caller's metadata reported (FileMetadata::new,
// file_identifier/mod.rs:65-97).  Files are planned into windows of consecutive files;
// the stager pool preads window k+1 into one pinned slot while window k's H2D copy,
// kernels and D2H run on the other slot's stream.
int sd_cas_ids_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n, char* out_hex17,
                     int32_t* status, int nthreads) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!paths || !sizes || !out_hex17 || !status))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    StagePool& pool = ctx->stage_pool(nthreads);
    const uint64_t WINDOW = (uint64_t)std::max(1, tuning_get(SD_TUNE_FILES_WINDOW_MB)) << 20;
    std::unique_ptr<Slot> slots[2] = {ctx->acquire(), ctx->acquire()};
    struct Rel {
        sd_cas_ctx* c;
        std::unique_ptr<Slot>* s;
        ~Rel() {
            for (int k = 0; k < 2; k++)
                if (s[k]) {
                    (void)hipStreamSynchronize(s[k]->stream);
                    c->release(std::move(s[k]));
                }
        }
    } rel{ctx, slots};
    sd_cas_batch batches[2];
    struct Win {
        std::vector<size_t> files;  // hashed files of the window, in extent order
        bool busy = false;
    } wins[2];
    auto harvest = [&](int k) {
        if (!wins[k].busy) return;
        HIP_CHECK(hipStreamSynchronize(slots[k]->stream));
        const uint8_t* h = reinterpret_cast<const uint8_t*>(slots[k]->host_hashes.p);
        for (size_t q = 0; q < wins[k].files.size(); q++)
            to_hex(h + q * 32, 8, out_hex17 + wins[k].files[q] * 17);  // cas.rs:61 to_hex()[..16]
        wins[k].busy = false;
    };
    std::vector<sd_extent> ext;
    std::vector<size_t> idx;
    size_t i = 0;
    for (int w = 0; i < n; w ^= 1) {
        // the next window: consecutive files whose messages fit WINDOW bytes
        ext.clear();
        idx.clear();
        uint64_t off = 0;
        while (i < n) {
            const bool whole = sizes[i] <= SD_MINIMUM_FILE_SIZE;  // cas.rs:27
            const uint32_t len = whole ? (uint32_t)(8 + sizes[i]) : SD_SAMPLED_MSG_LEN;
            const uint64_t next = align_up(off + len, SD_STAGE_ALIGN);
            if (!ext.empty() && next > WINDOW) break;
            ext.push_back(sd_extent{sizes[i], off, len, whole ? (uint32_t)SD_KIND_WHOLE : (uint32_t)SD_KIND_SAMPLED});
            idx.push_back(i);
            off = next;
            i++;
        }
        harvest(w);  // slot w's previous window is done: its pinned buffer is free
        Slot& sl = *slots[w];
        sl.window.ensure(off + 64);
        uint8_t* win = reinterpret_cast<uint8_t*>(sl.window.p);
        pool.run(ext.size(), [&](size_t q) { status[idx[q]] = stage_one(paths[idx[q]], ext[q], win); });
        // failed files (I/O error, short read) keep their status and leave the window
        size_t m = 0;
        for (size_t q = 0; q < ext.size(); q++)
            if (status[idx[q]] == SD_FILE_OK) {
                ext[m] = ext[q];
                idx[m++] = idx[q];
            }
        ext.resize(m);
        idx.resize(m);
        if (m == 0) continue;
        plan_cas_batch(&batches[w], ext.data(), m, sl.stream);
        sl.staged.ensure(off + 64);
        sl.hashes.ensure(m * 32);
        sl.host_hashes.ensure(m * 32);
        HIP_CHECK(hipMemcpyAsync(sl.staged.p, win, off, hipMemcpyHostToDevice, sl.stream));
        run_cas_batch(&batches[w], sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, m * 32, hipMemcpyDeviceToHost, sl.stream));
        wins[w].files = idx;
        wins[w].busy = true;
    }
    harvest(0);
    harvest(1);
    return SD_OK;
    SD_GUARD_END
}

// ------------------------------------------------------------------- latency path
int sd_cas_id_path(sd_cas_ctx* ctx, const char* path, uint64_t size, char* out_hex17, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || !path || !out_hex17 || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    std::string err;
    const int rc = coalescer_submit(ctx->coalescer(), 0, path, size, out_hex17, status, &err);
    if (rc != SD_OK) set_err("%s", err.c_str());
    return rc;
    SD_GUARD_END
}

int sd_file_checksum_path(sd_cas_ctx* ctx, const char* path, char* out_hex65, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || !path || !out_hex65 || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    std::string err;
    const int rc = coalescer_submit(ctx->coalescer(), 1, path, 0, out_hex65, status, &err);
    if (rc != SD_OK) set_err("%s", err.c_str());
    return rc;
    SD_GUARD_END
}

int sd_coalescer_stats(sd_cas_ctx* ctx, uint64_t out[3]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    coalescer_stats(ctx->coalescer(), out);
    return SD_OK;
    SD_GUARD_END
}

// ---------------------------------------------------------------------- checksums
int sd_checksum_batch_create(sd_cas_ctx* ctx, const uint64_t* offsets, const uint64_t* lens, size_t n,
                             sd_checksum_batch** out) {
    SD_GUARD_BEGIN
    if (!ctx || !out || (n && (!offsets || !lens))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    *out = build_checksum_batch(offsets, lens, n);
    return SD_OK;
    SD_GUARD_END
}

void sd_checksum_batch_destroy(sd_checksum_batch* b) {
    try {
        delete b;
    } catch (...) {
    }
}

int sd_checksum_batch_run(sd_cas_ctx* ctx, const sd_checksum_batch* b, const uint8_t* d_data, uint8_t* d_hash32,
                          void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !b || (b->n && (!d_data || !d_hash32))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    run_checksum_batch(b, d_data, d_hash32, ctx->pick(stream));
    return SD_OK;
    SD_GUARD_END
}

int sd_checksum_batch_stats(const sd_checksum_batch* b, uint64_t out[4]) {
    SD_GUARD_BEGIN
    if (!b || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = b->n; out[1] = b->total_bytes; out[2] = b->compressions; out[3] = b->blocks;
    return SD_OK;
    SD_GUARD_END
}

int sd_file_checksums(sd_cas_ctx* ctx, const char* const* paths, size_t n, char* out_hex65, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!paths || !out_hex65 || !status))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    // Two slots, each with a pinned window, a device window and a stream.  Files that fit
    // a window are packed (64-B aligned) into one batch per window; larger files stream
    // window by window into their own batch's leaf CVs, then reduce.  While the GPU hashes
    // one slot's window, the host reads the next window into the other slot.
    const uint64_t W = 256ull << 20;  // a multiple of the 1 MiB leaf block
    std::unique_ptr<Slot> slots[2] = {ctx->acquire(), ctx->acquire()};
    struct Rel {
        sd_cas_ctx* c;
        std::unique_ptr<Slot>* s;
        ~Rel() {
            for (int k = 0; k < 2; k++)
                if (s[k]) {
                    (void)hipStreamSynchronize(s[k]->stream);
                    c->release(std::move(s[k]));
                }
        }
    } rel{ctx, slots};
    for (int k = 0; k < 2; k++) {
        slots[k]->window.ensure(W + 128);
        slots[k]->staged.ensure(W + 128);
    }
    struct Pending {
        std::vector<size_t> files;  // files whose hashes land in this slot's host_hashes
        bool busy = false;
    } pend[2];
    sd_checksum_batch pack_batch[2], big;
    int cur = 0;
    auto harvest = [&](int k) {
        if (!pend[k].busy) return;
        HIP_CHECK(hipStreamSynchronize(slots[k]->stream));
        const uint8_t* h = reinterpret_cast<const uint8_t*>(slots[k]->host_hashes.p);
        for (size_t q = 0; q < pend[k].files.size(); q++)
            to_hex(h + 32 * q, 32, out_hex65 + pend[k].files[q] * 65);  // hash.rs:21-23
        pend[k].files.clear();
        pend[k].busy = false;
    };
    std::vector<size_t> pack;
    std::vector<uint64_t> pack_len;
    uint64_t pack_bytes = 0;
    auto submit_pack = [&]() {
        if (pack.empty()) return;
        const int k = cur;
        cur ^= 1;
        harvest(k);
        Slot& sl = *slots[k];
        uint8_t* win = reinterpret_cast<uint8_t*>(sl.window.p);
        std::vector<uint64_t> offs, lens;
        std::vector<size_t> ok;
        uint64_t off = 0;
        for (size_t q = 0; q < pack.size(); q++) {  // hash.rs:13-20 reads, one pread per file
            const size_t i = pack[q];
            const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
            if (fd < 0) {
                status[i] = io_status(errno);
                continue;
            }
            const int32_t st = pread_exact(fd, win + off, pack_len[q], 0);
            close(fd);
            if (st != SD_FILE_OK) {
                status[i] = st;
                continue;
            }
            memset(win + off + pack_len[q], 0, align_up(pack_len[q] + 1, 64) - pack_len[q]);
            offs.push_back(off);
            lens.push_back(pack_len[q]);
            ok.push_back(i);
            off = align_up(off + pack_len[q] + 1, 64);
        }
        pack.clear();
        pack_len.clear();
        pack_bytes = 0;
        if (ok.empty()) return;
        plan_checksum_batch(&pack_batch[k], offs.data(), lens.data(), ok.size(), sl.stream);
        sl.hashes.ensure(ok.size() * 32);
        sl.host_hashes.ensure(ok.size() * 32);
        HIP_CHECK(hipMemcpyAsync(sl.staged.p, win, off + 64, hipMemcpyHostToDevice, sl.stream));
        run_checksum_batch(&pack_batch[k], sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, ok.size() * 32, hipMemcpyDeviceToHost, sl.stream));
        pend[k].files = std::move(ok);
        pend[k].busy = true;
    };
    for (size_t i = 0; i < n; i++) {
        status[i] = SD_FILE_OK;
        struct stat stt;
        if (stat(paths[i], &stt) != 0) {
            status[i] = io_status(errno);
            continue;
        }
        const uint64_t len = (uint64_t)stt.st_size;  // hash.rs reads to EOF; the length is fixed here
        if (len + 128 <= W) {
            if (pack_bytes + align_up(len + 1, 64) + 64 > W) submit_pack();
            pack.push_back(i);
            pack_len.push_back(len);
            pack_bytes += align_up(len + 1, 64);
            continue;
        }
        // a large file: flush the pack, then stream windows through alternating slots
        submit_pack();
        harvest(0);
        harvest(1);
        const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
            status[i] = io_status(errno);
            continue;
        }
        const uint64_t off0 = 0;
        plan_checksum_batch(&big, &off0, &len, 1, nullptr);
        for (int k = 0; k < 2; k++) slots[k]->hashes.ensure(32);
        const uint32_t blocks_per_window = (uint32_t)(W / CK_BLOCK_BYTES);
        for (uint64_t pos = 0; pos < len && status[i] == SD_FILE_OK; pos += W) {
            const int k = cur;
            cur ^= 1;
            HIP_CHECK(hipStreamSynchronize(slots[k]->stream));  // its window is free again
            Slot& sl = *slots[k];
            uint8_t* win = reinterpret_cast<uint8_t*>(sl.window.p);
            const uint64_t n_here = std::min<uint64_t>(W, len - pos);
            const int32_t st = pread_exact(fd, win, n_here, pos);
            if (st != SD_FILE_OK) {
                status[i] = st;
                break;
            }
            memset(win + n_here, 0, 64);
            HIP_CHECK(hipMemcpyAsync(sl.staged.p, win, align_up(n_here, 64) + 64, hipMemcpyHostToDevice, sl.stream));
            const uint32_t wg0 = (uint32_t)(pos / CK_BLOCK_BYTES);
            const uint32_t wg1 = (uint32_t)std::min<uint64_t>(big.wg_map_h.size(), (uint64_t)wg0 + blocks_per_window);
            run_checksum_leaf(&big, sl.staged.as<uint8_t>(), pos, wg0, wg1, sl.hashes.as<uint32_t>(), sl.stream);
        }
        close(fd);
        HIP_CHECK(hipStreamSynchronize(slots[0]->stream));
        HIP_CHECK(hipStreamSynchronize(slots[1]->stream));
        if (status[i] != SD_FILE_OK) continue;
        Slot& sl = *slots[0];
        run_checksum_reduce(&big, sl.hashes.as<uint32_t>(), sl.stream);
        sl.host_hashes.ensure(32);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, 32, hipMemcpyDeviceToHost, sl.stream));
        HIP_CHECK(hipStreamSynchronize(sl.stream));
        to_hex(reinterpret_cast<const uint8_t*>(sl.host_hashes.p), 32, out_hex65 + i * 65);
    }
    submit_pack();
    harvest(0);
    harvest(1);
    return SD_OK;
    SD_GUARD_END
}

// -------------------------------------------------------------------------- dedup
int sd_dedup_partition(sd_cas_ctx* ctx, const uint8_t* d_hash32, const uint8_t* d_valid, uint64_t n,
                       uint64_t global_index_base, int nparts, uint64_t* d_counts, uint64_t* d_records,
                       uint64_t* n_valid, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !d_counts || !n_valid || (n && (!d_hash32 || !d_records)))
        throw sd_failure(SD_ERR_INVALID, "null argument");
    if (nparts < 1 || nparts > 64) throw sd_failure(SD_ERR_INVALID, "nparts must be in [1, 64]");
    ctx->bind();
    hipStream_t s = ctx->pick(stream);
    auto slot = ctx->acquire();  // scratch reused across calls; released after the sync below
    struct Rel {
        sd_cas_ctx* c;
        std::unique_ptr<Slot>* s;
        ~Rel() { c->release(std::move(*s)); }
    } rel{ctx, &slot};
    const size_t sb = sdk::dedup_partition_scratch(nparts);
    slot->hashes.ensure(sb);
    slot->host_hashes.ensure(sizeof(uint64_t));
    uint64_t* scratch = slot->hashes.as<uint64_t>();
    HIP_CHECK(sdk::dedup_partition(d_hash32, d_valid, n, global_index_base, nparts, d_counts, d_records, scratch, s));
    HIP_CHECK(hipMemcpyAsync(slot->host_hashes.p, scratch + sb / sizeof(uint64_t) - 1, sizeof(uint64_t),
                             hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    *n_valid = *reinterpret_cast<uint64_t*>(slot->host_hashes.p);
    return SD_OK;
    SD_GUARD_END
}

int sd_dedup_group(sd_cas_ctx* ctx, uint64_t* d_records, uint64_t m, int flags, uint64_t* d_rep,
                   uint64_t* n_groups, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !n_groups || (m && (!d_records || !d_rep))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    hipStream_t s = ctx->pick(stream);
    size_t need = 0;
    HIP_CHECK(sdk::dedup_group(d_records, m, flags, d_rep, nullptr, nullptr, &need, s));
    auto slot = ctx->acquire();
    struct Rel {
        sd_cas_ctx* c;
        std::unique_ptr<Slot>* s;
        ~Rel() { c->release(std::move(*s)); }
    } rel{ctx, &slot};
    const bool buckets = tuning_get(SD_TUNE_DEDUP_VARIANT) == 1 && m > 0 && m < (1ull << 31);
    if (buckets) need = std::max(need, sdk::dedup_group_buckets_scratch(m));
    slot->staged.ensure(need);
    slot->hashes.ensure(8 * sizeof(uint64_t));
    slot->host_hashes.ensure(2 * sizeof(uint64_t));
    size_t have = slot->staged.bytes;
    if (buckets) {
        HIP_CHECK(sdk::dedup_group_buckets(d_records, m, d_rep, slot->hashes.as<uint64_t>(), slot->staged.p, have, s));
        HIP_CHECK(hipMemcpyAsync(slot->host_hashes.p, slot->hashes.p, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        const uint64_t* st = reinterpret_cast<const uint64_t*>(slot->host_hashes.p);
        if (st[1] == 0) {
            *n_groups = st[0];
            return SD_OK;
        }
        flags &= ~SD_DEDUP_INDEX_SORTED;  // a bucket overflowed: d_records is now a permutation
    }
    HIP_CHECK(sdk::dedup_group(d_records, m, flags, d_rep, slot->hashes.as<uint64_t>(), slot->staged.p, &have, s));
    HIP_CHECK(hipMemcpyAsync(slot->host_hashes.p, slot->hashes.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    *n_groups = *reinterpret_cast<uint64_t*>(slot->host_hashes.p);
    return SD_OK;
    SD_GUARD_END
}

int sd_dedup_owners(sd_cas_ctx* ctx, const uint64_t* d_records, uint64_t m, const uint64_t* d_rep,
                    uint64_t chunk_size, uint64_t* d_owner, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || (m && (!d_records || !d_rep || !d_owner))) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (chunk_size == 0) throw sd_failure(SD_ERR_INVALID, "chunk_size must be positive");
    ctx->bind();
    HIP_CHECK(sdk::dedup_owners(d_records, m, d_rep, chunk_size, d_owner, ctx->pick(stream)));
    return SD_OK;
    SD_GUARD_END
}

// ----------------------------------------------------------------- synthetic data
int sd_synth_stage_cas(sd_cas_ctx* ctx, const uint64_t* d_sizes, const uint64_t* d_cids, const uint32_t* d_twins,
                       const sd_extent* d_extents, size_t n, uint8_t* d_staged, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!d_sizes || !d_cids || !d_extents || !d_staged))) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (n >= (1ull << 31)) throw sd_failure(SD_ERR_INVALID, "too many files");
    ctx->bind();
    HIP_CHECK(sdk::launch_synth_stage_cas(d_sizes, d_cids, d_twins, d_extents, (uint32_t)n, d_staged, ctx->pick(stream)));
    return SD_OK;
    SD_GUARD_END
}

int sd_synth_fill(sd_cas_ctx* ctx, uint64_t cid, uint32_t twin, uint64_t len, uint8_t* d_out, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || (len && !d_out)) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    HIP_CHECK(sdk::launch_synth_fill(cid, twin, len, d_out, ctx->pick(stream)));
    return SD_OK;
    SD_GUARD_END
}

// -------------------------------------------------------------- device utilities
int sd_device_malloc(sd_cas_ctx* ctx, uint64_t bytes, void** out) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    HIP_CHECK(hipMalloc(out, bytes ? bytes : 16));
    return SD_OK;
    SD_GUARD_END
}

void sd_device_free(sd_cas_ctx* ctx, void* p) {
    if (p) (void)hipFree(p);
}

int sd_memcpy(sd_cas_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || (bytes && (!dst || !src))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    hipStream_t s = ctx->pick(stream);
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return SD_OK;
    SD_GUARD_END
}

int sd_stream_sync(sd_cas_ctx* ctx, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    HIP_CHECK(hipStreamSynchronize(ctx->pick(stream)));
    return SD_OK;
    SD_GUARD_END
}

static int time_loop(sd_cas_ctx* ctx, void* stream, int iters, float* ms, const std::function<void(hipStream_t)>& fn);

int sd_cas_batch_time(sd_cas_ctx* ctx, const sd_cas_batch* batch, const uint8_t* d_staged, uint8_t* d_hash32,
                      int iters, void* stream, float* ms_total) {
    return time_loop(ctx, stream, iters, ms_total,
                     [&](hipStream_t s) { run_cas_batch(batch, d_staged, d_hash32, s); });
}

int sd_checksum_batch_time(sd_cas_ctx* ctx, const sd_checksum_batch* batch, const uint8_t* d_data, uint8_t* d_hash32,
                           int iters, void* stream, float* ms_total) {
    return time_loop(ctx, stream, iters, ms_total,
                     [&](hipStream_t s) { run_checksum_batch(batch, d_data, d_hash32, s); });
}

int sd_read_probe(sd_cas_ctx* ctx, const uint8_t* d_buf, uint64_t bytes, int pattern, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !d_buf || bytes % 4096) throw sd_failure(SD_ERR_INVALID, "bad argument (bytes % 4096 != 0)");
    ctx->bind();
    HIP_CHECK(sdk::launch_read_probe(d_buf, bytes, pattern, ctx->pick(stream)));
    return SD_OK;
    SD_GUARD_END
}

int sd_valu_peak(sd_cas_ctx* ctx, double* lane_ops_per_s) {
    SD_GUARD_BEGIN
    if (!ctx || !lane_ops_per_s) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, ctx->device));
    const uint32_t grid = (uint32_t)prop.multiProcessorCount * 8;  // 8 x 256 threads per CU
    const uint32_t iters = 512;
    DevBuf sink;
    sink.alloc((size_t)grid * 256 * 4);
    hipStream_t s = ctx->stream;
    HIP_CHECK(sdk::launch_valu_peak(sink.as<uint32_t>(), iters, grid, s));  // warm-up
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    HIP_CHECK(hipEventRecord(a, s));
    const int reps = 3;
    for (int r = 0; r < reps; r++) HIP_CHECK(sdk::launch_valu_peak(sink.as<uint32_t>(), iters, grid, s));
    HIP_CHECK(hipEventRecord(b, s));
    HIP_CHECK(hipEventSynchronize(b));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double ops = (double)reps * grid * 256.0 * iters * 96.0;  // 8 G-mixes x 12 ops per iteration
    *lane_ops_per_s = ops / (ms * 1e-3);
    return SD_OK;
    SD_GUARD_END
}

}  // extern "C"

// ----------------------------------------------------------------- internal helpers
namespace {
void run_checksum_leaf(const sd_checksum_batch* b, const uint8_t* d_data, uint64_t shift, uint32_t wg0, uint32_t wg1,
                       uint32_t* out, hipStream_t s) {
    if (wg1 <= wg0) return;
    HIP_CHECK(sdk::launch_ck_leaf(d_data, shift, b->files.as<ck_file>(), b->wg_map.as<uint2>() + wg0, wg1 - wg0,
                                  b->lvl[0].as<uint32_t>(), out, s));
}
}  // namespace

static int time_loop(sd_cas_ctx* ctx, void* stream, int iters, float* ms,
                     const std::function<void(hipStream_t)>& fn) {
    SD_GUARD_BEGIN
    if (!ctx || !ms || iters < 1) throw sd_failure(SD_ERR_INVALID, "bad argument");
    ctx->bind();
    hipStream_t s = ctx->pick(stream);
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    HIP_CHECK(hipEventRecord(a, s));
    for (int i = 0; i < iters; i++) fn(s);
    HIP_CHECK(hipEventRecord(b, s));
    HIP_CHECK(hipEventSynchronize(b));
    HIP_CHECK(hipEventElapsedTime(ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return SD_OK;
    SD_GUARD_END
}
