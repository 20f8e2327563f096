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
#include <atomic>
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

#include "sd_host.h"
#include "sd_internal.h"
#include "stage_pool.h"

namespace {

#define HIP_CHECK(expr)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            throw sd_failure(e_ == hipErrorOutOfMemory ? SD_ERR_NOMEM : SD_ERR_DEVICE,              \
                             std::string(#expr) + ": " + hipGetErrorString(e_));                    \
    } while (0)

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
    // File stager threads (sd_cas_ids_files).  One pool per context, grown to the largest
    // thread count any call asked for; a caller holds its shared_ptr while it runs, so a
    // concurrent call that grows the pool never destroys one in use.
    std::shared_ptr<StagePool> pool;
    std::shared_ptr<StagePool> stage_pool(int nthreads) {
        std::lock_guard<std::mutex> g(pool_mu);
        if (!pool || pool->threads() < nthreads) pool = std::make_shared<StagePool>(nthreads);
        return pool;
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

namespace {

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
        HIP_CHECK(hipStreamSynchronize(s[0]->stream));
        HIP_CHECK(hipStreamSynchronize(s[1]->stream));
    }
};

}  // namespace

struct sd_checksum_batch {
    size_t n = 0;
    CkPlan plan;
    DevBuf files, wg_map;
    DevBuf lvl[2];
    std::vector<std::unique_ptr<DevBuf>> pass_wgs;  // capacity reused across replans
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
    DevBuf ext, sidx, soff, full_items, tail_items, merge_a, merge_b, cvbuf, cv2;
    // whole-file messages longer than SD_WHOLE_ITEMS_MAX: a checksum sub-batch over their
    // byte ranges, its hashes scattered to out[long_idx[i]]
    sd_checksum_batch lng;
    DevBuf long_idx, long_out;
    // host copies backing async uploads
    std::vector<sd_extent> h_ext;
    std::vector<uint32_t> h_sidx, h_long_idx;
    std::vector<uint64_t> h_soff;
};

namespace {

// ----------------------------------------------------------- checksum batches (device)
// (Re)plans `b` for these byte ranges reusing its device buffers (grow-only).  With a
// stream, the small uploads are async on it and read from b's host copies, which stay
// valid until the next rebuild of `b` (the caller syncs the stream before that).
void plan_checksum_batch(sd_checksum_batch* b, const uint64_t* offsets, const uint64_t* lens, size_t n,
                         hipStream_t stream) {
    plan_checksum(b->plan, offsets, lens, n);
    b->n = n;
    b->files.upload(b->plan.files, stream);
    b->wg_map.upload(b->plan.wg_map, stream);
    while (b->pass_wgs.size() < b->plan.passes.size()) b->pass_wgs.push_back(std::make_unique<DevBuf>());
    for (size_t k = 0; k < b->plan.passes.size(); k++) b->pass_wgs[k]->upload(b->plan.passes[k], stream);
    b->lvl[0].ensure(b->plan.lvl_cap[0] * 32);
    b->lvl[1].ensure(b->plan.lvl_cap[1] * 32);
}

void run_checksum_reduce(const sd_checksum_batch* b, uint32_t* out, hipStream_t s) {
    for (size_t k = 0; k < b->plan.passes.size(); k++) {
        const int src = (int)(k & 1);  // level 0 -> 1 -> 0 ...
        HIP_CHECK(sdk::launch_ck_reduce(b->lvl[src].as<uint32_t>(), b->lvl[1 - src].as<uint32_t>(),
                                        b->pass_wgs[k]->as<ck_reduce_wg>(), (uint32_t)b->plan.passes[k].size(), out,
                                        s));
    }
}

void run_checksum_batch(const sd_checksum_batch* b, const uint8_t* d_data, uint8_t* d_hash32, hipStream_t s) {
    uint32_t* out = reinterpret_cast<uint32_t*>(d_hash32);
    HIP_CHECK(sdk::launch_ck_leaf(d_data, 0, 0, b->files.as<ck_file>(), b->wg_map.as<uint2>(),
                                  (uint32_t)b->plan.wg_map.size(), b->lvl[0].as<uint32_t>(), out, s));
    run_checksum_reduce(b, out, s);
}

// ---------------------------------------------------------------- cas batches (device)
// (Re)plans `b` for these extents, reusing its device buffers (see plan_checksum_batch for
// the stream / host-copy lifetime rule).
void plan_cas_batch(sd_cas_batch* b, const sd_extent* ext, size_t n, hipStream_t stream) {
    if (n >= (1ull << 31)) throw sd_failure(SD_ERR_INVALID, "batch too large");
    b->n = n;
    b->n_whole = 0;
    b->compressions = b->msg_bytes = b->whole_chunks = 0;
    b->h_sidx.clear();
    b->h_soff.clear();
    b->h_long_idx.clear();
    std::vector<uint64_t> loff, llen;
    uint64_t end = 0;
    for (size_t i = 0; i < n; i++) {
        const sd_extent& e = ext[i];
        validate_extent(e, i);
        end = std::max<uint64_t>(end, align_up(e.msg_offset + e.msg_len, SD_STAGE_PAD));
        b->msg_bytes += e.msg_len;
        if (e.kind == SD_KIND_SAMPLED) {
            b->h_sidx.push_back((uint32_t)i);
            b->h_soff.push_back(e.msg_offset);
            b->compressions += 953;  // 56 x 16 + 1 blocks, 56 parents
        } else if (e.msg_len <= SD_WHOLE_ITEMS_MAX) {
            b->n_whole++;
            b->whole_chunks += msg_chunks(e.msg_len);
            b->compressions += msg_compressions(e.msg_len);
        } else {
            b->h_long_idx.push_back((uint32_t)i);
            loff.push_back(e.msg_offset);
            llen.push_back(e.msg_len);
        }
    }
    b->staged_bytes = end;
    b->n_sampled = (uint32_t)b->h_sidx.size();
    b->n_long = (uint32_t)b->h_long_idx.size();
    plan_whole_items(b->whole, ext, n);
    b->h_ext.assign(ext, ext + n);
    b->ext.upload(b->h_ext, stream);
    b->sidx.upload(b->h_sidx, stream);
    b->soff.upload(b->h_soff, stream);
    b->full_items.upload(b->whole.full, stream);
    b->tail_items.upload(b->whole.tail, stream);
    b->merge_a.upload(b->whole.merge_a, stream);
    b->merge_b.upload(b->whole.merge_b, stream);
    b->cvbuf.ensure((size_t)b->whole.n_cv * 32);
    b->cv2.ensure((size_t)b->whole.n_cv2 * 32);
    if (b->n_long) {
        plan_checksum_batch(&b->lng, loff.data(), llen.data(), b->n_long, stream);
        b->compressions += b->lng.plan.compressions;
        b->long_idx.upload(b->h_long_idx, stream);
        b->long_out.ensure((size_t)b->n_long * 32);
    }
}

void run_cas_batch(const sd_cas_batch* b, const uint8_t* d_staged, uint8_t* d_hash32, hipStream_t s,
                   int parts = SD_PART_SAMPLED | SD_PART_WHOLE) {
    uint32_t* out = reinterpret_cast<uint32_t*>(d_hash32);
    if (parts & SD_PART_SAMPLED)
        HIP_CHECK(sdk::launch_cas_sampled(d_staged, b->soff.as<uint64_t>(), b->sidx.as<uint32_t>(), b->n_sampled, out,
                                          s));
    if (parts & SD_PART_WHOLE) {
        const WholePlan& w = b->whole;
        HIP_CHECK(sdk::launch_whole_items(d_staged, b->full_items.as<uint4>(), (uint32_t)w.full.size(),
                                          b->tail_items.as<uint4>(), (uint32_t)w.tail.size(), b->merge_a.as<uint4>(),
                                          (uint32_t)w.merge_a.size(), b->merge_b.as<uint4>(),
                                          (uint32_t)w.merge_b.size(), b->cvbuf.as<uint32_t>(),
                                          b->cv2.as<uint32_t>(), out, s));
        if (b->n_long) {
            run_checksum_batch(&b->lng, d_staged, b->long_out.as<uint8_t>(), s);
            HIP_CHECK(sdk::launch_scatter_hash(b->long_out.as<uint32_t>(), b->long_idx.as<uint32_t>(), b->n_long, out,
                                               s));
        }
    }
}

// ------------------------------------------------------- streaming (unknown length)
// Hashes messages read front to back from a MsgSource through 256 MiB windows on the two
// alternating slots.  A message's length is only known when its source ends, which is all
// the 1 MiB-block tree needs: a full window (more than 1 MiB) holds 256 complete, non-final
// blocks whose subtree CVs do not depend on the total, so they are hashed as the windows
// arrive (a provisional one-message table of unbounded length); the final window then runs
// with the message's real length, and the reduce passes merge all block CVs.
//
// Nothing waits for a message to finish: its final window, reduce and the 32-byte D2H are
// queued on one slot's stream (after an event wait on the other slot's last window of the
// same message), and the hash is handed to `done(tag, h32)` the next time that stream is
// synchronised -- by the Streamer itself before it reuses the slot's window, by the
// caller's collect(), or by finish().  So the host reads the next file while the GPU
// finishes the last one.  Two per-message plans alternate; a plan is rebuilt only after
// the events of the message that last used it have completed.
struct Streamer {
    static constexpr uint64_t W = 256ull << 20;  // a multiple of the 1 MiB leaf block
    static constexpr uint32_t BPW = (uint32_t)(W / SD_CK_BLOCK);
    static constexpr size_t RING = 16;  // results queued per slot between two syncs of it
    using Done = std::function<void(size_t tag, const uint8_t* h32)>;

    struct Msg {
        sd_checksum_batch fin;  // the final plan: one message of the final length
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool used[2] = {false, false};  // ev[k] recorded since the plan was last rebuilt
    };
    Msg msg[2];
    int next_msg = 0;
    DevBuf prov_files, prov_map;  // full windows: {0, 2^62, 0} and (0, b) for b < BPW
    bool prov_ready = false;
    DevBuf rdev[2];
    PinnedBuf rhost[2];
    std::vector<size_t> rtag[2];
    Done done;

    explicit Streamer(Done d) : done(std::move(d)) {}
    Streamer(const Streamer&) = delete;
    Streamer& operator=(const Streamer&) = delete;
    ~Streamer() {
        for (auto& m : msg)
            for (auto& e : m.ev)
                if (e) (void)hipEventDestroy(e);
    }

    static void prepare(SlotPair& sl) {
        for (int k = 0; k < 2; k++) {
            sl[k].window.ensure(W + 128);
            sl[k].staged.ensure(W + 128);
            sl[k].hashes.ensure(32);
            sl[k].host_hashes.ensure(32);
        }
    }
    // Hands over the hashes queued on slot k.  The caller has synchronised its stream.
    void collect(int k) {
        for (size_t q = 0; q < rtag[k].size(); q++) done(rtag[k][q], rhost[k].u8() + 32 * q);
        rtag[k].clear();
    }
    void sync_collect(SlotPair& sl, int k) {
        HIP_CHECK(hipStreamSynchronize(sl[k].stream));
        collect(k);
    }
    void finish(SlotPair& sl) {
        sync_collect(sl, 0);
        sync_collect(sl, 1);
    }
    void record(Msg& m, SlotPair& sl, int k) {
        if (!m.ev[k]) HIP_CHECK(hipEventCreateWithFlags(&m.ev[k], hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(m.ev[k], sl[k].stream));
        m.used[k] = true;
    }
    void wait_idle(Msg& m) {  // every launch of the message that last used this plan is done
        for (int k = 0; k < 2; k++)
            if (m.used[k]) {
                HIP_CHECK(hipEventSynchronize(m.ev[k]));
                m.used[k] = false;
            }
    }

    // Queues the hash of one message; SD_FILE_OK means done(tag, ...) will follow, anything
    // else is the source's I/O status (no result for this tag).
    int32_t hash_async(SlotPair& sl, int& cur, MsgSource& src, uint64_t size_hint, size_t tag) {
        prepare(sl);
        if (!prov_ready) {
            std::vector<ck_file> f{ck_file{0, 1ull << 62, 0}};
            std::vector<sd_u32x2> mp(BPW);
            for (uint32_t b = 0; b < BPW; b++) mp[b] = sd_u32x2{0, b};
            prov_files.upload(f);
            prov_map.upload(mp);
            for (int k = 0; k < 2; k++) {
                rdev[k].ensure(RING * 32);
                rhost[k].ensure(RING * 32);
            }
            prov_ready = true;
        }
        Msg& m = msg[next_msg];
        next_msg ^= 1;
        wait_idle(m);
        sd_checksum_batch& fin = m.fin;
        const uint64_t cap0 = (uint64_t)std::max<uint64_t>(size_hint / SD_CK_BLOCK + 2, 2 * BPW) * 32;
        if (cap0 > fin.lvl[0].bytes) fin.lvl[0].grow_preserve(cap0);  // nothing of this plan in flight
        uint64_t pos = 0;
        for (;;) {
            const int k = cur;
            cur ^= 1;
            sync_collect(sl, k);  // its window is free again
            uint8_t* win = sl[k].window.u8();
            const uint64_t got = src.read(win, W);
            if (src.err) return io_status(src.err);
            if (got == W && !src.done) {  // a full window with more to come
                const uint32_t blk0 = (uint32_t)(pos / SD_CK_BLOCK);
                if ((uint64_t)(blk0 + BPW) * 32 > fin.lvl[0].bytes) {
                    sl.sync_all();  // both slots may hold windows of this message
                    fin.lvl[0].grow_preserve((size_t)(blk0 + BPW) * 64);
                }
                HIP_CHECK(hipMemcpyAsync(sl[k].staged.p, win, W, hipMemcpyHostToDevice, sl[k].stream));
                HIP_CHECK(sdk::launch_ck_leaf(sl[k].staged.as<uint8_t>(), pos, blk0, prov_files.as<ck_file>(),
                                              prov_map.as<uint2>(), BPW, fin.lvl[0].as<uint32_t>(),
                                              sl[k].hashes.as<uint32_t>(), sl[k].stream));
                record(m, sl, k);
                pos += W;
                continue;
            }
            const uint64_t L = pos + got;
            const uint64_t nb = L == 0 ? 1 : (L + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
            if (nb * 32 > fin.lvl[0].bytes) {  // grew past the hint: keep the CVs
                sl.sync_all();
                fin.lvl[0].grow_preserve((size_t)nb * 32);
            }
            if (m.used[k ^ 1]) HIP_CHECK(hipStreamWaitEvent(sl[k].stream, m.ev[k ^ 1], 0));  // its windows first
            const uint64_t off0 = 0;
            // async uploads from fin's host tables: they stay valid until wait_idle(m)
            plan_checksum_batch(&fin, &off0, &L, 1, sl[k].stream);
            if (rtag[k].size() == RING) sync_collect(sl, k);
            const size_t q = rtag[k].size();
            uint32_t* out = rdev[k].as<uint32_t>() + 8 * q;
            if (got > 0 || L == 0) {
                memset(win + got, 0, 64);
                HIP_CHECK(hipMemcpyAsync(sl[k].staged.p, win, align_up(got, 64) + 64, hipMemcpyHostToDevice,
                                         sl[k].stream));
                const uint32_t wg0 = (uint32_t)(pos / SD_CK_BLOCK);
                HIP_CHECK(sdk::launch_ck_leaf(sl[k].staged.as<uint8_t>(), pos, 0, fin.files.as<ck_file>(),
                                              fin.wg_map.as<uint2>() + wg0, (uint32_t)(nb - wg0),
                                              fin.lvl[0].as<uint32_t>(), out, sl[k].stream));
            }
            run_checksum_reduce(&fin, out, sl[k].stream);
            HIP_CHECK(hipMemcpyAsync(rhost[k].u8() + 32 * q, out, 32, hipMemcpyDeviceToHost, sl[k].stream));
            record(m, sl, k);
            rtag[k].push_back(tag);
            return SD_FILE_OK;
        }
    }

    // One message, waited for (the rare paths: cas messages that outgrew their extent).
    int32_t hash(SlotPair& sl, int& cur, MsgSource& src, uint64_t size_hint, uint8_t out32[32]) {
        finish(sl);  // earlier messages' results go to their own callback
        Done keep = std::move(done);
        done = [&](size_t, const uint8_t* h) { memcpy(out32, h, 32); };
        int32_t rc;
        try {
            rc = hash_async(sl, cur, src, size_hint, 0);
            finish(sl);
        } catch (...) {
            done = std::move(keep);
            throw;
        }
        done = std::move(keep);
        return rc;
    }
};

inline void to_hex(const uint8_t* h, int nbytes, char* out) { hex_lower(h, nbytes, out); }

// Hashes (GPU, streaming) the whole-file cas message of a file that held more bytes than
// its staged extent could take: le64(size) || every byte fs::read returns (cas.rs:25,29).
int32_t cas_overflow(SlotPair& sl, int& cur, Streamer& st, const char* path, uint64_t size, uint8_t out32[32]) {
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return io_status(errno);
    MsgSource src(fd, MsgSource::READ_TO_EOF);
    src.set_prefix_le64(size);
    int32_t rc;
    try {
        rc = st.hash(sl, cur, src, size + 8, out32);
    } catch (...) {
        close(fd);
        throw;
    }
    close(fd);
    return rc;
}

}  // namespace

int sd_ctx_device(const sd_cas_ctx* ctx) { return ctx->device; }
const SplitPlan& sd_split_plan_of(const sd_split_checksum* x) { return x->sp; }

// Grouping, and (owner_chunk > 0) the Object rule on its output, with one host sync: with
// the LDS-bucket grouping the owners kernel is queued right behind it, before the sync that
// reads the group count and the overflow flag; on an overflow both run again on the radix
// path.  Throws sd_failure.
void dedup_group_owners(sd_cas_ctx* ctx, uint64_t* d_records, uint64_t m, int flags, uint64_t* d_rep,
                        uint64_t owner_chunk, uint64_t* d_owner, uint64_t* n_groups, hipStream_t s) {
    ctx->bind();
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
        if (owner_chunk) HIP_CHECK(sdk::dedup_owners(d_records, m, d_rep, owner_chunk, d_owner, s));  // speculative
        HIP_CHECK(hipStreamSynchronize(s));
        const uint64_t* st = reinterpret_cast<const uint64_t*>(slot->host_hashes.p);
        if (st[1] == 0) {
            *n_groups = st[0];
            return;
        }
        flags &= ~SD_DEDUP_INDEX_SORTED;  // a bucket overflowed: d_records is now a permutation
    }
    HIP_CHECK(sdk::dedup_group(d_records, m, flags, d_rep, slot->hashes.as<uint64_t>(), slot->staged.p, &have, s));
    HIP_CHECK(hipMemcpyAsync(slot->host_hashes.p, slot->hashes.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if (owner_chunk) HIP_CHECK(sdk::dedup_owners(d_records, m, d_rep, owner_chunk, d_owner, s));
    HIP_CHECK(hipStreamSynchronize(s));
    *n_groups = *reinterpret_cast<uint64_t*>(slot->host_hashes.p);
}

// ============================================================================ C ABI
extern "C" {

int sd_cas_ctx_create(int device, sd_cas_ctx** out) {
    SD_GUARD_BEGIN
    if (!out) throw sd_failure(SD_ERR_INVALID, "out is null");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        throw sd_failure(SD_ERR_DEVICE, "no HIP device available (the sd_cpu_* entry points need none)");
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
        extents_out[i] = plan_extent(sizes[i], off);
        off = align_up(off + extents_out[i].msg_len, SD_STAGE_ALIGN);
    }
    *total_bytes_out = off;
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_stage_file(const char* path, sd_extent* ext, uint8_t* staged, int32_t* status) {
    SD_GUARD_BEGIN
    if (!path || !ext || !staged || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    validate_extent(*ext, 0);
    *status = stage_one(path, *ext, staged);
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_stage_files(const char* const* paths, sd_extent* extents, size_t n, uint8_t* staged, int32_t* status,
                       int nthreads) {
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
    auto b = std::make_unique<sd_cas_batch>();
    plan_cas_batch(b.get(), extents, n, nullptr);
    *out = b.release();
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

int sd_cas_batch_stats(const sd_cas_batch* b, uint64_t out[8]) {
    SD_GUARD_BEGIN
    if (!b || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = b->n; out[1] = b->n_sampled; out[2] = b->n_whole + b->n_long; out[3] = b->whole_chunks;
    out[4] = b->compressions; out[5] = b->msg_bytes;
    out[6] = b->whole.full.size(); out[7] = b->whole.tail.size();
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
    SlotPair slots(ctx);
    sd_cas_batch batches[2];
    Win wins[2];
    auto harvest = [&](int k) {
        if (!wins[k].busy) return;
        HIP_CHECK(hipStreamSynchronize(slots[k].stream));
        const uint8_t* h = slots[k].host_hashes.u8();
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
        Slot& sl = slots[w];
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
// the stager pool reads window k+1 into one pinned slot while window k's H2D copy,
// kernels and D2H run on the other slot's stream.  A whole-kind file that turns out
// longer than its planned extent (it grew since the caller's stat) is hashed afterwards
// from the file itself, streamed (fs::read hashes every byte, cas.rs:29).
namespace {
// The body of sd_cas_ids_files (hex to host memory) and sd_cas_hashes_files (the 32-byte
// hashes to device memory, for the multi-GPU dedup): out_hex17 xor d_hash32.
void cas_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n, char* out_hex17,
               uint8_t* d_hash32, int32_t* status, int nthreads) {
    ctx->bind();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    // nthreads reader threads stage in the background (start/wait) while this thread plans,
    // launches and harvests the windows
    std::shared_ptr<StagePool> pool = ctx->stage_pool(nthreads + 1);
    const uint64_t WINDOW = (uint64_t)std::max(1, tuning_get(SD_TUNE_FILES_WINDOW_MB)) << 20;
    SlotPair slots(ctx);
    sd_cas_batch batches[2];
    struct Win {  // the window being staged into a slot's pinned buffer
        std::vector<sd_extent> ext;
        std::vector<size_t> idx;                // input index of each extent
        std::vector<std::vector<uint8_t>> cap;  // a pipe's / device's whole content (stage_one)
        uint64_t bytes = 0;
    } wins[2];
    struct Launched {  // the window in flight on a slot's stream
        std::vector<size_t> files;  // hashed files, in extent order
        bool busy = false;
    } launched[2];
    hipEvent_t copied[2] = {nullptr, nullptr};  // the slot's pinned buffer has been read by its H2D
    bool copy_pending[2] = {false, false};
    struct Cleanup {  // on any exit: no reader left writing, no event leaked
        StagePool* pool;
        bool staging = false;
        hipEvent_t* ev;
        ~Cleanup() {
            if (staging) pool->wait();
            for (int k = 0; k < 2; k++)
                if (ev[k]) (void)hipEventDestroy(ev[k]);
        }
    } cleanup{pool.get(), false, copied};
    for (int k = 0; k < 2; k++) HIP_CHECK(hipEventCreateWithFlags(&copied[k], hipEventDisableTiming));
    auto harvest = [&](int k) {
        if (!launched[k].busy) return;
        HIP_CHECK(hipStreamSynchronize(slots[k].stream));
        const uint8_t* h = slots[k].host_hashes.u8();
        if (out_hex17)
            for (size_t q = 0; q < launched[k].files.size(); q++)
                to_hex(h + q * 32, 8, out_hex17 + launched[k].files[q] * 17);  // cas.rs:61 to_hex()[..16]
        launched[k].busy = false;
    };
    DevBuf dev_idx[2];                          // device output: the launched window's file rows
    std::vector<uint32_t> dev_idx_h[2];         // (their host copies, alive until the harvest)
    auto put_hash = [&](size_t f, const uint8_t h[32]) {  // a hash computed off the windows
        if (out_hex17) to_hex(h, 8, out_hex17 + f * 17);       // cas.rs:61 to_hex()[..16]
        else HIP_CHECK(hipMemcpy(d_hash32 + 32 * f, h, 32, hipMemcpyHostToDevice));
    };
    std::vector<size_t> overflow;                                      // regular files that grew
    std::vector<std::pair<size_t, std::vector<uint8_t>>> captured;    // pipes / devices, read whole
    size_t i = 0;
    // plans the next window (consecutive files whose messages fit WINDOW bytes) into slot w
    // and starts the readers on it; false when no files are left
    auto begin_window = [&](int w) -> bool {
        if (i >= n) return false;
        Win& W = wins[w];
        W.ext.clear();
        W.idx.clear();
        uint64_t off = 0;
        while (i < n) {
            const sd_extent e = plan_extent(sizes[i], off);
            const uint64_t next = align_up(off + e.msg_len, SD_STAGE_ALIGN);
            if (!W.ext.empty() && next > WINDOW) break;
            W.ext.push_back(e);
            W.idx.push_back(i);
            off = next;
            i++;
        }
        W.bytes = off;
        W.cap.assign(W.ext.size(), {});
        if (copy_pending[w]) {  // the slot's last H2D must have read its buffer
            HIP_CHECK(hipEventSynchronize(copied[w]));
            copy_pending[w] = false;
        }
        if (slots[w].window.bytes < off + 64) {
            harvest(w);  // a reallocation frees the buffer: nothing may still use it
            slots[w].window.ensure(off + 64);
        }
        uint8_t* win = slots[w].window.u8();
        pool->start(W.ext.size(), [&W, win, paths, status](size_t q) {
            status[W.idx[q]] = stage_one(paths[W.idx[q]], W.ext[q], win, &W.cap[q]);
        });
        cleanup.staging = true;
        return true;
    };
    int w = 0;
    bool staging = begin_window(w);
    while (staging) {
        pool->wait();  // window w is staged
        cleanup.staging = false;
        Win& W = wins[w];
        Slot& sl = slots[w];
        // failed files (I/O error, short read) keep their status and leave the window;
        // files longer than their extent are hashed from disk after the windows
        size_t m = 0;
        for (size_t q = 0; q < W.ext.size(); q++) {
            if (status[W.idx[q]] == SD_FILE_OK) {
                W.ext[m] = W.ext[q];
                W.idx[m++] = W.idx[q];
            } else if (status[W.idx[q]] == SD_FILE_CHANGED) {
                if (W.cap[q].empty()) overflow.push_back(W.idx[q]);
                else captured.emplace_back(W.idx[q], std::move(W.cap[q]));
            }
        }
        W.ext.resize(m);
        W.idx.resize(m);
        const int next = w ^ 1;
        staging = begin_window(next);  // the readers go on with the next window...
        if (m) {                        // ...while this one is planned and launched
            harvest(w);                 // slot w's previous launch (two windows back)
            plan_cas_batch(&batches[w], W.ext.data(), m, sl.stream);
            sl.staged.ensure(W.bytes + 64);
            sl.hashes.ensure(m * 32);
            sl.host_hashes.ensure(m * 32);
            HIP_CHECK(hipMemcpyAsync(sl.staged.p, sl.window.p, W.bytes, hipMemcpyHostToDevice, sl.stream));
            HIP_CHECK(hipEventRecord(copied[w], sl.stream));
            copy_pending[w] = true;
            run_cas_batch(&batches[w], sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
            if (d_hash32) {  // device output: the window's hashes scattered to their files' rows
                dev_idx_h[w].assign(W.idx.begin(), W.idx.end());
                dev_idx[w].upload(dev_idx_h[w], sl.stream);
                HIP_CHECK(sdk::launch_scatter_hash(sl.hashes.as<uint32_t>(), dev_idx[w].as<uint32_t>(), (uint32_t)m,
                                                   reinterpret_cast<uint32_t*>(d_hash32), sl.stream));
            } else {
                HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, m * 32, hipMemcpyDeviceToHost, sl.stream));
            }
            launched[w].files = W.idx;
            launched[w].busy = true;
        }
        w = next;
    }
    harvest(0);
    harvest(1);
    if (!overflow.empty() || !captured.empty()) {
        Streamer st([](size_t, const uint8_t*) {});
        int cur = 0;
        for (size_t f : overflow) {
            uint8_t h[32];
            status[f] = cas_overflow(slots, cur, st, paths[f], sizes[f], h);
            if (status[f] == SD_FILE_OK) put_hash(f, h);
        }
        for (auto& c : captured) {  // le64(size) || every byte the pipe gave (cas.rs:25,29)
            MsgSource src(-1, MsgSource::READ_TO_EOF);
            src.set_prefix_le64(sizes[c.first]);
            src.set_memory(c.second.data(), c.second.size());
            uint8_t h[32];
            status[c.first] = st.hash(slots, cur, src, c.second.size() + 8, h);
            if (status[c.first] == SD_FILE_OK) put_hash(c.first, h);
        }
    }
}
}  // namespace

int sd_cas_ids_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n, char* out_hex17,
                     int32_t* status, int nthreads) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!paths || !sizes || !out_hex17 || !status))) throw sd_failure(SD_ERR_INVALID, "null argument");
    cas_files(ctx, paths, sizes, n, out_hex17, nullptr, status, nthreads);
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_hashes_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n,
                        uint8_t* d_hash32, uint8_t* d_valid, int32_t* status, int nthreads) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!paths || !sizes || !d_hash32 || !status))) throw sd_failure(SD_ERR_INVALID, "null argument");
    cas_files(ctx, paths, sizes, n, nullptr, d_hash32, status, nthreads);
    if (d_valid && n) {  // the records sd_cas_dedup_mgpu takes: hashed, and not empty (mod.rs:80-88)
        std::vector<uint8_t> v(n);
        for (size_t i = 0; i < n; i++) v[i] = status[i] == SD_FILE_OK && sizes[i] != 0;
        HIP_CHECK(hipMemcpy(d_valid, v.data(), n, hipMemcpyHostToDevice));
    }
    return SD_OK;
    SD_GUARD_END
}

// ------------------------------------------------------------------- latency path
int sd_cas_id_path(sd_cas_ctx* ctx, const char* path, uint64_t size, char* out_hex17, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || !path || !out_hex17 || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    std::string err;
    const int rc = coalescer_submit(ctx->coalescer(), 0, path, size, out_hex17, status, &err);
    if (rc != SD_OK) sd_set_err("%s", err.c_str());
    return rc;
    SD_GUARD_END
}

int sd_file_checksum_path(sd_cas_ctx* ctx, const char* path, char* out_hex65, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || !path || !out_hex65 || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    std::string err;
    const int rc = coalescer_submit(ctx->coalescer(), 1, path, 0, out_hex65, status, &err);
    if (rc != SD_OK) sd_set_err("%s", err.c_str());
    return rc;
    SD_GUARD_END
}

int sd_coalescer_stats(sd_cas_ctx* ctx, uint64_t out[4]) {
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
    auto b = std::make_unique<sd_checksum_batch>();
    plan_checksum_batch(b.get(), offsets, lens, n, nullptr);
    *out = b.release();
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
    out[0] = b->n; out[1] = b->plan.total_bytes; out[2] = b->plan.compressions; out[3] = b->plan.blocks;
    return SD_OK;
    SD_GUARD_END
}

// ------------------------------------------------------------ one file over many GPUs
int sd_split_checksum_create(sd_cas_ctx* ctx, uint64_t total_len, int nranks, int rank, sd_split_checksum** out) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    *out = nullptr;
    ctx->bind();
    auto x = std::make_unique<sd_split_checksum>();
    x->sp = split_plan(total_len, nranks, rank);
    const uint64_t off0 = 0;
    plan_checksum_batch(&x->plan, &off0, &total_len, 1, nullptr);
    *out = x.release();
    return SD_OK;
    SD_GUARD_END
}

void sd_split_checksum_destroy(sd_split_checksum* x) {
    try {
        delete x;
    } catch (...) {
    }
}

// k_ck_leaf over this rank's blocks of the one-message plan: the slice holds message bytes
// [off, off + len) (shift = off), block b's CV lands in d_cvs slot b (cv_base 0); a
// one-block file writes its root hash to `out` = slot 0.
int sd_split_checksum_leaves(sd_cas_ctx* ctx, const sd_split_checksum* x, const uint8_t* d_slice, uint8_t* d_cvs,
                             void* stream) {
    SD_GUARD_BEGIN
    const SplitPlan& p = x ? x->sp : SplitPlan{};
    if (!ctx || !x || !d_cvs || (p.b1 > p.b0 && !d_slice)) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (p.b1 > p.b0 && reinterpret_cast<uintptr_t>(d_slice) % 16)
        throw sd_failure(SD_ERR_INVALID, "d_slice not 16-byte aligned");
    ctx->bind();
    if (p.b1 > p.b0) {  // a rank past the last block holds nothing
        uint32_t* cvs = reinterpret_cast<uint32_t*>(d_cvs);
        HIP_CHECK(sdk::launch_ck_leaf(d_slice, p.off, 0, x->plan.files.as<ck_file>(),
                                      x->plan.wg_map.as<uint2>() + p.b0, (uint32_t)(p.b1 - p.b0), cvs, cvs,
                                      ctx->pick(stream)));
    }
    return SD_OK;
    SD_GUARD_END
}

int sd_split_checksum_root(sd_cas_ctx* ctx, sd_split_checksum* x, const uint8_t* d_cvs, uint8_t* d_hash32,
                           void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !x || !d_cvs || !d_hash32) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    hipStream_t s = ctx->pick(stream);
    if (x->sp.nb == 1) {
        HIP_CHECK(hipMemcpyAsync(d_hash32, d_cvs, 32, hipMemcpyDeviceToDevice, s));
    } else {
        HIP_CHECK(hipMemcpyAsync(x->plan.lvl[0].p, d_cvs, x->sp.nb * 32, hipMemcpyDeviceToDevice, s));
        run_checksum_reduce(&x->plan, reinterpret_cast<uint32_t*>(d_hash32), s);
    }
    return SD_OK;
    SD_GUARD_END
}

// file_checksum (hash.rs:10-24) for n paths.  Each file is read as the reference reads it:
// hash.rs's 1 MiB read calls until one returns fewer.  For a regular file those reads are
// exactly its bytes up to EOF, so regular files are read with parallel preads on the
// context's stager pool ("read_threads"); anything else (a pipe, a device) with the
// literal sequential loop.  Small regular files are packed (64-B aligned) into the current
// slot's pinned window by their stat length -- one batch per window, read in parallel,
// each file probed past its length in case it grew --; while the GPU hashes one slot's
// window the host reads the next into the other.  Larger files, files that grew, and
// non-regular files stream window by window (Streamer), whatever their final length.
int sd_file_checksums(sd_cas_ctx* ctx, const char* const* paths, size_t n, char* out_hex65, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!paths || !out_hex65 || !status))) throw sd_failure(SD_ERR_INVALID, "null argument");
    ctx->bind();
    constexpr uint64_t W = Streamer::W;
    std::shared_ptr<StagePool> pool = ctx->stage_pool(std::max(1, std::min(64, tuning_get(SD_TUNE_READ_THREADS))));
    SlotPair slots(ctx);
    Streamer::prepare(slots);
    // stat every file in parallel: its length picks the route (regular files only)
    std::vector<uint64_t> hint(n, 0);
    std::vector<uint8_t> regular(n, 0);
    pool->run(n, [&](size_t i) {
        struct stat st;
        if (stat(paths[i], &st) == 0 && S_ISREG(st.st_mode)) {
            hint[i] = (uint64_t)st.st_size;
            regular[i] = 1;
        }
    });
    struct Pending {
        std::vector<size_t> files;  // files whose hashes land in this slot's host_hashes
        bool busy = false;
    } pend[2];
    sd_checksum_batch pack_batch[2];
    // streamed files' hashes arrive when their slot is next synchronised
    Streamer streamer([&](size_t i, const uint8_t* h) { to_hex(h, 32, out_hex65 + i * 65); });  // hash.rs:21-23
    int cur = 0;
    auto harvest = [&](int k) {  // slot k idle: its window is free, its results delivered
        HIP_CHECK(hipStreamSynchronize(slots[k].stream));
        streamer.collect(k);
        if (!pend[k].busy) return;
        const uint8_t* h = slots[k].host_hashes.u8();
        for (size_t q = 0; q < pend[k].files.size(); q++)
            to_hex(h + 32 * q, 32, out_hex65 + pend[k].files[q] * 65);  // hash.rs:21-23
        pend[k].files.clear();
        pend[k].busy = false;
    };
    // one file streamed (sequential reads, or parallel preads for a regular file); its hash
    // lands in out_hex65 through the streamer's callback, at a later sync of its slot
    auto stream_file = [&](size_t i) {
        const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);  // hash.rs:11
        if (fd < 0) {
            status[i] = io_status(errno);
            return;
        }
        struct stat st;
        const bool reg = fstat(fd, &st) == 0 && S_ISREG(st.st_mode);
        MsgSource src(fd, MsgSource::CHECKSUM_READS);
        if (reg) {
            src.set_parallel(pool.get());
            src.set_eof_hint((uint64_t)st.st_size);  // a window-multiple file ends with its last window
        }
        try {
            status[i] = streamer.hash_async(slots, cur, src, reg ? (uint64_t)st.st_size : 0, i);
        } catch (...) {
            close(fd);
            throw;
        }
        close(fd);
    };
    // the pack: regular files laid out by their stat lengths in slot `cur`'s window
    std::vector<size_t> pack, grew;
    std::vector<uint64_t> pack_off, pack_len;
    uint64_t pack_end = 0;
    auto submit_pack = [&]() {
        if (pack.empty()) return;
        const int k = cur;
        harvest(k);  // slot k's previous batch is done: its window is free
        Slot& sl = slots[k];
        uint8_t* win = sl.window.u8();
        pool->run(pack.size(), [&](size_t q) {
            const size_t i = pack[q];
            const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
            if (fd < 0) {
                status[i] = io_status(errno);
                return;
            }
            const int64_t got = pread_full(fd, win + pack_off[q], hint[i], 0);
            uint8_t probe;
            const int64_t more = got == (int64_t)hint[i] ? pread_full(fd, &probe, 1, hint[i]) : 0;
            close(fd);
            if (got < 0 || more < 0) {
                status[i] = io_status((int)-(got < 0 ? got : more));
            } else if (more > 0) {
                status[i] = SD_FILE_CHANGED;  // grew since stat: stream it below
            } else {
                status[i] = SD_FILE_OK;
                pack_len[q] = (uint64_t)got;  // shrank: hash.rs stops at EOF
                memset(win + pack_off[q] + got, 0, align_up(got, 64) - got);
            }
        });
        std::vector<uint64_t> offs, lens;
        std::vector<size_t> ok;
        for (size_t q = 0; q < pack.size(); q++) {
            if (status[pack[q]] == SD_FILE_OK) {
                ok.push_back(pack[q]);
                offs.push_back(pack_off[q]);
                lens.push_back(pack_len[q]);
            } else if (status[pack[q]] == SD_FILE_CHANGED) {
                grew.push_back(pack[q]);
            }
        }
        pack.clear();
        pack_off.clear();
        pack_len.clear();
        const uint64_t span = pack_end;
        pack_end = 0;
        if (ok.empty()) return;
        cur ^= 1;
        plan_checksum_batch(&pack_batch[k], offs.data(), lens.data(), ok.size(), sl.stream);
        sl.hashes.ensure(ok.size() * 32);
        sl.host_hashes.ensure(ok.size() * 32);
        HIP_CHECK(hipMemcpyAsync(sl.staged.p, win, span + 64, hipMemcpyHostToDevice, sl.stream));
        run_checksum_batch(&pack_batch[k], sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, ok.size() * 32, hipMemcpyDeviceToHost, sl.stream));
        pend[k].files = std::move(ok);
        pend[k].busy = true;
    };
    for (size_t i = 0; i < n; i++) {
        status[i] = SD_FILE_OK;
        if (!regular[i] || hint[i] + 128 > W / 2) {  // a pipe / device / unreadable path, or large
            submit_pack();
            stream_file(i);
            continue;
        }
        if (pack_end + align_up(hint[i], 64) + 64 > W) submit_pack();
        pack.push_back(i);
        pack_off.push_back(pack_end);
        pack_len.push_back(hint[i]);
        pack_end = align_up(pack_end + hint[i], 64);
    }
    submit_pack();
    for (size_t i : grew) {
        status[i] = SD_FILE_OK;
        stream_file(i);
    }
    harvest(0);
    harvest(1);
    streamer.finish(slots);
    return SD_OK;
    SD_GUARD_END
}

// Full BLAKE3 of n byte ranges of a host buffer (hash.rs:10-24 on data already in memory):
// consecutive ranges whose span fits a 256 MiB window are copied with one H2D each and
// hashed as one batch; a larger range streams window by window into its leaf CVs (known
// length: one plan), then reduces.  Two slots alternate so copies overlap kernels.
int sd_checksums(sd_cas_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, size_t n,
                 char* out_hex65) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!data || !offsets || !lens || !out_hex65))) throw sd_failure(SD_ERR_INVALID, "null argument");
    for (size_t i = 0; i < n; i++)
        if (offsets[i] % 16) throw sd_failure(SD_ERR_INVALID, "range " + std::to_string(i) + " not 16-byte aligned");
    ctx->bind();
    constexpr uint64_t W = Streamer::W;
    SlotPair slots(ctx);
    Streamer::prepare(slots);
    sd_checksum_batch batches[2], big;
    struct Pending {
        size_t i0 = 0, i1 = 0;
        bool busy = false;
    } pend[2];
    auto harvest = [&](int k) {
        if (!pend[k].busy) return;
        HIP_CHECK(hipStreamSynchronize(slots[k].stream));
        const uint8_t* h = slots[k].host_hashes.u8();
        for (size_t i = pend[k].i0; i < pend[k].i1; i++) to_hex(h + 32 * (i - pend[k].i0), 32, out_hex65 + 65 * i);
        pend[k].busy = false;
    };
    // copies on one queue (copy_stream), kernels on the two slots' streams, joined by events:
    // copied[k] = slot k's window has landed; used[k] = slot k's kernels no longer read it
    hipStream_t cs = slots.copy_stream();
    hipEvent_t copied[2] = {nullptr, nullptr}, used[2] = {nullptr, nullptr};
    bool used_set[2] = {false, false};
    struct Events {
        hipEvent_t* e[2];
        ~Events() {
            for (auto* p : e)
                for (int k = 0; k < 2; k++)
                    if (p[k]) (void)hipEventDestroy(p[k]);
        }
    } ev_guard{{copied, used}};
    for (int k = 0; k < 2; k++) {
        HIP_CHECK(hipEventCreateWithFlags(&copied[k], hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&used[k], hipEventDisableTiming));
    }
    // H2D of `bytes` from `src` into slot k's device window, after its previous kernels
    auto copy_in = [&](int k, const uint8_t* src, uint64_t bytes) {
        if (used_set[k]) HIP_CHECK(hipStreamWaitEvent(cs, used[k], 0));
        HIP_CHECK(hipMemcpyAsync(slots[k].staged.p, src, bytes, hipMemcpyHostToDevice, cs));
        HIP_CHECK(hipEventRecord(copied[k], cs));
        HIP_CHECK(hipStreamWaitEvent(slots[k].stream, copied[k], 0));
    };
    auto done_with = [&](int k) {
        HIP_CHECK(hipEventRecord(used[k], slots[k].stream));
        used_set[k] = true;
    };
    int cur = 0;
    std::vector<uint64_t> offs, ls;
    for (size_t i = 0; i < n;) {
        if (lens[i] + 128 > W) {  // one large range, streamed
            harvest(0);
            harvest(1);
            const uint64_t off0 = 0, L = lens[i];
            plan_checksum_batch(&big, &off0, &L, 1, nullptr);
            const uint64_t nb = big.plan.wg_map.size();
            for (uint64_t pos = 0; pos < L; pos += W) {
                const int k = cur;
                cur ^= 1;
                const uint64_t here = std::min<uint64_t>(W, L - pos);
                copy_in(k, data + offsets[i] + pos, align_up(here, 64));
                const uint32_t wg0 = (uint32_t)(pos / SD_CK_BLOCK);
                const uint32_t wg1 = (uint32_t)std::min<uint64_t>(nb, wg0 + W / SD_CK_BLOCK);
                HIP_CHECK(sdk::launch_ck_leaf(slots[k].staged.as<uint8_t>(), pos, 0, big.files.as<ck_file>(),
                                              big.wg_map.as<uint2>() + wg0, wg1 - wg0, big.lvl[0].as<uint32_t>(),
                                              slots[k].hashes.as<uint32_t>(), slots[k].stream));
                done_with(k);
            }
            slots.sync_all();
            Slot& sl = slots[0];
            run_checksum_reduce(&big, sl.hashes.as<uint32_t>(), sl.stream);
            HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, 32, hipMemcpyDeviceToHost, sl.stream));
            HIP_CHECK(hipStreamSynchronize(sl.stream));
            to_hex(sl.host_hashes.u8(), 32, out_hex65 + 65 * i);
            i++;
            continue;
        }
        // the next window: consecutive ranges whose span fits
        const uint64_t lo = offsets[i] / 16 * 16;
        uint64_t hi = 0;
        size_t j = i;
        while (j < n && lens[j] + 128 <= W) {
            const uint64_t nlo = std::min(lo, offsets[j] / 16 * 16);
            const uint64_t nhi = std::max(hi, align_up(offsets[j] + lens[j], 64));
            if (j > i && (nlo < lo || nhi - lo > W)) break;
            hi = nhi;
            j++;
        }
        const int k = cur;
        cur ^= 1;
        harvest(k);
        Slot& sl = slots[k];
        offs.assign(offsets + i, offsets + j);
        ls.assign(lens + i, lens + j);
        for (auto& o : offs) o -= lo;
        plan_checksum_batch(&batches[k], offs.data(), ls.data(), j - i, sl.stream);
        sl.hashes.ensure((j - i) * 32);
        sl.host_hashes.ensure((j - i) * 32);
        copy_in(k, data + lo, std::max<uint64_t>(hi - lo, 16));
        run_checksum_batch(&batches[k], sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        done_with(k);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, (j - i) * 32, hipMemcpyDeviceToHost, sl.stream));
        pend[k] = Pending{i, j, true};
        i = j;
    }
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
    dedup_group_owners(ctx, d_records, m, flags, d_rep, 0, nullptr, n_groups, ctx->pick(stream));
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
    return sd_synth_fill_at(ctx, cid, twin, 0, len, d_out, stream);
}

int sd_synth_fill_at(sd_cas_ctx* ctx, uint64_t cid, uint32_t twin, uint64_t offset, uint64_t len, uint8_t* d_out,
                     void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || (len && !d_out)) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (offset % 8 || reinterpret_cast<uintptr_t>(d_out) % 8)
        throw sd_failure(SD_ERR_INVALID, "offset and d_out must be 8-byte aligned");
    ctx->bind();
    HIP_CHECK(sdk::launch_synth_fill(cid, twin, offset, len, d_out, ctx->pick(stream)));
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
