// sd_files.cpp -- the file-reading pipelines of the C ABI (include/sd_cas.h) and the
// streaming hash of messages of unknown length:
//   sd_cas_ids_files / sd_cas_hashes_files   generate_cas_id (cas.rs:23-62) for (path, size)
//                                            pairs: stager pool -> pinned windows -> kernels
//   sd_file_checksums                        file_checksum (hash.rs:10-24) for paths
//   sd_checksums                             file_checksum over ranges of host memory
// The context, batches and kernels they drive are in sd_cas_api.cpp / sd_api_impl.h.
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include <emmintrin.h>

#include "sd_api_impl.h"

using namespace sdi;

namespace {

// host-side co-hashing (sd_checksums): ranges from this size on are hashed block-parallel
constexpr uint64_t SD_CPU_SPLIT_MIN = 8ull << 20;
void check_rc(int rc) {
    if (rc != SD_OK) throw sd_failure(rc, sd_cas_last_error());
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
        sl[k].sync();
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
                HIP_CHECK(sdk::launch_ck_leaf(sl[k].staged.as<uint8_t>(), pos, 0, fin.d_files(),
                                              fin.d_map() + wg0, (uint32_t)(nb - wg0),
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


// A reader thread's cache-resident staging buffer (the longest cas message, padded).
uint8_t* hot_buffer() {
    thread_local std::vector<uint8_t> buf(SD_WHOLE_ITEMS_MAX + 256 + 64);
    return reinterpret_cast<uint8_t*>(align_up(reinterpret_cast<uintptr_t>(buf.data()), 64));
}

// n bytes (a multiple of 64) from a cache-resident buffer to a 64-byte aligned destination
// with streaming stores: the destination's lines are written without being read first
void stream_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
    for (uint64_t o = 0; o < n; o += 64) {
        const __m128i a = _mm_load_si128(reinterpret_cast<const __m128i*>(src + o));
        const __m128i b = _mm_load_si128(reinterpret_cast<const __m128i*>(src + o + 16));
        const __m128i c = _mm_load_si128(reinterpret_cast<const __m128i*>(src + o + 32));
        const __m128i d = _mm_load_si128(reinterpret_cast<const __m128i*>(src + o + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 48), d);
    }
    _mm_sfence();
}

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

extern "C" {

// Path-based drop-in batch: generate_cas_id (cas.rs:23-62) for n (path, size) pairs,
// the sizes being the ones the caller's metadata reported (FileMetadata::new,
// file_identifier/mod.rs:65-97).  A whole-kind file that turns out longer than its
// planned extent (it grew since the caller's stat) is hashed afterwards from the file
// itself, streamed (fs::read hashes every byte, cas.rs:29).
namespace {
// The body of sd_cas_ids_files (hex to host memory) and sd_cas_hashes_files (the 32-byte
// hashes to device memory, for the multi-GPU dedup): out_hex17 xor d_hash32.
//
// The pipeline.  Every file's message is planned up front into windows of consecutive
// files (messages at 128-B starts, at most "files_window_mb" per window).  The stager
// pool's threads take the files in order from ONE cursor for the whole call and read each
// into its window's buffer in a ring of "files_ring" pinned buffers, so no reader waits at
// a window boundary for the window's slowest file or for this thread.  The reader that
// completes a window's last file wakes this thread, which copies the window to the device
// and queues its kernels and D2H on one of two device slots, then hands the previous
// window's buffer (its copy done) back to the readers.  A reader waits only when it is a
// whole ring ahead of the copies.  (Round 2 read one window at a time with a barrier
// after each: 0.70 M files/s from tmpfs against 1.06 M for the same reads into one
// buffer, profiles/r3/r3d_stager_probe.txt.)
void cas_files(sd_cas_ctx* ctx, const char* const* paths, const uint64_t* sizes, size_t n, char* out_hex17,
               uint8_t* d_hash32, int32_t* status, int nthreads) {
    ctx->bind();
    if (n == 0) return;
    nthreads = std::min(64, cap_host_threads(nthreads));  // the process's host budget (sd_host.h)
    // nthreads reader threads stage in the background (start/wait) while this thread plans,
    // launches and harvests the windows
    std::shared_ptr<StagePool> pool = ctx->stage_pool(nthreads + 1);
    const uint64_t WINDOW = (uint64_t)std::max(1, tuning_get(SD_TUNE_FILES_WINDOW_MB)) << 20;
    const int RING = std::max(2, std::min(16, tuning_get(SD_TUNE_FILES_RING)));
    // ---- the plan: extents relative to their window's start, windows of consecutive files
    std::vector<sd_extent> ext(n);
    std::vector<size_t> win_first;
    std::vector<uint64_t> win_bytes;
    {
        uint64_t off = 0;
        for (size_t i = 0; i < n; i++) {
            sd_extent e = plan_extent(sizes[i], off);
            uint64_t next = align_up(off + e.msg_len, SD_STAGE_ALIGN);
            if (win_first.empty() || (i > win_first.back() && next > WINDOW)) {
                if (!win_first.empty()) win_bytes.push_back(off);
                win_first.push_back(i);
                e = plan_extent(sizes[i], 0);
                next = align_up(e.msg_len, SD_STAGE_ALIGN);
            }
            ext[i] = e;
            off = next;
        }
        win_bytes.push_back(off);
    }
    const size_t nw = win_first.size();
    win_first.push_back(n);
    std::vector<uint32_t> win_of(n);
    uint64_t max_win = 0;
    for (size_t w = 0; w < nw; w++) {
        for (size_t i = win_first[w]; i < win_first[w + 1]; i++) win_of[i] = (uint32_t)w;
        max_win = std::max(max_win, win_bytes[w]);
    }
    // ---- the ring of pinned buffers (persistent: borrowed from the context's slot pool)
    struct Ring {
        sd_cas_ctx* c;
        std::vector<std::unique_ptr<Slot>> s;
        ~Ring() {
            for (auto& x : s)
                if (x) c->release(std::move(x));
        }
    } ring{ctx, {}};
    for (int r = 0; r < RING; r++) {
        ring.s.push_back(ctx->acquire());
        ring.s.back()->window.ensure(max_win + 64);
    }
    SlotPair slots(ctx);
    // ---- reader / launcher handshake
    struct Shared {
        std::mutex mu;
        std::condition_variable to_main, to_readers;
        std::unique_ptr<std::atomic<uint32_t>[]> left;      // files of window w not yet staged
        std::unique_ptr<std::atomic<int64_t>[]> ring_win;   // the window ring buffer r may take
        std::atomic<bool> abort{false};
        std::vector<std::pair<size_t, std::vector<uint8_t>>> captured;  // pipes / devices, read whole
    } sh;
    sh.left.reset(new std::atomic<uint32_t>[nw]);
    for (size_t w = 0; w < nw; w++) sh.left[w].store((uint32_t)(win_first[w + 1] - win_first[w]));
    sh.ring_win.reset(new std::atomic<int64_t>[RING]);
    for (int r = 0; r < RING; r++) sh.ring_win[r].store(r);
    std::vector<uint8_t*> ring_buf(RING);
    for (int r = 0; r < RING; r++) ring_buf[r] = ring.s[r]->window.u8();
    hipEvent_t copied[16] = {};          // ring buffer r's H2D (events on the device slots' streams)
    bool copy_pending[16] = {};
    struct Launched {  // the window in flight on a device slot's stream
        std::vector<size_t> files;  // hashed files, in extent order
        bool busy = false;
    } launched[2];
    // (everything the readers touch is declared before `cleanup`, whose destructor waits for
    // them: a throw below must not end those lifetimes while a reader still runs)
    const bool stage_hot = tuning_get(SD_TUNE_FILES_STAGE_HOT) != 0;
    struct Cleanup {  // on any exit: no reader left writing or waiting, no event leaked
        StagePool* pool;
        Shared* sh;
        bool staging = false;
        hipEvent_t* ev;
        ~Cleanup() {
            if (staging) {
                {
                    std::lock_guard<std::mutex> g(sh->mu);
                    sh->abort = true;
                }
                sh->to_readers.notify_all();
                pool->wait();
            }
            for (int k = 0; k < 16; k++)
                if (ev[k]) (void)hipEventDestroy(ev[k]);
        }
    } cleanup{pool.get(), &sh, false, copied};
    // this thread's waits block (hipEventBlockingSync) instead of spinning: the readers need
    // the cores (a container's CPU quota counts a spinning waiter as a busy core)
    for (int r = 0; r < RING; r++)
        HIP_CHECK(hipEventCreateWithFlags(&copied[r], hipEventDisableTiming | hipEventBlockingSync));
    hipEvent_t done_ev[2] = {nullptr, nullptr};  // a device slot's last D2H / scatter
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() {
            for (int k = 0; k < 2; k++)
                if (e[k]) (void)hipEventDestroy(e[k]);
        }
    } done_guard{done_ev};
    for (int k = 0; k < 2; k++)
        HIP_CHECK(hipEventCreateWithFlags(&done_ev[k], hipEventDisableTiming | hipEventBlockingSync));
    auto harvest = [&](int k) {
        if (!launched[k].busy) return;
        HIP_CHECK(hipEventSynchronize(done_ev[k]));
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
    // ---- the readers: file i into its window's ring buffer
    pool->start(n, [&](size_t i) {
        const uint32_t w = win_of[i];
        const int r = (int)(w % (uint32_t)RING);
        if (sh.ring_win[r].load(std::memory_order_acquire) != (int64_t)w) {  // a whole ring ahead
            std::unique_lock<std::mutex> g(sh.mu);
            sh.to_readers.wait(g, [&] { return sh.abort.load() || sh.ring_win[r].load() == (int64_t)w; });
        }
        if (sh.abort.load(std::memory_order_relaxed)) return;
        std::vector<uint8_t> cap;
        if (stage_hot) {  // read into this thread's cache-resident buffer, then stream it out
            sd_extent e = ext[i];
            e.msg_offset = 0;
            uint8_t* hot = hot_buffer();
            status[i] = stage_one(paths[i], e, hot, &cap);
            if (status[i] == SD_FILE_OK) {
                stream_copy(ring_buf[r] + ext[i].msg_offset, hot, sd_align_up(e.msg_len, SD_STAGE_PAD));
                ext[i].msg_len = e.msg_len;
            }
        } else {
            status[i] = stage_one(paths[i], ext[i], ring_buf[r], &cap);
        }
        if (!cap.empty()) {
            std::lock_guard<std::mutex> g(sh.mu);
            sh.captured.emplace_back(i, std::move(cap));
        }
        if (sh.left[w].fetch_sub(1, std::memory_order_acq_rel) == 1) {  // the window's last file
            std::lock_guard<std::mutex> g(sh.mu);
            sh.to_main.notify_one();
        }
    }, nthreads);  // this call's readers only: the pool may hold more from an earlier call
    cleanup.staging = true;
    // SD_PROFILE_FILES=1: one stderr line per call (where this thread's time goes)
    static const bool prof = getenv("SD_PROFILE_FILES") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t_call = clk::now();
    double wait_s = 0, copy_wait_s = 0;
    std::vector<sd_extent> wext;
    std::vector<size_t> widx;
    for (size_t w = 0; w < nw; w++) {
        const auto tw = clk::now();
        if (sh.left[w].load(std::memory_order_acquire) != 0) {
            std::unique_lock<std::mutex> g(sh.mu);
            sh.to_main.wait(g, [&] { return sh.left[w].load(std::memory_order_acquire) == 0; });
        }
        wait_s += std::chrono::duration<double>(clk::now() - tw).count();
        const int r = (int)(w % (size_t)RING), k = (int)(w & 1);
        Slot& sl = slots[k];
        // failed files (I/O error, short read) keep their status and leave the window;
        // files longer than their extent are hashed from disk after the windows
        wext.clear();
        widx.clear();
        for (size_t i = win_first[w]; i < win_first[w + 1]; i++)
            if (status[i] == SD_FILE_OK) {
                wext.push_back(ext[i]);
                widx.push_back(i);
            }
        const size_t m = wext.size();
        if (m) {
            harvest(k);  // device slot k's previous launch (two windows back)
            plan_cas_batch(&sl.cas, wext.data(), m, sl.stream);
            sl.staged.ensure(win_bytes[w] + 64);
            sl.hashes.ensure(m * 32);
            sl.host_hashes.ensure(m * 32);
            HIP_CHECK(hipMemcpyAsync(sl.staged.p, ring_buf[r], win_bytes[w], hipMemcpyHostToDevice, sl.stream));
            HIP_CHECK(hipEventRecord(copied[r], sl.stream));
            copy_pending[r] = true;
            run_cas_batch(&sl.cas, sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
            if (d_hash32) {  // device output: the window's hashes scattered to their files' rows
                dev_idx_h[k].assign(widx.begin(), widx.end());
                dev_idx[k].upload(dev_idx_h[k], sl.stream);
                HIP_CHECK(sdk::launch_scatter_hash(sl.hashes.as<uint32_t>(), dev_idx[k].as<uint32_t>(), (uint32_t)m,
                                                   reinterpret_cast<uint32_t*>(d_hash32), sl.stream));
            } else {
                HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, m * 32, hipMemcpyDeviceToHost, sl.stream));
            }
            HIP_CHECK(hipEventRecord(done_ev[k], sl.stream));
            launched[k].files = widx;
            launched[k].busy = true;
        }
        // the previous window's buffer goes back to the readers once its copy has read it
        if (w >= 1 && w - 1 + RING < nw) {
            const int rp = (int)((w - 1) % (size_t)RING);
            const auto tc = clk::now();
            if (copy_pending[rp]) HIP_CHECK(hipEventSynchronize(copied[rp]));
            copy_pending[rp] = false;
            copy_wait_s += std::chrono::duration<double>(clk::now() - tc).count();
            {
                std::lock_guard<std::mutex> g(sh.mu);
                sh.ring_win[rp].store((int64_t)(w - 1 + RING), std::memory_order_release);
            }
            sh.to_readers.notify_all();
        }
    }
    pool->wait();  // every reader has returned (all windows are complete)
    cleanup.staging = false;
    const auto th = clk::now();
    harvest(0);
    harvest(1);
    if (prof)
        fprintf(stderr,
                "[sd_files] cas_files n=%zu windows=%zu ring=%d window_mb=%d wall=%.3f ms wait=%.3f ms "
                "copy_wait=%.3f ms tail=%.3f ms\n",
                n, nw, RING, (int)(WINDOW >> 20), std::chrono::duration<double>(clk::now() - t_call).count() * 1e3,
                wait_s * 1e3, copy_wait_s * 1e3, std::chrono::duration<double>(clk::now() - th).count() * 1e3);
    // regular files that grew: SD_FILE_CHANGED and not captured by the reader
    std::vector<std::pair<size_t, std::vector<uint8_t>>>& captured = sh.captured;
    std::vector<size_t> overflow;
    {
        std::vector<uint8_t> cap_flag(n, 0);
        for (auto& c : captured) cap_flag[c.first] = 1;
        for (size_t i = 0; i < n; i++)
            if (status[i] == SD_FILE_CHANGED && !cap_flag[i]) overflow.push_back(i);
    }
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
    // batch-size policy: an identifier step's few files are hashed
    // sooner on the host than through reads -> H2D -> kernels -> D2H; "batch_cpu_max" = 0
    // sends every call to the GPU
    if (n <= (size_t)std::max(0, tuning_get(SD_TUNE_BATCH_CPU_MAX))) {
        ctx->files_calls_cpu.fetch_add(1, std::memory_order_relaxed);
        return sd_cpu_cas_ids_files(paths, sizes, n, out_hex17, status, nthreads);
    }
    ctx->files_calls_gpu.fetch_add(1, std::memory_order_relaxed);
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

namespace {

// stat every file in parallel: its length picks the route (regular files only)
void stat_files(StagePool& pool, const char* const* paths, size_t n, std::vector<uint64_t>& hint,
                std::vector<uint8_t>& regular, int threads) {
    hint.assign(n, 0);
    regular.assign(n, 0);
    pool.run(n, [&](size_t i) {
        struct stat st;
        if (stat(paths[i], &st) == 0 && S_ISREG(st.st_mode)) {
            hint[i] = (uint64_t)st.st_size;
            regular[i] = 1;
        }
    }, threads);  // the caller and threads - 1 workers, whatever the pool grew to before
}

// The GPU route of sd_file_checksums over the files next() yields (SIZE_MAX ends them), on
// `read_threads` reader threads.  Each file is read as the reference reads it: hash.rs's
// 1 MiB read calls until one returns fewer.  For a regular file those reads are exactly its
// bytes up to EOF, so regular files are read with parallel preads; anything else (a pipe,
// a device) with the literal sequential loop.  Small regular files are packed (128-B
// aligned) into the current slot's pinned window by their stat length -- one batch per
// window, read in parallel, each file probed past its length in case it grew --; while the
// GPU hashes one slot's window the host reads the next into the other.  Larger files,
// files that grew, and non-regular files stream window by window (Streamer), whatever their
// final length.  hint / regular: stat_files' output for all n files.
void gpu_file_checksums(sd_cas_ctx* ctx, const char* const* paths, char* out_hex65, int32_t* status,
                        int read_threads, const std::vector<uint64_t>& hint, const std::vector<uint8_t>& regular,
                        const std::function<size_t()>& next) {
    ctx->bind();
    // packs of at most 32 MiB: a pack is read whole before its copy starts, so smaller packs
    // let the next pack's reads overlap this one's H2D and kernels (one 80 MB pack of 100
    // files took 4.7 ms against 2.3 ms for the CPU path, read-bound alike)
    constexpr uint64_t PACK = 32ull << 20;
    // the readers deliver through pread_stream (page cache -> L2 -> streaming stores into the
    // pinned window): 0.068 host ns/B against 0.087 for pread straight into the window, and
    // one DRAM read of the window's lines fewer (profiles/r4/r4b_ck_host_cost.jsonl)
    const bool stream_hot = tuning_get(SD_TUNE_CHECKSUM_STAGE_HOT) != 0;
    // the pools may hold more threads than this call's read_threads (a previous call grew
    // them): every run below is limited to read_threads
    std::shared_ptr<StagePool> pool = ctx->stage_pool(read_threads);  // per-file tasks (packs)
    std::shared_ptr<StagePool> iopool;  // preads of one open file (streamed files), created on first use
    SlotPair slots(ctx);
    Streamer::prepare(slots);
    struct Pending {
        std::vector<size_t> files;  // files whose hashes land in this slot's host_hashes
        bool busy = false;
    } pend[2];
    // streamed files' hashes arrive when their slot is next synchronised
    Streamer streamer([&](size_t i, const uint8_t* h) { to_hex(h, 32, out_hex65 + i * 65); });  // hash.rs:21-23
    int cur = 0;
    auto harvest = [&](int k) {  // slot k idle: its window is free, its results delivered
        slots[k].sync();
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
            if (!iopool) iopool = ctx->io_pool(read_threads);
            src.set_parallel(iopool.get(), read_threads, stream_hot);
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
            const int64_t got = stream_hot ? pread_stream(fd, win + pack_off[q], hint[i], 0)
                                           : pread_full(fd, win + pack_off[q], hint[i], 0);
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
        }, read_threads);
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
        plan_checksum_batch(&sl.ck, offs.data(), lens.data(), ok.size(), sl.stream);
        sl.hashes.ensure(ok.size() * 32);
        sl.host_hashes.ensure(ok.size() * 32);
        HIP_CHECK(hipMemcpyAsync(sl.staged.p, win, span + 64, hipMemcpyHostToDevice, sl.stream));
        run_checksum_batch(&sl.ck, sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, ok.size() * 32, hipMemcpyDeviceToHost, sl.stream));
        pend[k].files = std::move(ok);
        pend[k].busy = true;
    };
    for (size_t i; (i = next()) != SIZE_MAX;) {
        status[i] = SD_FILE_OK;
        if (!regular[i] || hint[i] + 128 > PACK / 2) {  // a pipe / device / unreadable path, or large
            submit_pack();
            stream_file(i);
            continue;
        }
        // files start on whole 128-B lines (SD_STAGE_ALIGN): a start mid-line makes every
        // line-pair load of k_ck_leaf straddle two lines (5% slower, scripts/ck_align_probe.py)
        if (pack_end + align_up(hint[i], SD_STAGE_ALIGN) + 64 > PACK) submit_pack();
        pack.push_back(i);
        pack_off.push_back(pack_end);
        pack_len.push_back(hint[i]);
        pack_end = align_up(pack_end + hint[i], SD_STAGE_ALIGN);
    }
    submit_pack();
    for (size_t i : grew) {
        status[i] = SD_FILE_OK;
        stream_file(i);
    }
    harvest(0);
    harvest(1);
    streamer.finish(slots);
}


// sd_file_checksums' split, claimed block by block (round 5).  Every
// large regular file's 1 MiB blocks form one queue, in file order (largest file first); the
// call's `threads` threads (the caller included) all take from it.  A thread first looks for
// a free GPU slot (at most `gpu_slots`): if one is free it claims a run of up to 32 blocks
// of one file, reads them into the slot's pinned window (pread_stream), queues the H2D on
// the call's one copy queue and k_ck_leaf + the blocks' CVs back to the host table on the
// slot's stream, and moves on; otherwise it hashes the small files (whole-file tasks, CPU
// path) and then ONE block at a time on the CPU (cpu_block_cv_fd).  So the GPU takes as much
// as its slots keep moving -- PCIe fills with the fewest reader threads -- and the rest is
// hashed on the host with 1 MiB granularity: no route waits on the other's last whole file
// (round 4's split claimed whole files and lost up to one file's time at the end; the GPU's
// claims shrink towards the end as well).  The threads make HIP calls, so they run on the
// context's shared-fd-table pool (io_pool: a private table's copies of the runtime's device
// descriptors are closed); a thread keeps its descriptor while its claims stay in one file,
// so the shared table's lock sees about one open per file and thread.  Each file's root is
// merged on the host from its block CVs (cpu_root_from_cvs); a file that turns out shorter
// or longer than its stat length is hashed again with hash.rs's sequential loop, as the CPU
// path does.
void split_checksums_blocks(sd_cas_ctx* ctx, const char* const* paths, char* out_hex65, int32_t* status,
                            int threads, int gpu_slots, const std::vector<size_t>& big,
                            const std::vector<size_t>& rest, const std::vector<uint64_t>& hint) {
    ctx->bind();
    constexpr uint64_t GPU_RUN = 32;  // blocks per GPU claim while plenty is left
    const size_t nf = big.size();
    // one plan over every large file: file q's blocks are CV slots [fb[q], fb[q+1]) and its
    // message bytes sit at the virtual offset fb[q] MiB, so a window holding its blocks
    // [b0, b1) is shifted by (fb[q] + b0) MiB
    std::vector<ck_file> files(nf);
    std::vector<uint64_t> fb(nf + 1, 0);
    for (size_t q = 0; q < nf; q++) {
        const uint64_t len = hint[big[q]];
        files[q] = ck_file{fb[q] * SD_CK_BLOCK, len, fb[q]};
        fb[q + 1] = fb[q] + (len + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
    }
    const uint64_t nb_total = fb[nf];
    if (nb_total >= (1ull << 31)) throw sd_failure(SD_ERR_INVALID, "split call too large");
    std::vector<sd_u32x2> map(nb_total);
    for (size_t q = 0; q < nf; q++)
        for (uint64_t b = fb[q]; b < fb[q + 1]; b++) map[b] = sd_u32x2{(uint32_t)q, (uint32_t)(b - fb[q])};
    struct GpuSlot {
        std::unique_ptr<Slot> s;
        hipEvent_t copied = nullptr;
        bool filling = false;          // a thread is reading into it (under mu)
        std::atomic<uint32_t> busy{0};  // 1 from its claim until its run's CVs are home
    };
    struct Slots {
        sd_cas_ctx* c;
        std::vector<GpuSlot> g;
        std::unique_ptr<Slot> cp;  // the call's one H2D queue (SlotPair::copy_stream)
        ~Slots() {
            for (auto& x : g) {
                if (x.s) {
                    (void)hipStreamSynchronize(x.s->stream);
                    c->release(std::move(x.s));
                }
                if (x.copied) (void)hipEventDestroy(x.copied);
            }
            if (cp) {
                (void)hipStreamSynchronize(cp->stream);
                c->release(std::move(cp));
            }
        }
    } sl{ctx, std::vector<GpuSlot>(std::max(1, gpu_slots)), nullptr};
    sl.cp = ctx->acquire();
    // the call's tables and CV tables live on its copy slot, grow-only in the context's slot
    // pool: no per-call hipMalloc/hipHostMalloc, and no hipFree/hipHostFree (each of which
    // synchronises the device and stalled concurrent calls)
    Tables& tab = sl.cp->aux;
    tab.begin();
    const size_t o_files = tab.add(files), o_map = tab.add(map);
    tab.upload(nullptr);
    DevBuf& d_cv = sl.cp->hashes;
    d_cv.ensure(nb_total * 32);
    PinnedBuf& h_cv = sl.cp->host_hashes;  // every block's CV, from either side
    h_cv.ensure(nb_total * 32);
    for (auto& x : sl.g) {
        x.s = ctx->acquire();
        x.s->window.ensure(GPU_RUN * SD_CK_BLOCK + 128);
        x.s->staged.ensure(GPU_RUN * SD_CK_BLOCK + 128);
        HIP_CHECK(hipEventCreateWithFlags(&x.copied, hipEventDisableTiming));
    }
    // a slot's run is done when the stream reaches this host function: it clears `busy`,
    // so the threads look for free slots without a HIP call (an hipEventQuery per claim,
    // made under the claim lock, stalled every thread whenever it was slow)
    const hipHostFn_t slot_done = [](void* p) { static_cast<std::atomic<uint32_t>*>(p)->store(0, std::memory_order_release); };

    std::mutex mu, copy_mu;
    size_t cf = 0;  // claim cursor: file cf, its block cb
    uint64_t cb = 0, left = nb_total;
    std::atomic<size_t> small_next{0};
    std::vector<uint8_t> failed(nf, 0);  // a short read: hashed again with the read loop
    std::atomic<uint64_t> gpu_bytes{0}, cpu_bytes{0};
    std::atomic<bool> stop{false};
    int err_rc = SD_OK;
    std::string err_msg;
    // [b0, b1) of file q, at most `want` blocks (under mu)
    auto claim = [&](uint64_t want, size_t& q, uint64_t& b0, uint64_t& b1) -> bool {
        while (cf < nf && cb >= fb[cf + 1] - fb[cf]) {
            cf++;
            cb = 0;
        }
        if (cf >= nf) return false;
        q = cf;
        b0 = cb;
        b1 = std::min(fb[cf + 1] - fb[cf], cb + want);
        cb = b1;
        left -= b1 - b0;
        return true;
    };
    auto worker = [&](size_t) {
        int fd = -1;               // this thread's descriptor of file fd_q, kept across its claims
        size_t fd_q = SIZE_MAX;
        auto file = [&](size_t q) {
            if (q != fd_q) {
                if (fd >= 0) close(fd);
                fd = open(paths[big[q]], O_RDONLY | O_CLOEXEC);  // hash.rs:11
                fd_q = q;
            }
            return fd;
        };
        try {
            ctx->bind();  // (the caller's device is already current; a pool thread's may not be)
            while (!stop.load(std::memory_order_relaxed)) {
                int k = -1;
                size_t q = 0;
                uint64_t b0 = 0, b1 = 0;
                {
                    std::lock_guard<std::mutex> g(mu);
                    if (left > 0)
                        for (int j = 0; j < (int)sl.g.size() && k < 0; j++)
                            if (!sl.g[j].filling && sl.g[j].busy.load(std::memory_order_acquire) == 0) k = j;
                    // the GPU's runs shrink towards the end, so its last ones finish with the host's
                    if (k >= 0 && claim(std::max<uint64_t>(4, std::min<uint64_t>(GPU_RUN, left / (2 * (uint64_t)threads))),
                                        q, b0, b1)) {
                        sl.g[k].filling = true;
                        sl.g[k].busy.store(1, std::memory_order_relaxed);
                    } else {
                        k = -1;
                    }
                }
                if (k >= 0) {
                    GpuSlot& x = sl.g[k];
                    Slot& s = *x.s;
                    const uint64_t off = b0 * SD_CK_BLOCK, bytes = std::min(b1 * SD_CK_BLOCK, files[q].len) - off;
                    const int f = file(q);
                    const int64_t got = f < 0 ? -1 : pread_stream(f, s.window.u8(), bytes, off);
                    if (got != (int64_t)bytes) {
                        std::lock_guard<std::mutex> g(mu);
                        failed[q] = 1;
                        x.busy.store(0, std::memory_order_relaxed);
                        x.filling = false;
                        continue;
                    }
                    {
                        std::lock_guard<std::mutex> g(copy_mu);  // the copy and its event, back to back on the queue
                        HIP_CHECK(hipMemcpyAsync(s.staged.p, s.window.p, bytes, hipMemcpyHostToDevice, sl.cp->stream));
                        HIP_CHECK(hipEventRecord(x.copied, sl.cp->stream));
                    }
                    HIP_CHECK(hipStreamWaitEvent(s.stream, x.copied, 0));
                    HIP_CHECK(sdk::launch_ck_leaf(s.staged.as<uint8_t>(), files[q].offset + off, 0,
                                                  tab.at<ck_file>(o_files), tab.at<uint2>(o_map) + fb[q] + b0,
                                                  (uint32_t)(b1 - b0), d_cv.as<uint32_t>(), d_cv.as<uint32_t>(),
                                                  s.stream));
                    HIP_CHECK(hipMemcpyAsync(h_cv.u8() + 32 * (fb[q] + b0), d_cv.as<uint8_t>() + 32 * (fb[q] + b0),
                                             32 * (b1 - b0), hipMemcpyDeviceToHost, s.stream));
                    HIP_CHECK(hipLaunchHostFunc(s.stream, slot_done, &x.busy));
                    gpu_bytes.fetch_add(bytes, std::memory_order_relaxed);
                    std::lock_guard<std::mutex> g(mu);
                    x.filling = false;
                    continue;
                }
                const size_t i = small_next.fetch_add(1, std::memory_order_relaxed);
                if (i < rest.size()) {  // the small and non-regular files: whole-file tasks, CPU path
                    status[rest[i]] = cpu_checksum_file(paths[rest[i]], out_hex65 + 65 * rest[i]);
                    cpu_bytes.fetch_add(hint[rest[i]], std::memory_order_relaxed);
                    continue;
                }
                {
                    std::lock_guard<std::mutex> g(mu);
                    if (!claim(1, q, b0, b1)) break;
                    if (failed[q]) continue;
                }
                const int f = file(q);
                const bool ok = f >= 0 && cpu_block_cv_fd(f, files[q].len, b0, h_cv.u8() + 32 * (fb[q] + b0));
                if (!ok) {
                    std::lock_guard<std::mutex> g(mu);
                    failed[q] = 1;
                }
                cpu_bytes.fetch_add(std::min(SD_CK_BLOCK, files[q].len - b0 * SD_CK_BLOCK), std::memory_order_relaxed);
            }
        } catch (const sd_failure& e) {
            std::lock_guard<std::mutex> g(mu);
            if (err_rc == SD_OK) {
                err_rc = e.rc;
                err_msg = e.what();
            }
            stop.store(true);
        } catch (...) {
            std::lock_guard<std::mutex> g(mu);
            if (err_rc == SD_OK) {
                err_rc = SD_ERR_NOMEM;
                err_msg = "host allocation failed in a split sd_file_checksums call";
            }
            stop.store(true);
        }
        if (fd >= 0) close(fd);
    };
    // the shared-fd-table pool: these threads make HIP calls (see above)
    std::shared_ptr<StagePool> pool = ctx->io_pool(threads);
    pool->run((size_t)threads, worker, threads);
    for (auto& x : sl.g) HIP_CHECK(hipStreamSynchronize(x.s->stream));  // every CV is in h_cv
    if (err_rc != SD_OK) throw sd_failure(err_rc, err_msg);
    ctx->checksum_bytes_gpu.fetch_add(gpu_bytes.load(), std::memory_order_relaxed);
    ctx->checksum_bytes_cpu_split.fetch_add(cpu_bytes.load(), std::memory_order_relaxed);
    // each file's root from its block CVs -- unless a read came back short, or a byte lies
    // past the stat length (it grew): then hash.rs's sequential loop, to EOF
    for (size_t q = 0; q < nf; q++) {
        const size_t i = big[q];
        bool at_end = false;
        if (!failed[q]) {
            const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
            uint8_t probe;
            at_end = fd >= 0 && pread_full(fd, &probe, 1, files[q].len) == 0;
            if (fd >= 0) close(fd);
        }
        if (at_end) {
            uint8_t h[32];
            cpu_root_from_cvs(h_cv.u8() + 32 * fb[q], fb[q + 1] - fb[q], h);
            to_hex(h, 32, out_hex65 + 65 * i);  // hash.rs:21-23
            status[i] = SD_FILE_OK;
        } else {
            status[i] = cpu_checksum_file(paths[i], out_hex65 + 65 * i);
        }
    }
}

}  // namespace

// file_checksum (hash.rs:10-24) for n paths: the batch policy picks the CPU path, the GPU
// route (gpu_file_checksums) or both at once.
//   * "checksum_cpu_max" = 0: the GPU route for every call.
//   * Hybrid ("checksum_hybrid_threads" = g, default 6): a call whose regular files of
//     >= 8 MiB add up to >= 512 MiB is split.  Handing a byte to the GPU costs the host
//     0.07-0.10 ns (pread into a cache-resident buffer, streaming stores into the pinned
//     window: pread_stream), hashing it on the CPU path 0.17-0.18 ns (the pread plus 0.11 ns
//     of AVX-512 BLAKE3) -- scripts/ck_host_cost.cpp, profiles/r4/r4b_ck_host_cost.jsonl,
//     profiles/r5/r5c_ck_host_bound.jsonl -- and both are bound by host CPU time, not DRAM
//     (the split moves 150-230 GB/s of DRAM traffic against the 16 threads' measured 450-650
//     GB/s).  So the threads feed the GPU while it has room (g slots) and hash the rest:
//     split_checksums_blocks above, claimed by 1 MiB blocks ("checksum_split_blocks" 1,
//     profiles/r5/r5e_hybrid_blocks.json: 1.13-1.43x the CPU path alone from the page cache).
//     With "checksum_split_blocks" 0, round 4's split: the GPU route on g reader threads and
//     the CPU path on the rest on a second host thread, whole large files to whichever is
//     free next (one shared cursor, largest first; 0.9-1.24x, the last whole file the tail).
//     The split's gain depends on the host: 0.93-1.34x the CPU path alone on round 5's four
//     boxes.  So ("checksum_split_adapt" k, default 8) each such call takes the split or the
//     CPU path alone, by the GB/s this context measured for each: each once, then the
//     faster, the other every k-th call (split_route_choose, sd_host.h).
//   * Otherwise calls of at most "checksum_cpu_max" files (default: all) take the CPU path:
//     from the page cache the host's threads hash faster than PCIe carries the bytes.
int sd_file_checksums(sd_cas_ctx* ctx, const char* const* paths, size_t n, char* out_hex65, int32_t* status) {
    SD_GUARD_BEGIN
    if (!ctx || (n && (!paths || !out_hex65 || !status))) throw sd_failure(SD_ERR_INVALID, "null argument");
    const int threads = std::min(64, cap_host_threads(tuning_get(SD_TUNE_READ_THREADS)));
    const int cpu_max = std::max(0, tuning_get(SD_TUNE_CHECKSUM_CPU_MAX));
    // the GPU route's share of the readers in a split call: "checksum_hybrid_threads" g of
    // 16, scaled down with a smaller host budget (g = 4: 2 of 8 threads, 1 of 4)
    const int hyb_knob = std::max(0, tuning_get(SD_TUNE_CHECKSUM_HYBRID_THREADS));
    const int hyb = threads >= 16 ? hyb_knob : std::min(hyb_knob, std::max(1, hyb_knob * threads / 16));
    std::vector<uint64_t> hint;
    std::vector<uint8_t> regular;
    // the learned route compares whole calls: from here, so the split's stat pass counts
    // against it as the CPU path's own stat pass does against that route
    const auto t0 = std::chrono::steady_clock::now();
    if (cpu_max != 0 && hyb > 0 && hyb < threads && n >= 2) {
        constexpr uint64_t BIG_FILE = 8ull << 20, BIG_TOTAL = 512ull << 20;
        stat_files(*ctx->stage_pool(threads), paths, n, hint, regular, threads);
        std::vector<size_t> big, rest;
        uint64_t big_bytes = 0;
        for (size_t i = 0; i < n; i++) {
            if (regular[i] && hint[i] >= BIG_FILE) {
                big.push_back(i);
                big_bytes += hint[i];
            } else {
                rest.push_back(i);
            }
        }
        if (big.size() >= 2 && big_bytes >= BIG_TOTAL) {
            // the split, or the CPU path alone where this host has hashed faster by itself
            // ("checksum_split_adapt" k > 0: each route once, then the faster by its recent
            // GB/s, the other every k-th call; sd_host.h split_route_choose)
            const int adapt = std::max(0, tuning_get(SD_TUNE_CHECKSUM_SPLIT_ADAPT));
            int route = 0;
            if (adapt) {
                std::lock_guard<std::mutex> g(ctx->split_mu);
                // what either route's rate depends on: a change of it starts the learning again
                const uint64_t gen = split_route_tuning_gen();
                if (ctx->split_routes_gen != gen) {
                    ctx->split_routes = SplitRoutes{};
                    ctx->split_routes_gen = gen;
                }
                route = split_route_choose(ctx->split_routes, (uint32_t)adapt);
            }
            uint64_t call_bytes = 0;
            for (size_t q = 0; q < n; q++) call_bytes += hint[q];
            auto learn = [&](int r) {
                if (!adapt) return;
                const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                std::lock_guard<std::mutex> g(ctx->split_mu);
                split_route_record(ctx->split_routes, r, (double)call_bytes / std::max(s, 1e-9) / 1e9);
            };
            if (route == 1) {
                ctx->checksum_calls_cpu.fetch_add(1, std::memory_order_relaxed);
                const int rc = sd_cpu_file_checksums(paths, n, out_hex65, status, threads);
                if (rc == SD_OK) learn(1);
                return rc;
            }
            ctx->checksum_calls_hybrid.fetch_add(1, std::memory_order_relaxed);
            std::stable_sort(big.begin(), big.end(), [&](size_t a, size_t b) { return hint[a] > hint[b]; });
            if (tuning_get(SD_TUNE_CHECKSUM_SPLIT_BLOCKS) != 0) {
                split_checksums_blocks(ctx, paths, out_hex65, status, threads, hyb, big, rest, hint);
                learn(0);
                return SD_OK;
            }
            std::atomic<size_t> cursor{0};
            auto next_big = [&]() -> size_t {
                const size_t k = cursor.fetch_add(1, std::memory_order_relaxed);
                return k < big.size() ? big[k] : SIZE_MAX;
            };
            const int cpu_threads = threads - hyb;
            int cpu_rc = SD_OK;
            std::string cpu_err;
            std::thread cpu([&] {
              library_thread_place();  // the device's NUMA node (sd_host.h)
              try {
                if (!rest.empty()) {  // the small and non-regular files: one CPU-path call
                    std::vector<const char*> p(rest.size());
                    std::vector<char> hex(rest.size() * 65);
                    std::vector<int32_t> st(rest.size());
                    uint64_t rest_bytes = 0;
                    for (size_t q = 0; q < rest.size(); q++) {
                        p[q] = paths[rest[q]];
                        rest_bytes += hint[rest[q]];
                    }
                    ctx->checksum_bytes_cpu_split.fetch_add(rest_bytes, std::memory_order_relaxed);
                    cpu_rc = sd_cpu_file_checksums(p.data(), rest.size(), hex.data(), st.data(), cpu_threads);
                    if (cpu_rc != SD_OK) {
                        cpu_err = sd_cas_last_error();
                        cursor.store(big.size());  // stop the GPU route at its next file
                        return;
                    }
                    for (size_t q = 0; q < rest.size(); q++) {
                        status[rest[q]] = st[q];
                        memcpy(out_hex65 + 65 * rest[q], hex.data() + 65 * q, 65);
                    }
                }
                // then large files, as they come.  The CPU path hashes a file's 1 MiB blocks on
                // all its threads and idles them at the file's last blocks, so it claims files
                // until it holds about 16 MiB per thread (the large ones come first, singly; the
                // smaller tail of the list a few at a time)
                const uint64_t group_bytes = (uint64_t)cpu_threads << 24;
                std::vector<size_t> grp;
                std::vector<const char*> gp;
                std::vector<char> ghex;
                std::vector<int32_t> gst;
                for (;;) {
                    grp.clear();
                    uint64_t bytes = 0;
                    for (size_t i; bytes < group_bytes && (i = next_big()) != SIZE_MAX;) {
                        grp.push_back(i);
                        bytes += hint[i];
                    }
                    if (grp.empty()) break;
                    ctx->checksum_bytes_cpu_split.fetch_add(bytes, std::memory_order_relaxed);
                    gp.resize(grp.size());
                    ghex.resize(grp.size() * 65);
                    gst.resize(grp.size());
                    for (size_t q = 0; q < grp.size(); q++) gp[q] = paths[grp[q]];
                    cpu_rc = sd_cpu_file_checksums(gp.data(), grp.size(), ghex.data(), gst.data(), cpu_threads);
                    if (cpu_rc != SD_OK) {
                        cpu_err = sd_cas_last_error();
                        cursor.store(big.size());
                        return;
                    }
                    for (size_t q = 0; q < grp.size(); q++) {
                        status[grp[q]] = gst[q];
                        memcpy(out_hex65 + 65 * grp[q], ghex.data() + 65 * q, 65);
                    }
                }
              } catch (...) {  // an allocation here: nothing may escape a thread
                cpu_rc = SD_ERR_NOMEM;
                cpu_err = "host allocation failed in the CPU half of a split sd_file_checksums call";
                cursor.store(big.size());
              }
            });
            try {
                gpu_file_checksums(ctx, paths, out_hex65, status, hyb, hint, regular, [&]() -> size_t {
                    const size_t i = next_big();
                    if (i != SIZE_MAX) ctx->checksum_bytes_gpu.fetch_add(hint[i], std::memory_order_relaxed);
                    return i;
                });
            } catch (...) {
                cursor.store(big.size());  // the CPU thread takes no further file
                cpu.join();
                throw;
            }
            cpu.join();
            if (cpu_rc != SD_OK) throw sd_failure(cpu_rc, cpu_err);
            learn(0);
            return SD_OK;
        }
    }
    if (n <= (size_t)cpu_max) {
        ctx->checksum_calls_cpu.fetch_add(1, std::memory_order_relaxed);
        return sd_cpu_file_checksums(paths, n, out_hex65, status, threads);
    }
    ctx->checksum_calls_gpu.fetch_add(1, std::memory_order_relaxed);
    if (hint.size() != n) stat_files(*ctx->stage_pool(threads), paths, n, hint, regular, threads);
    size_t i = 0;
    uint64_t all = 0;
    for (size_t q = 0; q < n; q++) all += hint[q];
    ctx->checksum_bytes_gpu.fetch_add(all, std::memory_order_relaxed);
    gpu_file_checksums(ctx, paths, out_hex65, status, threads, hint, regular,
                       [&]() -> size_t { return i < n ? i++ : SIZE_MAX; });
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
    // Co-hashed calls (below) or the CPU path alone, learned per context as sd_file_checksums
    // learns its split ("checksum_split_adapt" k, split_route_choose): the co-hashed call
    // reaches 98 % of its two halves' sum on one host (13 threads + PCIe) and lost to 16
    // threads alone on a host whose CPU path read 127 GB/s (0.95x, profiles/r6/r6f_*), so no
    // fixed choice is right everywhere.  Calls are timed from here, either route.
    const int cohash_cap = std::max(0, std::min({64, tuning_get(SD_TUNE_HOST_COHASH_THREADS),
                                                 checksum_cohash_cap(host_cpu_budget())}));
    uint64_t call_bytes = 0;
    for (size_t q = 0; q < n; q++) call_bytes += lens[q];
    const int adapt = std::max(0, tuning_get(SD_TUNE_CHECKSUM_SPLIT_ADAPT));
    const bool learn_route = adapt > 0 && cohash_cap > 0 && n && call_bytes >= (1ull << 30);
    const auto t_call = std::chrono::steady_clock::now();
    auto learn = [&](int route) {
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_call).count();
        std::lock_guard<std::mutex> g(ctx->split_mu);
        split_route_record(ctx->cohash_routes, route, (double)call_bytes / std::max(sec, 1e-9) / 1e9);
    };
    if (learn_route) {
        int route;
        {
            std::lock_guard<std::mutex> g(ctx->split_mu);
            const uint64_t gen = split_route_tuning_gen();
            if (ctx->cohash_routes_gen != gen) {
                ctx->cohash_routes = SplitRoutes{};
                ctx->cohash_routes_gen = gen;
            }
            route = split_route_choose(ctx->cohash_routes, (uint32_t)adapt);
        }
        if (route == 1) {  // the CPU path alone, on the host budget's threads
            std::vector<uint8_t> h32(32 * n);
            check_rc(sd_cpu_checksums(data, offsets, lens, n, h32.data(), host_cpu_budget()));
            for (size_t q = 0; q < n; q++) to_hex(h32.data() + 32 * q, 32, out_hex65 + 65 * q);
            ctx->checksums_host_bytes.fetch_add(call_bytes, std::memory_order_relaxed);
            learn(1);
            return SD_OK;
        }
    }
    constexpr uint64_t W = Streamer::W;
    SlotPair slots(ctx);
    Streamer::prepare(slots);
    sd_checksum_batch big;
    struct Pending {
        size_t i0 = 0, i1 = 0;
        bool busy = false;
    } pend[2];
    auto harvest = [&](int k) {
        if (!pend[k].busy) return;
        slots[k].sync();
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
        HIP_CHECK(hipEventCreateWithFlags(&used[k], hipEventDisableTiming | hipEventBlockingSync));
    }
    // H2D of `bytes` from `src` to byte `dst` of slot k's device window, after its previous
    // kernels (first piece of a window) / before its next kernels (last piece)
    auto copy_in = [&](int k, const uint8_t* src, uint64_t bytes, uint64_t dst = 0, bool first = true,
                       bool last = true) {
        if (first && used_set[k]) HIP_CHECK(hipStreamWaitEvent(cs, used[k], 0));
        HIP_CHECK(hipMemcpyAsync(slots[k].staged.as<uint8_t>() + dst, src, bytes, hipMemcpyHostToDevice, cs));
        if (!last) return;
        HIP_CHECK(hipEventRecord(copied[k], cs));
        HIP_CHECK(hipStreamWaitEvent(slots[k].stream, copied[k], 0));
    };
    auto done_with = [&](int k) {
        HIP_CHECK(hipEventRecord(used[k], slots[k].stream));
        used_set[k] = true;
    };
    int cur = 0;
    std::vector<uint64_t> offs, ls;
    struct RunT {  // a piece of a window copied with one H2D
        uint64_t host_lo, host_end, dev_lo;
    };
    std::vector<RunT> runs;
    // Co-hashing (as sd_cas_ids, "host_cohash_threads" h > 0, calls of >= 1 GiB): one host
    // thread claims ranges from the END -- one large range, or consecutive small ones up to
    // 64 MiB -- and hashes them with h pool threads on the CPU path (a range of 8 MiB or
    // more block-parallel: its 1 MiB blocks' chaining values on all threads, then the root),
    // while the loop below claims its windows and streamed ranges from the front.
    // One range of >= 256 MiB is shared at block granularity instead of claimed whole, so the
    // two sides finish together (a whole claim leaves the other side idle for up to one
    // range's time; a call of one huge range would go to whichever side claims it first):
    // `sh`, chosen before either side starts, is the range holding the byte where the two
    // are predicted to meet (the GPU at the H2D rate, the host at h threads' hashing rate),
    // or the large range nearest it.  Each side claims whole ranges until it reaches `sh`;
    // there the GPU loop claims its 1 MiB blocks a window at a time from the front, the
    // host thread 64 blocks at a time from the back into a host CV table; when none is
    // left, the GPU loop uploads the host's CVs next to its own and runs the reduce passes.
    // Never more host threads than the process's host budget less 3/16 of it (at least one:
    // this thread), i.e. 13 of 16.  Measured on the box (16-CPU quota, 4 x 1 GiB, interleaved
    // rounds; scripts/cohash_checksum_probe.py, profiles/r5/r5g_cohash_checksum.json and
    // r5h_cohash_ck.json): 13 co-hashing threads 138-151 GB/s, 14: 136-148, 15: 123-129 --
    // at 15 the process burns 16.5 CPUs of time per call for fewer bytes (no throttled
    // periods: the contention is the cores', not the quota's).  The headroom scales with the
    // budget (an absolute 3 left one thread of a 4-CPU budget): 8 -> 6, 4 -> 3,
    // 2 -> 1 (checksum_cohash_cap, sd_host.h).  sd_cas_ids keeps budget - 1: there 15
    // measured best (4.86 vs 4.51 M files/s at 13, r5h_cohash_cas.json).
    const int cohash = cohash_cap;
    const uint64_t all_bytes = call_bytes;
    std::mutex claim_mu;
    size_t back = n, front = 0;  // [back, n) claimed by the host, [0, front) by the GPU loop
    constexpr uint64_t SHARED_MIN = 256ull << 20, HOST_UNIT = 64;  // bytes; blocks per host claim
    // the meet prediction's rates: the H2D copy bounds the GPU side, ~5.5 GB/s a host thread
    // (BLAKE3 with AVX-512, profiles/r4/r4j_shared_range_probe.json); only the split point
    // depends on them, never a result
    constexpr double GPU_GBPS = 55.0, HOST_THREAD_GBPS = 5.5;
    struct SharedRange {
        size_t idx = SIZE_MAX;  // the range (one per call)
        uint64_t nb = 0, sf = 0, sb = 0;  // its blocks: [0, sf) the GPU's, [sb, nb) the host's
        int inflight = 0;      // host claims being hashed
        std::vector<uint8_t> cvs;  // the host's block CVs, 32 B at 32 * block
        std::condition_variable cv;
    } sh;
    int host_rc = SD_OK;
    std::string host_err;
    std::atomic<uint64_t> host_bytes{0};  // bytes the host threads hashed (sd_checksums_stats)
    std::thread host;
    struct JoinHost {
        std::thread& t;
        std::mutex& mu;
        size_t& back;
        SharedRange& sh;
        ~JoinHost() {
            {
                std::lock_guard<std::mutex> g(mu);
                back = 0;
                sh.sb = sh.sf;  // the host takes no further block
            }
            if (t.joinable()) t.join();
        }
    } join_host{host, claim_mu, back, sh};
    if (cohash > 0 && n && all_bytes >= (1ull << 30)) {
        sh.idx = shared_range_pick(lens, n, SHARED_MIN, cohash, GPU_GBPS, HOST_THREAD_GBPS);
        if (sh.idx != SIZE_MAX) {
            sh.nb = (lens[sh.idx] + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
            sh.sf = 0;
            sh.sb = sh.nb;
            sh.cvs.resize(sh.nb * 32);
        }
        host = std::thread([&] {
            library_thread_place();  // the device's NUMA node (sd_host.h)
            try {
                std::vector<uint8_t> h32, cvs;
                for (;;) {
                    size_t b0, b1;
                    uint64_t u0 = 0, u1 = 0;  // a claim of the shared range's blocks
                    {
                        std::lock_guard<std::mutex> g(claim_mu);
                        // the shared range's blocks once every range after it is claimed
                        if (sh.idx != SIZE_MAX && back <= sh.idx + 1 && sh.sb > sh.sf) {
                            u1 = sh.sb;
                            u0 = std::max(sh.sf, u1 > HOST_UNIT ? u1 - HOST_UNIT : 0);
                            sh.sb = u0;
                            sh.inflight++;
                        }
                    }
                    if (u1 > u0) {
                        struct Done {  // on every exit, so the GPU loop's wait ends
                            SharedRange& s;
                            std::mutex& mu;
                            ~Done() {
                                {
                                    std::lock_guard<std::mutex> g(mu);
                                    s.inflight--;
                                }
                                s.cv.notify_all();
                            }
                        } done{sh, claim_mu};
                        cpu_block_cvs(data + offsets[sh.idx], lens[sh.idx], u0, u1, sh.cvs.data(), cohash);
                        host_bytes.fetch_add(std::min(u1 * SD_CK_BLOCK, lens[sh.idx]) - u0 * SD_CK_BLOCK,
                                             std::memory_order_relaxed);
                        continue;
                    }
                    {
                        std::lock_guard<std::mutex> g(claim_mu);
                        if (back <= front) return;
                        b1 = back;
                        if (b1 - 1 == sh.idx) {  // the shared range: its blocks only, above
                            back = sh.idx;
                            continue;
                        }
                        // (the host reaches ranges before `sh` only once its blocks are gone)
                        b0 = b1 - 1;
                        uint64_t sum = lens[b0];
                        while (b0 > front && lens[b0] < SD_CPU_SPLIT_MIN && lens[b0 - 1] < SD_CPU_SPLIT_MIN &&
                               sum + lens[b0 - 1] <= (64ull << 20)) {
                            b0--;
                            sum += lens[b0];
                        }
                        back = b0;
                    }
                    h32.resize((b1 - b0) * 32);
                    if (b1 - b0 == 1 && lens[b0] >= SD_CPU_SPLIT_MIN) {  // one large range, block-parallel
                        uint64_t o = 0, l = 0, cvb = 0;
                        check_rc(sd_split_range(lens[b0], 1, 0, &o, &l, &cvb));
                        cvs.resize(cvb);
                        check_rc(sd_cpu_split_leaves(data + offsets[b0], lens[b0], 1, 0, cvs.data(), cohash));
                        check_rc(sd_cpu_split_root(cvs.data(), lens[b0], h32.data()));
                    } else {
                        check_rc(sd_cpu_checksums(data, offsets + b0, lens + b0, b1 - b0, h32.data(), cohash));
                    }
                    for (size_t q = b0; q < b1; q++) {
                        to_hex(h32.data() + 32 * (q - b0), 32, out_hex65 + 65 * q);
                        host_bytes.fetch_add(lens[q], std::memory_order_relaxed);
                    }
                }
            } catch (const sd_failure& e) {
                host_rc = e.rc;
                host_err = e.what();
            } catch (...) {
                host_rc = SD_ERR_NOMEM;
                host_err = "host allocation failed in a co-hashed sd_checksums call";
            }
            std::lock_guard<std::mutex> g(claim_mu);
            back = front;  // the GPU loop takes nothing further from here on: stop it
        });
    }
    // the GPU loop's claims: range i is the GPU's if no host thread took it
    auto claim = [&](size_t i) -> bool {
        std::lock_guard<std::mutex> g(claim_mu);
        if (i >= back && i != sh.idx) return false;
        front = std::max(front, i + 1);
        return true;
    };
    for (size_t i = 0; i < n;) {
        if (!claim(i)) {
            // the host took range i and everything after it -- except the shared range,
            // which may lie beyond ranges the host claimed whole after sharing it
            size_t s;
            {
                std::lock_guard<std::mutex> g(claim_mu);
                s = sh.idx;
            }
            if (s != SIZE_MAX && s > i) {
                i = s;
                continue;
            }
            break;
        }
        if (i == sh.idx) {  // the shared range: windows of blocks from the front until the host's
            harvest(0);
            harvest(1);
            const uint64_t off0 = 0, L = lens[i];
            plan_checksum_batch(&big, &off0, &L, 1, nullptr);
            constexpr uint64_t BPW = W / SD_CK_BLOCK;
            for (;;) {
                uint64_t w0, w1;
                // claim at the device's pace, not the enqueue rate (the copies are async from
                // pinned memory): slot cur's previous window must have been hashed first, so
                // at most two windows are the GPU's ahead of the host's claims
                if (used_set[cur]) HIP_CHECK(hipEventSynchronize(used[cur]));
                {
                    std::lock_guard<std::mutex> g(claim_mu);
                    if (sh.sf >= sh.sb) break;
                    // windows shrink to a third of what is left (>= 32 blocks), so the
                    // GPU's last windows in flight are short when the two sides meet
                    w0 = sh.sf;
                    w1 = std::min(sh.sb, w0 + std::min<uint64_t>(BPW, std::max<uint64_t>(32, (sh.sb - w0) / 3)));
                    sh.sf = w1;
                }
                const int k = cur;
                cur ^= 1;
                const uint64_t pos = w0 * SD_CK_BLOCK, here = std::min(w1 * SD_CK_BLOCK, L) - pos;
                copy_in(k, data + offsets[i] + pos, here);
                HIP_CHECK(sdk::launch_ck_leaf(slots[k].staged.as<uint8_t>(), pos, 0, big.d_files(),
                                              big.d_map() + w0, (uint32_t)(w1 - w0), big.lvl[0].as<uint32_t>(),
                                              slots[k].hashes.as<uint32_t>(), slots[k].stream));
                done_with(k);
            }
            uint64_t hb0;
            {
                std::unique_lock<std::mutex> lk(claim_mu);
                sh.cv.wait(lk, [&] { return sh.inflight == 0; });  // the host's claims are hashed
                hb0 = sh.sb;
            }
            slots.sync_all();
            Slot& sl = slots[0];
            if (hb0 < sh.nb)  // the host's block CVs beside the GPU's, then the reduce passes
                HIP_CHECK(hipMemcpyAsync(big.lvl[0].as<uint8_t>() + 32 * hb0, sh.cvs.data() + 32 * hb0,
                                         32 * (sh.nb - hb0), hipMemcpyHostToDevice, sl.stream));
            run_checksum_reduce(&big, sl.hashes.as<uint32_t>(), sl.stream);
            HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, 32, hipMemcpyDeviceToHost, sl.stream));
            sl.sync();
            to_hex(sl.host_hashes.u8(), 32, out_hex65 + 65 * i);
            i++;
            continue;
        }
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
                copy_in(k, data + offsets[i] + pos, here);  // exactly the range's bytes: the
                // kernels mask past a message's end, so nothing past it is read from `data`
                const uint32_t wg0 = (uint32_t)(pos / SD_CK_BLOCK);
                const uint32_t wg1 = (uint32_t)std::min<uint64_t>(nb, wg0 + W / SD_CK_BLOCK);
                HIP_CHECK(sdk::launch_ck_leaf(slots[k].staged.as<uint8_t>(), pos, 0, big.d_files(),
                                              big.d_map() + wg0, wg1 - wg0, big.lvl[0].as<uint32_t>(),
                                              slots[k].hashes.as<uint32_t>(), slots[k].stream));
                done_with(k);
            }
            slots.sync_all();
            Slot& sl = slots[0];
            run_checksum_reduce(&big, sl.hashes.as<uint32_t>(), sl.stream);
            HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, 32, hipMemcpyDeviceToHost, sl.stream));
            sl.sync();
            to_hex(sl.host_hashes.u8(), 32, out_hex65 + 65 * i);
            i++;
            continue;
        }
        // the next window: consecutive ranges whose device layout fits W.  Ranges keep their
        // host-relative offsets, so a run of them is one H2D, except that
        //  * a gap that holds a whole page no range touches opens a new run (the copy of a
        //    run reads its gaps: only pages that hold range bytes may be read, since the
        //    caller's buffer can have unmapped holes between ranges);
        //  * a range of a leaf block or more that would start mid-line on the device opens a
        //    new run at the next 128-B line (a mid-line start costs k_ck_leaf 5%, DESIGN.md
        //    §3.2b).
        // Only ascending, non-overlapping ranges open runs.
        runs.clear();
        offs.clear();
        ls.clear();
        uint64_t dev_hi = 0;  // the device layout's padded end
        size_t j = i;
        while (j < n && lens[j] + 128 <= W && (j == i || claim(j))) {
            const uint64_t o = offsets[j], L = lens[j];
            const RunT* r = runs.empty() ? nullptr : &runs.back();
            const bool misaligned = r && (r->dev_lo + (o - r->host_lo)) % SD_STAGE_ALIGN != 0;
            const bool page_gap = r && o >= r->host_end && align_up(r->host_end, 4096) + 4096 <= o;
            const bool open = !r || page_gap || (o >= r->host_end && L >= SD_CK_BLOCK && misaligned);
            if (r && !open && o < r->host_lo) break;  // before its run: the next window takes it
            const uint64_t dev_lo = open ? (r ? align_up(dev_hi, SD_STAGE_ALIGN) : 0) : r->dev_lo;
            const uint64_t host_lo = open ? o : r->host_lo;
            const uint64_t d = dev_lo + (o - host_lo);
            const uint64_t nhi = std::max(dev_hi, align_up(d + L, 64));
            if (j > i && nhi > W) break;  // (a range claimed here and not taken: see below)
            if (open) runs.push_back(RunT{o, o + L, dev_lo});
            else runs.back().host_end = std::max(runs.back().host_end, o + L);
            offs.push_back(d);
            ls.push_back(L);
            dev_hi = nhi;
            j++;
        }
        const int k = cur;
        cur ^= 1;
        harvest(k);
        Slot& sl = slots[k];
        plan_checksum_batch(&sl.ck, offs.data(), ls.data(), j - i, sl.stream);
        sl.hashes.ensure((j - i) * 32);
        sl.host_hashes.ensure((j - i) * 32);
        for (size_t q = 0; q < runs.size(); q++)  // not past a run's last range: `data` may end there
            copy_in(k, data + runs[q].host_lo, runs[q].host_end - runs[q].host_lo, runs[q].dev_lo, q == 0,
                    q + 1 == runs.size());
        run_checksum_batch(&sl.ck, sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        done_with(k);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, (j - i) * 32, hipMemcpyDeviceToHost, sl.stream));
        pend[k] = Pending{i, j, true};
        i = j;
    }
    harvest(0);
    harvest(1);
    if (host.joinable()) host.join();
    if (host_rc != SD_OK) throw sd_failure(host_rc, host_err);
    ctx->checksums_host_bytes.fetch_add(host_bytes.load(), std::memory_order_relaxed);
    ctx->checksums_gpu_bytes.fetch_add(all_bytes - std::min(all_bytes, host_bytes.load()), std::memory_order_relaxed);
    if (learn_route) learn(0);
    return SD_OK;
    SD_GUARD_END
}

int sd_checksums_stats(sd_cas_ctx* ctx, uint64_t out[2]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = ctx->checksums_gpu_bytes.load(std::memory_order_relaxed);
    out[1] = ctx->checksums_host_bytes.load(std::memory_order_relaxed);
    return SD_OK;
    SD_GUARD_END
}

}  // extern "C"
