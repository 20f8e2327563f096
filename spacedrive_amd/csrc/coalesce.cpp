// coalesce.cpp -- the latency path: single-file calls coalesced into GPU batches.
//
// The reference hashes single files from per-event callers -- the location watcher
// (core/src/location/manager/watcher/utils.rs:235 on create, :393 on update, checksum
// recompute :438-446) and non_indexed::walk (core/src/location/non_indexed.rs:164-187),
// each an independent tokio task calling generate_cas_id(path, size) / file_checksum.
// A GPU round trip per file would waste the device, and libsdcas has no CPU path, so
// concurrent single-file calls meet here: a dispatcher thread per context waits for the
// first request, keeps collecting for a short window (tuning "coalesce_window_us",
// default 200) or until "coalesce_max" requests (default 4096) are queued, then stages
// the whole batch with the pread pool (sd_cas_stage_files) into pinned memory and hashes
// it with one sd_cas_ids / sd_file_checksums call.  Requests that arrive meanwhile form
// the next batch, so a busy watcher is served at batch throughput and an idle one at
// window + one small batch of latency.  Each caller blocks only on its own request.
#include <hip/hip_runtime.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sd_internal.h"

struct sd_coalescer {
    struct Req {
        int kind;  // 0 = cas id, 1 = checksum
        const char* path;
        uint64_t size;
        char* out;
        int32_t* status;
        int rc = SD_OK;
        std::string err;
        bool done = false;
    };
    sd_cas_ctx* ctx;
    std::mutex mu;
    std::condition_variable work, done;
    std::deque<Req*> q;
    bool stop = false;
    std::thread th;
    uint64_t n_requests = 0, n_batches = 0, max_batch = 0;
    void* pinned = nullptr;
    uint64_t pinned_bytes = 0;

    explicit sd_coalescer(sd_cas_ctx* c) : ctx(c) { th = std::thread([this] { loop(); }); }
    ~sd_coalescer() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        work.notify_all();
        if (th.joinable()) th.join();
        if (pinned) sd_cas_host_free(ctx, pinned);
    }

    int submit(Req& r) {
        std::unique_lock<std::mutex> g(mu);
        if (stop) return SD_ERR_INVALID;
        q.push_back(&r);
        n_requests++;
        work.notify_one();
        done.wait(g, [&] { return r.done; });
        return r.rc;
    }

    void fail(std::vector<Req*>& batch, int rc) {
        const char* m = sd_cas_last_error();
        for (Req* r : batch) {
            r->rc = rc;
            r->err = m;
        }
    }

    void run_cas(std::vector<Req*>& batch) {
        const size_t n = batch.size();
        std::vector<uint64_t> sizes(n);
        std::vector<const char*> paths(n);
        for (size_t i = 0; i < n; i++) {
            sizes[i] = batch[i]->size;
            paths[i] = batch[i]->path;
        }
        std::vector<sd_extent> ext(n);
        uint64_t total = 0;
        int rc = sd_cas_stage_plan(sizes.data(), n, ext.data(), &total);
        if (rc == SD_OK && total > pinned_bytes) {
            if (pinned) sd_cas_host_free(ctx, pinned);
            pinned = nullptr;
            pinned_bytes = 0;
            rc = sd_cas_host_alloc(ctx, total * 2, &pinned);
            if (rc == SD_OK) pinned_bytes = total * 2;
        }
        std::vector<int32_t> st(n, SD_FILE_OK);
        std::vector<char> hex(17 * n, 0);
        const int threads = (int)std::min<size_t>(16, n);
        if (rc == SD_OK)
            rc = sd_cas_stage_files(paths.data(), ext.data(), n, (uint8_t*)pinned, st.data(), threads);
        if (rc == SD_OK) rc = sd_cas_ids(ctx, (const uint8_t*)pinned, total, ext.data(), n, hex.data(), st.data());
        if (rc != SD_OK) return fail(batch, rc);
        for (size_t i = 0; i < n; i++) {
            *batch[i]->status = st[i];
            if (st[i] == SD_FILE_OK) memcpy(batch[i]->out, &hex[17 * i], 17);
        }
    }

    void run_checksums(std::vector<Req*>& batch) {
        const size_t n = batch.size();
        std::vector<const char*> paths(n);
        for (size_t i = 0; i < n; i++) paths[i] = batch[i]->path;
        std::vector<int32_t> st(n, SD_FILE_OK);
        std::vector<char> hex(65 * n, 0);
        const int rc = sd_file_checksums(ctx, paths.data(), n, hex.data(), st.data());
        if (rc != SD_OK) return fail(batch, rc);
        for (size_t i = 0; i < n; i++) {
            *batch[i]->status = st[i];
            if (st[i] == SD_FILE_OK) memcpy(batch[i]->out, &hex[65 * i], 65);
        }
    }

    void loop() {
        std::unique_lock<std::mutex> g(mu);
        for (;;) {
            work.wait(g, [&] { return stop || !q.empty(); });
            if (q.empty() && stop) return;
            const size_t cap = (size_t)std::max(1, tuning_get(SD_TUNE_COALESCE_MAX));
            const auto deadline =
                std::chrono::steady_clock::now() + std::chrono::microseconds(std::max(0, tuning_get(SD_TUNE_COALESCE_US)));
            while (!stop && q.size() < cap && work.wait_until(g, deadline) != std::cv_status::timeout) {
            }
            std::vector<Req*> cas, ck;
            while (!q.empty() && cas.size() + ck.size() < cap) {
                Req* r = q.front();
                q.pop_front();
                (r->kind == 0 ? cas : ck).push_back(r);
            }
            n_batches++;
            max_batch = std::max<uint64_t>(max_batch, cas.size() + ck.size());
            g.unlock();
            if (!cas.empty()) run_cas(cas);
            if (!ck.empty()) run_checksums(ck);
            g.lock();
            for (Req* r : cas) r->done = true;
            for (Req* r : ck) r->done = true;
            done.notify_all();
        }
    }
};

sd_coalescer* coalescer_create(sd_cas_ctx* ctx) { return new sd_coalescer(ctx); }
void coalescer_destroy(sd_coalescer* c) { delete c; }

int coalescer_submit(sd_coalescer* c, int kind, const char* path, uint64_t size, char* out, int32_t* status,
                     std::string* err) {
    sd_coalescer::Req r;
    r.kind = kind;
    r.path = path;
    r.size = size;
    r.out = out;
    r.status = status;
    const int rc = c->submit(r);
    if (rc != SD_OK) *err = r.err;
    return rc;
}

void coalescer_stats(sd_coalescer* c, uint64_t out[3]) {
    std::lock_guard<std::mutex> g(c->mu);
    out[0] = c->n_requests;
    out[1] = c->n_batches;
    out[2] = c->max_batch;
}
