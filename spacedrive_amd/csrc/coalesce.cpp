// coalesce.cpp -- the latency path: single-file calls coalesced into GPU batches.
//
// The reference hashes single files from per-event callers -- the location watcher
// (core/src/location/manager/watcher/utils.rs:235 on create, :393 on update, checksum
// recompute :438-446) and non_indexed::walk (core/src/location/non_indexed.rs:164-187),
// each an independent tokio task calling generate_cas_id(path, size) / file_checksum.
// Policy: one GPU round trip per file costs more than hashing
// the file on the host, so while fewer than "latency_cpu_max" (default 16) single-file
// calls are in flight on the context, a call is hashed on its own thread by the CPU path
// (cpu_blake3.cpp).  Beyond that, concurrent calls meet here: a dispatcher thread per
// context waits for the first request, keeps collecting for a short window (tuning
// "coalesce_window_us", default 200) or until "coalesce_max" requests (default 4096) are
// queued, then hashes the whole batch with one sd_cas_ids_files / sd_file_checksums
// call -- whose batch policies pick the route: with the defaults ("batch_cpu_max" 4096,
// "checksum_cpu_max" all) a coalesced batch is hashed on the CPU path's 16 threads, which
// bounds the threads a burst of callers occupies; with the policies at 0 it goes to the
// GPU.  Requests that arrive meanwhile form the next batch, so a busy watcher is served
// at batch throughput and an idle one at CPU latency.  Each caller blocks only on its own
// request.
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sd_host.h"

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
    uint64_t n_requests = 0, n_batches = 0, max_batch = 0, n_cpu = 0;
    uint64_t inflight = 0;  // single-file calls inside submit(), either route

    explicit sd_coalescer(sd_cas_ctx* c) : ctx(c) { th = std::thread([this] { loop(); }); }
    ~sd_coalescer() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        work.notify_all();
        if (th.joinable()) th.join();
    }

    int submit(Req& r) {
        std::unique_lock<std::mutex> g(mu);
        if (stop) return SD_ERR_INVALID;
        n_requests++;
        const int cpu_max = tuning_get(SD_TUNE_LATENCY_CPU_MAX);
        if (cpu_max > 0 && inflight < (uint64_t)cpu_max) {  // few callers: hash on this thread
            inflight++;
            n_cpu++;
            g.unlock();
            *r.status = r.kind == 0 ? cpu_cas_id_file(r.path, r.size, r.out) : cpu_checksum_file(r.path, r.out);
            g.lock();
            inflight--;
            return SD_OK;
        }
        inflight++;
        q.push_back(&r);
        work.notify_one();
        done.wait(g, [&] { return r.done; });
        inflight--;
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
        std::vector<int32_t> st(n, SD_FILE_OK);
        std::vector<char> hex(17 * n, 0);
        const int rc = sd_cas_ids_files(ctx, paths.data(), sizes.data(), n, hex.data(), st.data(),
                                        (int)std::min<size_t>(16, n));
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
                // system_clock: libstdc++ waits on it with pthread_cond_timedwait, which every
                // ThreadSanitizer runtime intercepts (a steady_clock wait becomes
                // pthread_cond_clockwait, which GCC 11's does not: false "double lock"
                // reports); a wall-clock step can only shorten or stretch one window
                std::chrono::system_clock::now() + std::chrono::microseconds(std::max(0, tuning_get(SD_TUNE_COALESCE_US)));
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

void coalescer_stats(sd_coalescer* c, uint64_t out[4]) {
    std::lock_guard<std::mutex> g(c->mu);
    out[0] = c->n_requests;
    out[1] = c->n_batches;
    out[2] = c->max_batch;
    out[3] = c->n_cpu;
}
