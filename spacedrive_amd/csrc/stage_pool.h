// stage_pool.h -- persistent host thread pool for the file stager (pread of the byte
// windows generate_cas_id reads, cas.rs:27-58).  run(n, f) calls f(0..n-1) on the pool
// and the calling thread and returns when all are done; start(n, f) / wait() do the same
// on the worker threads only while the caller goes on with other work.  One run at a time
// per pool (a start() holds the pool until its wait()).  A pool grows to the largest thread
// count any call asked for; `limit` makes one run use no more threads than its call asked
// for (the caller included in run()), so a call sized for 3 readers does not run on the 16
// a previous call left in the pool.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

// A worker thread of a pool made with private_fds = true runs on its own copy of the
// process's file-descriptor table, emptied of every inherited descriptor but stdio
// (unshare(CLONE_FILES) + close_range(3, ~0)): every open()/close() of the process
// otherwise serialises on one table lock, and with 16 threads opening and closing one
// file per task that lock -- not the reads -- bounded the stager and the CPU path
// (scripts/stage_bench.c mode 5).  Tasks on such a pool must open and
// close their own files: a descriptor opened by another thread is not valid there.
void private_fd_table();
// Places the calling library thread on the process's preferred CPUs (the GPU's NUMA node,
// set when a context is created; sd_host.h numa_prefer_device_cpus) if they changed since
// this thread last applied them.  Worker threads call it before each run's tasks; a pool's
// caller thread is never moved.
void library_thread_place();

class StagePool {
public:
    explicit StagePool(int nthreads, bool private_fds = false) : private_fds_(private_fds) {
        for (int t = 1; t < nthreads; t++) th_.emplace_back([this, t] { worker(t); });
    }
    bool private_fds() const { return private_fds_; }
    ~StagePool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int threads() const { return (int)th_.size() + 1; }
    void run(size_t n, const std::function<void(size_t)>& f, int limit = 1 << 30) {
        std::lock_guard<std::mutex> serial(run_mu_);
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &f;
            n_ = n;
            next_.store(0);
            busy_ = (int)th_.size();
            active_ = limit;  // workers 1 .. limit-1 take tasks; the caller is thread 0
            gen_++;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [&] { return busy_ == 0; });
        fn_ = nullptr;
    }

    void start(size_t n, std::function<void(size_t)> f, int limit = 1 << 30) {
        run_mu_.lock();  // held until wait(), on this thread
        async_fn_ = std::move(f);
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &async_fn_;
            n_ = n;
            next_.store(0);
            busy_ = (int)th_.size();
            active_ = limit < 1 ? 2 : limit + 1;  // the caller takes no tasks here: workers 1 .. limit
            gen_++;
        }
        cv_.notify_all();
        if (th_.empty()) drain();  // no worker threads: run inline
    }
    void wait() {
        {
            std::unique_lock<std::mutex> g(mu_);
            done_.wait(g, [&] { return busy_ == 0; });
            fn_ = nullptr;
        }
        async_fn_ = nullptr;
        run_mu_.unlock();
    }

private:
    void drain() {
        for (;;) {
            const size_t i = next_.fetch_add(1, std::memory_order_relaxed);
            if (i >= n_) break;
            (*fn_)(i);
        }
    }
    void worker(int idx) {
        if (private_fds_) private_fd_table();
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const bool take = idx < active_;
            g.unlock();
            library_thread_place();
            if (take) drain();
            g.lock();
            if (--busy_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t)>* fn_ = nullptr;
    std::function<void(size_t)> async_fn_;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    int busy_ = 0;
    int active_ = 1 << 30;  // this run's thread limit (worker index < active_ takes tasks)
    uint64_t gen_ = 0;
    bool stop_ = false;
    const bool private_fds_;
};
