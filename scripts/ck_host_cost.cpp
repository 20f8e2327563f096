// ck_host_cost.cpp -- host CPU cost per byte of the validator's paths from the page cache
// (VERDICT r3 item 4): what it costs the host to hand file bytes to the GPU, against what
// it costs to read and hash them on the CPU (sd_file_checksums' two routes, hash.rs:10-24).
//
// Files: NF x FL bytes written to /dev/shm (tmpfs: every read is a page-cache copy), then
// every mode reads all of them with T threads in 64 MiB units claimed from one cursor:
//   read_pinned    1 MiB preads straight into a pinned window (the GPU route's readers today)
//   read_hot_nt    256 KiB preads into a per-thread cache-resident buffer, then streaming
//                  (non-temporal) stores into the pinned window (the cas stager's copy)
//   read_hash      1 MiB preads into a per-thread buffer + BLAKE3 of it on this thread
//                  (sd_cpu_checksums, one thread: the CPU path's work per block)
//   read_hot       256 KiB preads into the per-thread buffer only (the read floor)
//   hash_hot       BLAKE3 of a cache-resident 1 MiB buffer, no read (the hash alone)
//   *_dma          the same, each filled 64 MiB unit DMA'd to the device (hipMemcpyAsync on
//                  the thread's stream, double-buffered): the GPU route's host side at PCIe rate
//   zero_copy_dma  no host copy at all: each 64 MiB unit of the file mmap'ed read-only,
//                  page-locked in place (hipHostRegister, read-only) and DMA'd from the page
//                  cache itself; the next unit is registered while the previous one's DMA runs
//   hybrid_g       g threads read_hot_nt_dma (or zero_copy_dma) + T-g threads read_hash on
//                  one shared cursor: sd_file_checksums split between the routes
// Each line: wall GB/s, and host CPU time per byte (every thread's CLOCK_THREAD_CPUTIME_ID,
// summed) in ns/B and in cycles/B at the clock given by --ghz (the box's nominal clock).
//
// Build (on the CPU container; runs on the GPU box):
//   hipcc -O2 -std=c++17 -mavx2 -o scripts/ck_host_cost scripts/ck_host_cost.cpp \
//         -Lspacedrive_amd -lsdcas -Wl,-rpath,'$ORIGIN/../spacedrive_amd' -lpthread
// Run: scripts/ck_host_cost [NF=32] [FL_MiB=256] [ghz=2.4] [quick|bound|wc|cold]  -> JSON lines on stdout
// (cold: SD_CK_DIR=<dir on a real filesystem>; every leg evicts the files first)
// ("quick": read_hash, read_hot_nt_dma and the hot_nt split at 16 threads only, for A/Bs
// such as scripts/numa_probe.sh's thread placements; "bound", VERDICT r4 item 3: what bounds
// the split -- STREAM-like host DRAM legs on 16 threads (read, non-temporal write, copy), the
// split's own memory traffic with the CPU half's hashing removed (hybrid_nohash: g threads
// of the GPU route's read_hot_nt + DMA, 16 - g of read_hot), the split itself (hybrid_hot_nt)
// and its CPU half alone on 16 - g threads, each line with its DRAM passes per byte moved:
// read_hot / read_hash 1 (the page-cache read; the per-thread buffer stays in cache),
// read_hot_nt + DMA 3 (page-cache read, streaming write to pinned memory, the device's DMA
// read), stream_read 1, stream_nt_write 1, stream_copy_nt 2)
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

extern "C" int sd_cpu_checksums(const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, size_t n,
                                uint8_t* out_hash32, int nthreads);

namespace {
constexpr uint64_t UNIT = 64ull << 20, MiB = 1ull << 20, HOT = 256ull << 10;
int NF = 32;
uint64_t FL = 256 * MiB;
double GHZ = 2.4;
std::string DIR = getenv("SD_CK_DIR") ? getenv("SD_CK_DIR") : "/dev/shm/sd_ckcost";

#define HIPOK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(3);                                                              \
        }                                                                         \
    } while (0)

double thread_cpu_s() {
    timespec t;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

void nt_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
    for (uint64_t o = 0; o < n; o += 64) {
        const __m256i a = _mm256_load_si256(reinterpret_cast<const __m256i*>(src + o));
        const __m256i b = _mm256_load_si256(reinterpret_cast<const __m256i*>(src + o + 32));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + o), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + o + 32), b);
    }
    _mm_sfence();
}

int64_t pread_all(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
    uint64_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, dst + got, n - got, (off_t)(off + got));
        if (r <= 0) return r < 0 ? -1 : (int64_t)got;
        got += (uint64_t)r;
    }
    return (int64_t)got;
}

std::string path_of(int f) { return DIR + "/f" + std::to_string(f); }

void make_files() {
    mkdir(DIR.c_str(), 0700);
    std::vector<std::thread> th;
    for (int t = 0; t < 8; t++)
        th.emplace_back([t] {
            std::vector<uint64_t> buf(MiB / 8);
            for (int f = t; f < NF; f += 8) {
                const int fd = open(path_of(f).c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0600);
                uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(f + 1);
                for (uint64_t o = 0; o < FL; o += MiB) {
                    for (auto& w : buf) {  // xorshift64*: incompressible, cheap
                        x ^= x >> 12;
                        x ^= x << 25;
                        x ^= x >> 27;
                        w = x * 0x2545F4914F6CDD1Dull;
                    }
                    if (write(fd, buf.data(), MiB) != (ssize_t)MiB) exit(4);
                }
                close(fd);
            }
        });
    for (auto& x : th) x.join();
}

// drop every file's pages from the page cache (written files are fsync'ed first): the
// next reads go to the storage ("cold" mode)
void evict_all() {
    for (int f = 0; f < NF; f++) {
        const int fd = open(path_of(f).c_str(), O_RDONLY);
        if (fd < 0) exit(8);
        fsync(fd);
        posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
        close(fd);
    }
}

struct Res {
    double wall = 0, cpu = 0;
    uint64_t bytes = 0;
    uint64_t bytes_dma = 0;  // of which the threads that DMA'd them to the device moved
};

enum Kind { READ_PINNED, READ_HOT_NT, READ_HASH, READ_HOT, HASH_HOT, ZERO_COPY, READ_PINNED_WC, READ_HASH_DIRECT,
            READ_PINNED_DIRECT };

// STREAM-like legs over an anonymous buffer, T threads, each its contiguous slice (first
// touched by that thread): kind 0 = read (AVX2 loads, summed), 1 = non-temporal write,
// 2 = copy with non-temporal stores (a read + a write per byte).  Returns bytes moved per
// second counting each byte once (a copy of n bytes = n).
double stream_leg(int kind, int T, uint8_t* a, uint8_t* b, uint64_t len, int reps) {
    std::vector<std::thread> th;
    std::atomic<uint64_t> sink{0};
    const uint64_t per = len / (uint64_t)T / 4096 * 4096;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            uint8_t* x = a + per * (uint64_t)t;
            uint8_t* y = b + per * (uint64_t)t;
            __m256i acc = _mm256_setzero_si256();
            for (int r = 0; r < reps; r++) {
                if (kind == 0) {
                    for (uint64_t o = 0; o < per; o += 64) {
                        acc = _mm256_add_epi64(acc, _mm256_load_si256(reinterpret_cast<const __m256i*>(x + o)));
                        acc = _mm256_add_epi64(acc, _mm256_load_si256(reinterpret_cast<const __m256i*>(x + o + 32)));
                    }
                } else if (kind == 1) {
                    const __m256i v = _mm256_set1_epi64x(r + 1);
                    for (uint64_t o = 0; o < per; o += 64) {
                        _mm256_stream_si256(reinterpret_cast<__m256i*>(x + o), v);
                        _mm256_stream_si256(reinterpret_cast<__m256i*>(x + o + 32), v);
                    }
                    _mm_sfence();
                } else {
                    nt_copy(y, x, per);
                }
            }
            sink += (uint64_t)_mm256_extract_epi64(acc, 0);
        });
    for (auto& x : th) x.join();
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return (double)per * T * reps / wall / 1e9 + (sink.load() == 42 ? 1e-12 : 0.0);
}
const char* NAMES[] = {"read_pinned", "read_hot_nt", "read_hash", "read_hot", "hash_hot", "zero_copy", "read_pinned_wc",
                       "read_hash_direct", "read_pinned_direct"};

struct ThreadBufs {
    uint8_t* pinned[2] = {nullptr, nullptr};  // two UNIT windows (double buffer for the DMA)
    uint8_t* wc[2] = {nullptr, nullptr};      // the same, write-combined ("wc" mode)
    uint8_t* hot = nullptr;                   // 1 MiB, cache-resident working buffer
    void* dev = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool pending[2] = {false, false};
    void* map[2] = {nullptr, nullptr};  // zero copy: the registered mapping behind ev[k]
};

// zero copy: release mapping k once its DMA is done
void zc_release(ThreadBufs& B, int k) {
    if (!B.map[k]) return;
    HIPOK(hipEventSynchronize(B.ev[k]));
    HIPOK(hipHostUnregister(B.map[k]));
    munmap(B.map[k], UNIT);
    B.map[k] = nullptr;
    B.pending[k] = false;
}

// runs `kinds[t]` on thread t (dma[t]: DMA each filled unit) over all units of all files
Res run(const std::vector<int>& kinds, const std::vector<int>& dma, std::vector<ThreadBufs>& bufs) {
    const int T = (int)kinds.size();
    const uint64_t per_file = FL / UNIT, units = per_file * (uint64_t)NF;
    std::atomic<uint64_t> cursor{0};
    std::vector<double> cpu(T, 0);
    std::atomic<uint64_t> total{0}, total_dma{0};
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            const double c0 = thread_cpu_s();
            ThreadBufs& B = bufs[t];
            int b = 0;
            uint8_t hash[32];
            const int kind = kinds[t];
            for (;;) {
                uint64_t u;
                if (kind == HASH_HOT) {
                    u = cursor.fetch_add(1);
                    if (u >= units) break;
                    for (uint64_t o = 0; o < UNIT; o += MiB) {
                        const uint64_t off = 0, len = MiB;
                        sd_cpu_checksums(B.hot, &off, &len, 1, hash, 1);
                    }
                    total += UNIT;
                    continue;
                }
                u = cursor.fetch_add(1);
                if (u >= units) break;
                const int f = (int)(u / per_file);
                const uint64_t base = (u % per_file) * UNIT;
                const bool direct = kind == READ_HASH_DIRECT || kind == READ_PINNED_DIRECT;
                const int fd = open(path_of(f).c_str(), O_RDONLY | (direct ? O_DIRECT : 0));
                if (fd < 0) exit(5);
                if (kind == ZERO_COPY) {  // map + pin this unit, DMA it, release the one before
                    void* m = mmap(nullptr, UNIT, PROT_READ, MAP_SHARED, fd, (off_t)base);
                    close(fd);
                    if (m == MAP_FAILED) exit(7);
                    zc_release(B, b);  // two units in flight at most
                    HIPOK(hipHostRegister(m, UNIT, hipHostRegisterReadOnly));
                    HIPOK(hipMemcpyAsync(B.dev, m, UNIT, hipMemcpyHostToDevice, B.s));
                    HIPOK(hipEventRecord(B.ev[b], B.s));
                    B.map[b] = m;
                    B.pending[b] = true;
                    b ^= 1;
                    total += UNIT;
                    continue;
                }
                if (dma[t] && B.pending[b]) {
                    HIPOK(hipEventSynchronize(B.ev[b]));
                    B.pending[b] = false;
                }
                uint8_t* win = kind == READ_PINNED_WC ? B.wc[b] : B.pinned[b];
                for (uint64_t o = 0; o < UNIT;) {
                    switch (kind) {
                        case READ_PINNED:
                        case READ_PINNED_WC:
                        case READ_PINNED_DIRECT:
                            if (pread_all(fd, win + o, MiB, base + o) != (int64_t)MiB) exit(6);
                            o += MiB;
                            break;
                        case READ_HOT_NT:
                            if (pread_all(fd, B.hot, HOT, base + o) != (int64_t)HOT) exit(6);
                            nt_copy(win + o, B.hot, HOT);
                            o += HOT;
                            break;
                        case READ_HASH:
                        case READ_HASH_DIRECT: {
                            if (pread_all(fd, B.hot, MiB, base + o) != (int64_t)MiB) exit(6);
                            const uint64_t off = 0, len = MiB;
                            sd_cpu_checksums(B.hot, &off, &len, 1, hash, 1);
                            o += MiB;
                            break;
                        }
                        case READ_HOT:
                            if (pread_all(fd, B.hot, HOT, base + o) != (int64_t)HOT) exit(6);
                            o += HOT;
                            break;
                    }
                }
                close(fd);
                if (dma[t]) {
                    HIPOK(hipMemcpyAsync(B.dev, win, UNIT, hipMemcpyHostToDevice, B.s));
                    HIPOK(hipEventRecord(B.ev[b], B.s));
                    B.pending[b] = true;
                    b ^= 1;
                    total_dma += UNIT;
                }
                total += UNIT;
            }
            for (int k = 0; k < 2; k++) {
                zc_release(B, k);
                if (B.pending[k]) {
                    HIPOK(hipEventSynchronize(B.ev[k]));
                    B.pending[k] = false;
                }
            }
            cpu[t] = thread_cpu_s() - c0;
        });
    for (auto& x : th) x.join();
    Res r;
    r.wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (double c : cpu) r.cpu += c;
    r.bytes = total.load();
    r.bytes_dma = total_dma.load();
    return r;
}

void report(const char* name, int T, int g, const Res& r) {
    const double ns_b = r.cpu * 1e9 / (double)r.bytes;
    // DRAM passes: a byte DMA'd after read_hot_nt 3 (page-cache read, streaming write, DMA
    // read); any other byte 1 (the page-cache read) -- read_pinned's DMA'd bytes are not
    // counted this way (its pread writes the pinned window through the cache)
    const double dram = ((double)r.bytes_dma * 3 + (double)(r.bytes - r.bytes_dma)) / r.wall / 1e9;
    printf("{\"mode\": \"%s\", \"threads\": %d, \"gpu_route_threads\": %d, \"GBps\": %.2f, \"cpu_ns_per_byte\": %.4f, "
           "\"cycles_per_byte\": %.3f, \"cpu_s\": %.3f, \"wall_s\": %.3f, \"bytes\": %llu, \"gpu_share\": %.3f, "
           "\"dram_GBps\": %.2f}\n",
           name, T, g, (double)r.bytes / r.wall / 1e9, ns_b, ns_b * GHZ, r.cpu, r.wall, (unsigned long long)r.bytes,
           r.bytes ? (double)r.bytes_dma / (double)r.bytes : 0.0, dram);
    fflush(stdout);
}
}  // namespace

int main(int argc, char** argv) {
    if (argc > 1) NF = atoi(argv[1]);
    if (argc > 2) FL = (uint64_t)atoi(argv[2]) * MiB;
    if (argc > 3) GHZ = atof(argv[3]);
    const bool quick = argc > 4 && strcmp(argv[4], "quick") == 0;
    if (FL % UNIT) FL = (FL / UNIT + 1) * UNIT;
    make_files();
    const int TMAX = 16;
    std::vector<ThreadBufs> bufs(TMAX);
    for (auto& B : bufs) {
        for (int k = 0; k < 2; k++) {
            HIPOK(hipHostMalloc(reinterpret_cast<void**>(&B.pinned[k]), UNIT, hipHostMallocDefault));
            memset(B.pinned[k], 0, UNIT);
            HIPOK(hipEventCreateWithFlags(&B.ev[k], hipEventDisableTiming));
        }
        B.hot = static_cast<uint8_t*>(aligned_alloc(4096, MiB));
        memset(B.hot, 1, MiB);
        HIPOK(hipMalloc(&B.dev, UNIT));
        HIPOK(hipStreamCreateWithFlags(&B.s, hipStreamNonBlocking));
    }
    // page cache warm (the files were just written) -- one untimed pass anyway
    run(std::vector<int>(TMAX, READ_HOT), std::vector<int>(TMAX, 0), bufs);
    const bool bound = argc > 4 && strcmp(argv[4], "bound") == 0;
    if (argc > 4 && strcmp(argv[4], "cold") == 0) {
        // (round 5) every leg from cold files (evicted before it runs, SD_CK_DIR on a real
        // filesystem): buffered preads (today's routes) against O_DIRECT ones -- into the
        // cache-resident buffer for the CPU path's hashing, straight into the pinned window
        // (the DMA source: no host copy at all) for the GPU route
        auto leg = [&](const char* name, int T, int g, std::vector<int> kinds, std::vector<int> dma) {
            evict_all();
            report(name, T, g, run(kinds, dma, bufs));
        };
        for (int rep = 0; rep < 3; rep++) {
            leg("read_hash", TMAX, 0, std::vector<int>(TMAX, READ_HASH), std::vector<int>(TMAX, 0));
            leg("read_hash_direct", TMAX, 0, std::vector<int>(TMAX, READ_HASH_DIRECT), std::vector<int>(TMAX, 0));
            leg("read_hot", TMAX, 0, std::vector<int>(TMAX, READ_HOT), std::vector<int>(TMAX, 0));
            for (int g : {4, 8}) {
                leg("read_hot_nt_dma", g, g, std::vector<int>(g, READ_HOT_NT), std::vector<int>(g, 1));
                leg("read_pinned_direct_dma", g, g, std::vector<int>(g, READ_PINNED_DIRECT), std::vector<int>(g, 1));
            }
            for (int g : {6}) {
                std::vector<int> k1(TMAX, READ_HASH), d1(TMAX, 0), k2(TMAX, READ_HASH_DIRECT), d2(TMAX, 0);
                for (int t = 0; t < g; t++) k1[t] = READ_HOT_NT, d1[t] = 1, k2[t] = READ_PINNED_DIRECT, d2[t] = 1;
                leg("hybrid_hot_nt", TMAX, g, k1, d1);
                leg("hybrid_direct", TMAX, g, k2, d2);
            }
        }
        for (int f = 0; f < NF; f++) unlink(path_of(f).c_str());
        rmdir(DIR.c_str());
        return 0;
    }
    if (argc > 4 && strcmp(argv[4], "wc") == 0) {
        // (round 5) preads straight into write-combined pinned windows: one pass, no
        // read-for-ownership of the destination, against read_pinned (write-back windows)
        // and read_hot_nt (a cache-resident bounce buffer + streaming stores)
        for (auto& B : bufs)
            for (int k = 0; k < 2; k++) {
                HIPOK(hipHostMalloc(reinterpret_cast<void**>(&B.wc[k]), UNIT, hipHostMallocWriteCombined));
                memset(B.wc[k], 0, UNIT);
            }
        for (int rep = 0; rep < 3; rep++) {
            for (int kind : {READ_PINNED, READ_HOT_NT, READ_PINNED_WC})
                report(NAMES[kind], 1, 0, run(std::vector<int>(1, kind), std::vector<int>(1, 0), bufs));
            for (int kind : {READ_PINNED, READ_HOT_NT, READ_PINNED_WC}) {
                const std::string name = std::string(NAMES[kind]) + "_dma";
                for (int T : {4, 6})
                    report(name.c_str(), T, T, run(std::vector<int>(T, kind), std::vector<int>(T, 1), bufs));
            }
            for (int gk : {READ_HOT_NT, READ_PINNED_WC}) {
                std::vector<int> kinds(TMAX, READ_HASH), dma(TMAX, 0);
                for (int t = 0; t < 6; t++) kinds[t] = gk, dma[t] = 1;
                report(gk == READ_HOT_NT ? "hybrid_hot_nt" : "hybrid_pinned_wc", TMAX, 6, run(kinds, dma, bufs));
            }
        }
        for (int f = 0; f < NF; f++) unlink(path_of(f).c_str());
        rmdir(DIR.c_str());
        return 0;
    }
    if (bound) {
        const uint64_t SLEN = 4ull << 30;  // two 4 GiB anonymous buffers: far past the caches
        uint8_t* sa = static_cast<uint8_t*>(aligned_alloc(4096, SLEN));
        uint8_t* sb = static_cast<uint8_t*>(aligned_alloc(4096, SLEN));
        stream_leg(1, TMAX, sa, sb, SLEN, 1);  // first touch by the threads that use the slices
        stream_leg(1, TMAX, sb, sa, SLEN, 1);
        for (int rep = 0; rep < 3; rep++) {
            for (int T : {8, 16}) {
                const char* names[3] = {"stream_read", "stream_nt_write", "stream_copy_nt"};
                const int passes[3] = {1, 1, 2};
                for (int k = 0; k < 3; k++) {
                    const double g = stream_leg(k, T, sa, sb, SLEN, 3);
                    printf("{\"mode\": \"%s\", \"threads\": %d, \"GBps\": %.2f, \"dram_passes\": %d, "
                           "\"dram_GBps\": %.2f, \"rep\": %d}\n", names[k], T, g, passes[k], g * passes[k], rep);
                    fflush(stdout);
                }
            }
            for (int g : {3, 4, 6}) {
                std::vector<int> kinds(TMAX, READ_HOT), dma(TMAX, 0);
                for (int t = 0; t < g; t++) kinds[t] = READ_HOT_NT, dma[t] = 1;
                report("hybrid_nohash", TMAX, g, run(kinds, dma, bufs));
                std::vector<int> kinds2(TMAX, READ_HASH), dma2(TMAX, 0);
                for (int t = 0; t < g; t++) kinds2[t] = READ_HOT_NT, dma2[t] = 1;
                report("hybrid_hot_nt", TMAX, g, run(kinds2, dma2, bufs));
                report("read_hash", TMAX - g, 0, run(std::vector<int>(TMAX - g, READ_HASH), std::vector<int>(TMAX - g, 0), bufs));
                report("read_hot_nt_dma", g, g, run(std::vector<int>(g, READ_HOT_NT), std::vector<int>(g, 1), bufs));
            }
            report("read_hot", TMAX, 0, run(std::vector<int>(TMAX, READ_HOT), std::vector<int>(TMAX, 0), bufs));
            report("read_hash", TMAX, 0, run(std::vector<int>(TMAX, READ_HASH), std::vector<int>(TMAX, 0), bufs));
        }
        free(sa);
        free(sb);
        for (int f = 0; f < NF; f++) unlink(path_of(f).c_str());
        rmdir(DIR.c_str());
        return 0;
    }
    if (quick) {
        for (int rep = 0; rep < 3; rep++) {
            report("read_hash", TMAX, 0, run(std::vector<int>(TMAX, READ_HASH), std::vector<int>(TMAX, 0), bufs));
            report("read_hot_nt_dma", 8, 8, run(std::vector<int>(8, READ_HOT_NT), std::vector<int>(8, 1), bufs));
            std::vector<int> kinds(TMAX, READ_HASH), dma(TMAX, 0);
            for (int t = 0; t < 4; t++) kinds[t] = READ_HOT_NT, dma[t] = 1;
            report("hybrid_hot_nt", TMAX, 4, run(kinds, dma, bufs));
        }
        for (int f = 0; f < NF; f++) unlink(path_of(f).c_str());
        rmdir(DIR.c_str());
        return 0;
    }
    for (int T : {1, 4, 8, 16})
        for (int kind : {READ_PINNED, READ_HOT_NT, READ_HASH, READ_HOT, HASH_HOT})
            report(NAMES[kind], T, 0, run(std::vector<int>(T, kind), std::vector<int>(T, 0), bufs));
    for (int T : {2, 4, 8})  // the GPU route's host side at PCIe rate
        for (int kind : {READ_PINNED, READ_HOT_NT}) {
            const std::string name = std::string(NAMES[kind]) + "_dma";
            report(name.c_str(), T, T, run(std::vector<int>(T, kind), std::vector<int>(T, 1), bufs));
        }
    for (int T : {1, 2, 4, 8})  // the GPU route with no host copy
        report("zero_copy_dma", T, T, run(std::vector<int>(T, ZERO_COPY), std::vector<int>(T, 1), bufs));
    for (int g : {0, 2, 3, 4, 6}) {  // 16 threads split between the routes
        for (int gk : {READ_PINNED, READ_HOT_NT, ZERO_COPY}) {
            if (g == 0 && gk != READ_PINNED) continue;
            std::vector<int> kinds(TMAX, READ_HASH), dma(TMAX, 0);
            for (int t = 0; t < g; t++) {
                kinds[t] = gk;
                dma[t] = 1;
            }
            const std::string name = std::string("hybrid_") +
                                     (gk == READ_PINNED ? "pinned" : gk == READ_HOT_NT ? "hot_nt" : "zero_copy");
            report(name.c_str(), TMAX, g, run(kinds, dma, bufs));
        }
    }
    for (int f = 0; f < NF; f++) unlink(path_of(f).c_str());
    rmdir(DIR.c_str());
    return 0;
}
