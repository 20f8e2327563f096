// host_selftest.cpp -- the GPU-free half of libsdcas under ASan + UBSan and TSan
// (`make sanitize`; SURVEY.md §5 "ASan/UBSan builds of the C++ host lib").
//
// Exercises, with real threads and real files: the batch planners (plan_whole_items,
// plan_checksum), the stager with generate_cas_id's read semantics (stage_one, cas.rs:
// 23-62), the sequential and parallel message readers (MsgSource, hash.rs:14-20), the
// stager thread pool (StagePool, incl. the context's grow-while-in-use pattern), the CPU
// path (CpuHasher, sd_cpu_*), and the latency-path coalescer with both of its routes.  The
// coalescer's GPU batch calls are stubbed here with the CPU path (no device in this
// build); everything else is the library's own code.  Prints "host_selftest: ok" or the
// failed checks and exits non-zero.
#include <dirent.h>
#include <sched.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "sd_host.h"

// ---- the two GPU entry points coalesce.cpp calls, stubbed with the CPU path
extern "C" int sd_cas_ids_files(sd_cas_ctx*, const char* const* paths, const uint64_t* sizes, size_t n,
                                char* out_hex17, int32_t* status, int nthreads) {
    return sd_cpu_cas_ids_files(paths, sizes, n, out_hex17, status, nthreads);
}
extern "C" int sd_file_checksums(sd_cas_ctx*, const char* const* paths, size_t n, char* out_hex65, int32_t* status) {
    return sd_cpu_file_checksums(paths, n, out_hex65, status, 4);
}

namespace {

std::atomic<int> g_fail{0};
#define CHECK(c)                                                                \
    do {                                                                        \
        if (!(c)) {                                                             \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);        \
            g_fail++;                                                           \
        }                                                                       \
    } while (0)

std::string hex(const uint8_t* p, int n) {
    char buf[129];
    hex_lower(p, n, buf);
    return buf;
}

std::vector<uint8_t> content(uint64_t seed, size_t n) {
    std::vector<uint8_t> v(n);
    std::mt19937_64 g(seed);
    for (size_t i = 0; i < n; i += 8) {
        const uint64_t x = g();
        memcpy(v.data() + i, &x, std::min<size_t>(8, n - i));
    }
    return v;
}

std::string g_dir;
std::string write_file(const std::string& name, const std::vector<uint8_t>& data) {
    const std::string p = g_dir + "/" + name;
    FILE* f = fopen(p.c_str(), "wb");
    if (!f) abort();
    if (!data.empty() && fwrite(data.data(), 1, data.size(), f) != data.size()) abort();
    fclose(f);
    return p;
}

// ------------------------------------------------------------------ BLAKE3
void test_blake3() {
    uint8_t h[32];
    cpu_blake3(nullptr, 0, h);
    CHECK(hex(h, 32) == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262");
    cpu_blake3((const uint8_t*)"abc", 3, h);
    CHECK(hex(h, 32) == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85");
    // incremental updates at arbitrary split points == one shot
    std::mt19937 g(7);
    for (size_t n : {1u, 64u, 1024u, 1025u, 2048u, 16384u, 16385u, 57352u, 300001u, 1u << 21}) {
        const auto d = content(n, n);
        uint8_t one[32], inc[32];
        cpu_blake3(d.data(), n, one);
        CpuHasher hs;
        size_t pos = 0;
        while (pos < n) {
            const size_t k = std::min<size_t>(n - pos, 1 + g() % 5000);
            hs.update(d.data() + pos, k);
            pos += k;
        }
        hs.finalize(inc);
        CHECK(memcmp(one, inc, 32) == 0);
    }
    // batches: the chunks of many messages packed across the SIMD lanes == one at a time;
    // every length 0..2100 in steps of 3 (every block and chunk boundary class), cas
    // message sizes, and two past the batch's 1 MiB limit, shuffled, from one buffer
    std::vector<uint64_t> lens;
    for (uint64_t n = 0; n <= 2100; n += 3) lens.push_back(n);
    for (uint64_t n : {1024ull, 2048ull, 57352ull, 102408ull, 1ull << 20, (1ull << 20) + 1, 3ull << 20})
        lens.push_back(n);
    std::shuffle(lens.begin(), lens.end(), g);
    uint64_t total = 0;
    for (uint64_t n : lens) total += n;
    const auto buf = content(99, total + 1);
    std::vector<const uint8_t*> msgs;
    uint64_t off = 0;
    for (uint64_t n : lens) {
        msgs.push_back(buf.data() + off);
        off += n;
    }
    std::vector<uint8_t> got(32 * lens.size());
    cpu_blake3_batch(msgs.data(), lens.data(), lens.size(), reinterpret_cast<uint8_t(*)[32]>(got.data()));
    int bad = 0;
    for (size_t i = 0; i < lens.size(); i++) {
        uint8_t one[32];
        cpu_blake3(msgs[i], lens[i], one);
        bad += memcmp(one, got.data() + 32 * i, 32) != 0;
    }
    CHECK(bad == 0);
}

// ------------------------------------------------------------------ planners
void test_planners() {
    std::mt19937_64 g(11);
    std::vector<sd_extent> ext;
    uint64_t off = 0;
    for (int i = 0; i < 3000; i++) {
        const uint64_t size = g() % 3 == 0 ? 102401 + g() % 1000000 : g() % 102401;
        sd_extent e = plan_extent(size, off);
        if (e.kind == SD_KIND_WHOLE && g() % 10 == 0) e.msg_len = 8 + (uint32_t)(g() % 102401);  // file != size
        validate_extent(e, i);
        ext.push_back(e);
        off = sd_align_up(off + e.msg_len, SD_STAGE_ALIGN);
    }
    WholePlan p;
    plan_whole_items(p, ext.data(), ext.size());
    // every chunk pair of every whole message is one item: full pairs (32 blocks) and
    // tail items (the rest); CV slots are unique; merge items cover each multi-pair message
    uint64_t want_pairs = 0;
    for (auto& e : ext)
        if (e.kind == SD_KIND_WHOLE) want_pairs += (msg_chunks(e.msg_len) + 1) / 2;
    CHECK(p.full.size() + p.tail.size() == want_pairs);
    std::vector<uint8_t> used(p.n_cv, 0);
    for (auto& it : p.full) {
        CHECK(it.z < p.n_cv);
        if (it.z < p.n_cv) used[it.z]++;
    }
    for (auto& it : p.tail)
        if (!(it.w >> 31)) {
            CHECK(it.z < p.n_cv);
            if (it.z < p.n_cv) used[it.z]++;
        }
    for (uint8_t u : used) CHECK(u == 1);
    uint32_t prev_cost = 99;
    for (auto& it : p.tail) {  // cost-sorted, descending
        const uint32_t glen = it.w & 0xFFF, l0 = std::min(glen, 1024u), l1 = glen - l0;
        const uint32_t cost = (l0 + 63) / 64 + (l1 ? (l1 + 63) / 64 + 1 : 0);
        CHECK(cost <= prev_cost);
        prev_cost = cost;
    }
    uint64_t roots = 0;
    for (auto& it : p.merge_a) roots += it.y >> 31;
    for (auto& it : p.merge_b) roots += it.y >> 31;
    uint64_t multi = 0;
    for (auto& e : ext)
        if (e.kind == SD_KIND_WHOLE && msg_chunks(e.msg_len) >= 3) multi++;
    CHECK(roots == multi);
    // checksum plan: one leaf per 1 MiB block; reduce passes end in one root per message
    std::vector<uint64_t> offs, lens;
    uint64_t o = 0;
    for (uint64_t L : {0ull, 1ull, 1ull << 20, (1ull << 20) + 1, 300ull << 20, 5ull << 30, 77ull}) {
        offs.push_back(o);
        lens.push_back(L);
        o = sd_align_up(o + L + 64, 64);
    }
    CkPlan c;
    plan_checksum(c, offs.data(), lens.data(), offs.size());
    uint64_t blocks = 0;
    for (uint64_t L : lens) blocks += L == 0 ? 1 : (L + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
    CHECK(c.wg_map.size() == blocks);
    uint64_t root_wgs = 0;
    for (auto& pass : c.passes)
        for (auto& w : pass) root_wgs += w.is_root;
    uint64_t multi_block = 0;
    for (uint64_t L : lens) multi_block += L > SD_CK_BLOCK;
    CHECK(root_wgs == multi_block);
}

// ------------------------------------------------------------------ stager
std::vector<uint8_t> ref_message(const std::vector<uint8_t>& file, uint64_t size, int32_t* st) {
    // cas.rs:23-62 restated inline: fs::read to EOF, or read_exact windows + End(-8192)
    std::vector<uint8_t> m(8);
    for (int i = 0; i < 8; i++) m[i] = (uint8_t)(size >> (8 * i));
    *st = SD_FILE_OK;
    if (size <= SD_MINIMUM_FILE_SIZE) {
        m.insert(m.end(), file.begin(), file.end());
        return m;
    }
    const uint64_t jump = (size - 16384) / 4;
    uint64_t pos = 8192;
    auto take = [&](uint64_t at, uint64_t n) {
        if (at + n > file.size()) {
            *st = SD_FILE_SHORT_READ;
            return false;
        }
        m.insert(m.end(), file.begin() + at, file.begin() + at + n);
        return true;
    };
    if (!take(0, 8192)) return m;
    for (;;) {
        if (!take(pos, 10240)) return m;
        if (pos >= 8192 + 3 * jump) break;
        pos += jump;
    }
    take(file.size() - 8192, 8192);
    return m;
}

void test_stager() {
    const std::pair<size_t, uint64_t> cases[] = {
        {5000, 9000}, {9000, 5000}, {150000, 1000}, {777, 0}, {0, 0}, {102400, 102400}, {700000, 300000},
        {700000, 900000}, {700000, 1600000}, {5000, 200000}, {102401, 102401}, {3 << 20, 3 << 20}};
    int k = 0;
    for (auto& c : cases) {
        const auto data = content(100 + k, c.first);
        const std::string p = write_file("st" + std::to_string(k++), data);
        int32_t want_st;
        const auto want = ref_message(data, c.second, &want_st);
        sd_extent e = plan_extent(c.second, 0);
        std::vector<uint8_t> staged(sd_align_up(std::max<uint64_t>(e.msg_len, 64), 64) + 64, 0xAB);
        const int32_t st = stage_one(p.c_str(), e, staged.data());
        if (c.second <= SD_MINIMUM_FILE_SIZE && c.first > c.second) {
            CHECK(st == SD_FILE_CHANGED);
            continue;
        }
        CHECK(st == want_st);
        if (st != SD_FILE_OK) continue;
        CHECK(e.msg_len == want.size());
        CHECK(memcmp(staged.data(), want.data(), want.size()) == 0);
        for (size_t i = want.size(); i < sd_align_up(want.size(), 64); i++) CHECK(staged[i] == 0);
        char hex17[17];
        CHECK(cpu_cas_id_file(p.c_str(), c.second, hex17) == SD_FILE_OK);
        uint8_t h[32];
        cpu_blake3(want.data(), want.size(), h);
        CHECK(hex(h, 8) == hex17);
    }
    int32_t st;
    sd_extent e = plan_extent(10, 0);
    std::vector<uint8_t> buf(128);
    st = stage_one((g_dir + "/missing").c_str(), e, buf.data());
    CHECK((st & 0xFFFF) == SD_FILE_IO_ERROR && (st >> 16) == ENOENT);
    // a FIFO (whole kind, metadata length 0): fs::read takes what the writer gives until it
    // closes; with a capture vector stage_one keeps every byte (a pipe cannot be re-read)
    for (size_t n : {size_t(0), size_t(1), size_t(4000), size_t(200000)}) {
        const std::string fifo = g_dir + "/fifo" + std::to_string(n);
        CHECK(mkfifo(fifo.c_str(), 0600) == 0);
        const auto data = content(900 + (int)n, n);
        std::thread writer([&] {
            const int fd = open(fifo.c_str(), O_WRONLY);
            for (size_t o = 0; o < n;) {  // 4000-byte writes, like test_oracle's FIFO
                const ssize_t w = write(fd, data.data() + o, std::min<size_t>(4000, n - o));
                if (w <= 0) break;
                o += (size_t)w;
            }
            close(fd);
        });
        sd_extent fe = plan_extent(0, 0);
        std::vector<uint8_t> fbuf(128, 0xAB), cap;
        const int32_t fst = stage_one(fifo.c_str(), fe, fbuf.data(), &cap);
        writer.join();
        if (n == 0) {
            CHECK(fst == SD_FILE_OK && fe.msg_len == 8 && cap.empty());
        } else {
            CHECK(fst == SD_FILE_CHANGED && cap == data);
            MsgSource src(-1, MsgSource::READ_TO_EOF);  // the message the caller hashes
            src.set_prefix_le64(0);
            src.set_memory(cap.data(), cap.size());
            std::vector<uint8_t> msg, win(3000);
            for (;;) {
                const uint64_t k = src.read(win.data(), win.size());
                msg.insert(msg.end(), win.begin(), win.begin() + k);
                if (src.done || src.err) break;
            }
            CHECK(msg.size() == n + 8 && std::equal(data.begin(), data.end(), msg.begin() + 8));
        }
        unlink(fifo.c_str());
    }
}

// ------------------------------------------------------------------ readers
void test_readers() {
    StagePool pool(4);
    for (size_t n : {0ul, 1ul, (1ul << 20) - 1, 1ul << 20, (1ul << 20) + 1, (5ul << 20) + 3}) {
        const auto data = content(n + 1, n);
        const std::string p = write_file("rd" + std::to_string(n), data);
        // par: parallel preads; hint: the EOF probe at the stat length (exact, or stale by
        // one byte short, as for a file that grew after its stat)
        for (int par = 0; par < 3; par++)  // 2: pread_stream on at most 3 of the pool's threads
            for (int hint = 0; hint < 3; hint++) {
                const int fd = open(p.c_str(), O_RDONLY);
                MsgSource src(fd, MsgSource::CHECKSUM_READS);
                if (par == 1) src.set_parallel(&pool);
                if (par == 2) src.set_parallel(&pool, 3, true);
                if (hint) src.set_eof_hint(hint == 1 ? n : (n ? n - 1 : 0));
                std::vector<uint8_t> got, win(2 << 20);  // (malloc'd: 16-byte aligned, as windows are)
                int reads = 0;
                for (;;) {
                    const uint64_t k = src.read(win.data(), win.size());
                    reads++;
                    got.insert(got.end(), win.begin(), win.begin() + k);
                    if (src.done || src.err) break;
                    CHECK(k == win.size());
                }
                close(fd);
                CHECK(src.err == 0 && got == data);
                // an exact hint ends a window-multiple file with its last full window
                if (hint == 1) CHECK(reads == (int)(n / win.size()) + (n % win.size() || n == 0 ? 1 : 0));
            }
        // READ_TO_EOF with the le64 prefix (a cas message's size header) and the EOF probe
        const int fd = open(p.c_str(), O_RDONLY);
        MsgSource src(fd, MsgSource::READ_TO_EOF);
        src.set_prefix_le64(0x1122334455667788ull);
        src.set_eof_hint(n);
        std::vector<uint8_t> got, win(333333);
        for (;;) {
            const uint64_t k = src.read(win.data(), win.size());
            got.insert(got.end(), win.begin(), win.begin() + k);
            if (src.done || src.err) break;
        }
        close(fd);
        CHECK(got.size() == n + 8 && got[0] == 0x88 && got[7] == 0x11);
        CHECK(std::equal(data.begin(), data.end(), got.begin() + 8));
    }
}

// pread_stream == pread_full: any length, any file offset, short files, an unaligned target
void test_pread_stream() {
    const size_t n = (3ul << 20) + 12345;
    const auto data = content(4242, n);
    const std::string p = write_file("pstream", data);
    const int fd = open(p.c_str(), O_RDONLY);
    CHECK(fd >= 0);
    std::vector<uint8_t> a(n + 256), b(n + 256);
    for (uint64_t off : {0ul, 1ul, 4096ul, (1ul << 20) + 7, n - 100, n, n + 5})
        for (uint64_t len : {0ul, 15ul, 16ul, 1000ul, 262144ul, 262145ul, (2ul << 20) + 33, n})
            for (size_t dst : {0ul, 16ul, 3ul}) {
                memset(a.data(), 0xAA, a.size());
                memset(b.data(), 0xAA, b.size());
                const uint64_t room = std::min<uint64_t>(len, a.size() - 64);
                const int64_t ra = pread_full(fd, a.data() + dst, room, off);
                const int64_t rb = pread_stream(fd, b.data() + dst, room, off);
                CHECK(ra == rb && a == b);
            }
    close(fd);
    CHECK(pread_stream(-1, a.data(), 10, 0) < 0);  // errors pass through
}

// a run limited to k threads runs its tasks on at most k distinct threads, on a larger pool
void test_pool_limit() {
    StagePool pool(8);
    for (int k : {1, 2, 3, 8}) {
        std::mutex mu;
        std::vector<std::thread::id> ids;
        std::atomic<int> sum{0};
        pool.run(
            400,
            [&](size_t i) {
                {
                    std::lock_guard<std::mutex> g(mu);
                    if (std::find(ids.begin(), ids.end(), std::this_thread::get_id()) == ids.end())
                        ids.push_back(std::this_thread::get_id());
                }
                volatile int spin = 0;
                for (int s = 0; s < 2000; s++) spin = spin + s;
                sum += (int)i;
            },
            k);
        CHECK(sum.load() == 399 * 400 / 2 && (int)ids.size() <= k);
        std::atomic<int> sum2{0};
        ids.clear();
        pool.start(
            100,
            [&](size_t i) {
                std::lock_guard<std::mutex> g(mu);
                if (std::find(ids.begin(), ids.end(), std::this_thread::get_id()) == ids.end())
                    ids.push_back(std::this_thread::get_id());
                sum2 += (int)i;
            },
            k);
        pool.wait();
        CHECK(sum2.load() == 99 * 100 / 2 && (int)ids.size() <= k);
    }
    // a pool grown by an earlier, larger call (the context's stage_pool only grows): the
    // next call's limit still holds -- cas_files' readers and stat_files pass theirs
    std::shared_ptr<StagePool> ctx_pool = std::make_shared<StagePool>(2);
    ctx_pool->run(64, [](size_t) {});
    ctx_pool = std::make_shared<StagePool>(16);  // a call asked for 16 readers
    for (int k : {2, 3}) {
        std::mutex mu;
        std::vector<std::thread::id> ids;
        auto note = [&](size_t) {
            std::lock_guard<std::mutex> g(mu);
            if (std::find(ids.begin(), ids.end(), std::this_thread::get_id()) == ids.end())
                ids.push_back(std::this_thread::get_id());
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        };
        ctx_pool->run(200, note, k);
        CHECK((int)ids.size() <= k);
        ids.clear();
        ctx_pool->start(200, note, k);
        ctx_pool->wait();
        CHECK((int)ids.size() <= k);
    }
}

// ------------------------------------------------------------------ pools and CPU batches
void test_pool_growth() {
    // the context's pattern: a mutex-held shared_ptr replaced by a larger pool while other
    // threads are still running on the old one
    std::mutex mu;
    std::shared_ptr<StagePool> pool;
    auto get = [&](int nt) {
        std::lock_guard<std::mutex> g(mu);
        if (!pool || pool->threads() < nt) pool = std::make_shared<StagePool>(nt);
        return pool;
    };
    std::atomic<uint64_t> total{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 6; t++)
        th.emplace_back([&, t] {
            for (int r = 0; r < 60; r++) {
                auto p = get(1 + (t * 60 + r) % 12);
                std::atomic<uint64_t> s{0};
                if (r % 2) {
                    p->run(97, [&](size_t i) { s += i; });
                } else {  // background run (sd_cas_ids_files' readers) while this thread works
                    p->start(97, [&](size_t i) { s += i; });
                    volatile uint64_t busy = 0;
                    for (int k = 0; k < 1000; k++) busy = busy + k;
                    p->wait();
                }
                total += s.load();
            }
        });
    for (auto& t : th) t.join();
    CHECK(total.load() == 6ull * 60 * (96 * 97 / 2));
}

void test_cpu_batches() {
    std::vector<std::string> names;
    std::vector<uint64_t> sizes;
    std::mt19937_64 g(5);
    for (int i = 0; i < 120; i++) {
        const size_t n = i % 4 == 0 ? 200000 + g() % 3000000 : g() % 102401;
        names.push_back(write_file("cb" + std::to_string(i), content(500 + i, n)));
        sizes.push_back(i % 17 == 0 ? n + 10 : n);  // a few stale sizes
    }
    names.push_back(g_dir + "/nope");
    sizes.push_back(10);
    std::vector<const char*> paths;
    for (auto& s : names) paths.push_back(s.c_str());
    const size_t n = paths.size();
    std::vector<char> a(17 * n), b(17 * n), ca(65 * n), cb(65 * n);
    std::vector<int32_t> sa(n), sb(n), ta(n), tb(n);
    CHECK(sd_cpu_cas_ids_files(paths.data(), sizes.data(), n, a.data(), sa.data(), 1) == SD_OK);
    CHECK(sd_cpu_cas_ids_files(paths.data(), sizes.data(), n, b.data(), sb.data(), 8) == SD_OK);
    CHECK(sd_cpu_file_checksums(paths.data(), n, ca.data(), ta.data(), 1) == SD_OK);
    CHECK(sd_cpu_file_checksums(paths.data(), n, cb.data(), tb.data(), 8) == SD_OK);
    CHECK(sa == sb && ta == tb);
    for (size_t i = 0; i < n; i++) {
        if (sa[i] == SD_FILE_OK) CHECK(memcmp(&a[17 * i], &b[17 * i], 17) == 0);
        if (ta[i] == SD_FILE_OK) CHECK(memcmp(&ca[65 * i], &cb[65 * i], 65) == 0);
    }
    CHECK((sa[n - 1] & 0xFFFF) == SD_FILE_IO_ERROR && (ta[n - 1] & 0xFFFF) == SD_FILE_IO_ERROR);
}

// many large files in one call under a low descriptor limit: sd_cpu_file_checksums holds no
// descriptor per large file across the call, so every file still hashes
void test_cpu_checksums_fd_limit() {
    constexpr int NF = 40;
    constexpr uint64_t LEN = (8ull << 20) + 4097;  // block-parallel (>= 8 MiB), sparse: zeros
    std::vector<std::string> names;
    for (int i = 0; i < NF; i++) {
        const std::string p = g_dir + "/fdlim" + std::to_string(i);
        const int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0600);
        CHECK(fd >= 0 && ftruncate(fd, (off_t)LEN) == 0);
        if (fd >= 0) close(fd);
        names.push_back(p);
    }
    std::vector<uint8_t> zeros(LEN, 0);
    uint8_t want[32];
    cpu_blake3(zeros.data(), LEN, want);
    int open_now = 0;  // descriptors this process holds
    if (DIR* d = opendir("/proc/self/fd")) {
        while (readdir(d)) open_now++;
        closedir(d);
    }
    struct rlimit old;
    CHECK(getrlimit(RLIMIT_NOFILE, &old) == 0);
    struct rlimit low = old;
    low.rlim_cur = (rlim_t)open_now + 12;  // far fewer than NF
    CHECK(setrlimit(RLIMIT_NOFILE, &low) == 0);
    std::vector<const char*> paths;
    for (auto& s : names) paths.push_back(s.c_str());
    std::vector<char> out(65 * NF);
    std::vector<int32_t> st(NF, -1);
    CHECK(sd_cpu_file_checksums(paths.data(), NF, out.data(), st.data(), 4) == SD_OK);
    CHECK(setrlimit(RLIMIT_NOFILE, &old) == 0);
    for (int i = 0; i < NF; i++) {
        CHECK(st[i] == SD_FILE_OK);
        CHECK(std::string(&out[65 * i]) == hex(want, 32));
    }
}

// ------------------------------------------------------------------ host thread budget
void test_cpu_budget() {
    // the rule: min(affinity share, quota rounded up / ranks), at least 1; the affinity is
    // split over the ranks only when it holds every online CPU
    CpuBudget b = cpu_budget_resolve(256, 256, 16.0, 8);  // an 8-GPU node, one 16-CPU quota
    CHECK(b.budget == 2 && b.affinity == 256 && b.online == 256 && b.quota_milli == 16000 && b.local_world == 8);
    CHECK(cpu_budget_resolve(256, 256, 16.0, 1).budget == 16);  // one rank: the whole quota
    CHECK(cpu_budget_resolve(256, 256, 128.0, 8).budget == 16);
    CHECK(cpu_budget_resolve(8, 8, 0.0, 1).budget == 8);      // no quota: the affinity mask
    CHECK(cpu_budget_resolve(8, 8, 0.0, 1).quota_milli == 0);
    CHECK(cpu_budget_resolve(4, 4, 16.0, 8).budget == 1);     // never below one thread
    CHECK(cpu_budget_resolve(64, 64, 1.5, 1).budget == 2);    // a fractional quota rounds up
    CHECK(cpu_budget_resolve(3, 3, 64.0, 0).budget == 3);     // a bogus world size counts as 1
    // ranks bound to their own CPUs (numactl, --cpu-bind): the mask is this rank's share
    CHECK(cpu_budget_resolve(16, 256, 0.0, 8).budget == 16);
    CHECK(cpu_budget_resolve(16, 256, 64.0, 8).budget == 8);   // the shared quota still splits
    CHECK(cpu_budget_resolve(256, 256, 0.0, 8).budget == 32);  // unbound, no quota: the node's CPUs split
    CHECK(cpu_budget_resolve(16, 8, 0.0, 1).online == 16);     // online never below the mask
    // a container pinned to a 16-CPU cpuset with no quota (docker --cpuset-cpus, k8s without
    // limits) on a 256-CPU host: the scope passed is the cpuset, so 8 ranks split it
    CHECK(cpu_budget_resolve(16, 16, 0.0, 8).budget == 2);
    CHECK(cpu_budget_resolve(2, 16, 0.0, 8).budget == 2);      // ranks bound inside the cpuset
    CHECK(cpulist_count("0-15\n") == 16 && cpulist_count("0-3,8,10-11") == 7 && cpulist_count("5") == 1);
    CHECK(cpulist_count("") == 0 && cpulist_count("3-1") == 0 && cpulist_count("a") == 0);
    // the cgroup readers, on fake cgroup trees
    const std::string v2 = g_dir + "/cg2", v1 = g_dir + "/cg1", v1c = v1 + "/cpu", none = g_dir + "/cg0";
    CHECK(mkdir(v2.c_str(), 0700) == 0 && mkdir(v1.c_str(), 0700) == 0 && mkdir(v1c.c_str(), 0700) == 0 &&
          mkdir(none.c_str(), 0700) == 0);
    auto put = [](const std::string& p, const char* s) {
        FILE* f = fopen(p.c_str(), "w");
        if (!f) abort();
        fputs(s, f);
        fclose(f);
    };
    put(v2 + "/cpu.max", "1600000 100000\n");
    CHECK(cgroup_cpu_quota(v2.c_str()) == 16.0);
    put(v2 + "/cpu.max", "max 100000\n");
    CHECK(cgroup_cpu_quota(v2.c_str()) == 0.0);
    put(v1c + "/cpu.cfs_quota_us", "250000\n");
    put(v1c + "/cpu.cfs_period_us", "100000\n");
    CHECK(cgroup_cpu_quota(v1.c_str()) == 2.5);
    put(v1c + "/cpu.cfs_quota_us", "-1\n");
    CHECK(cgroup_cpu_quota(v1.c_str()) == 0.0);
    CHECK(cgroup_cpu_quota(none.c_str()) == 0.0);
    // the process's own cgroup, nested below the mount root (cgroupns=host, systemd slices):
    // the tightest limit on the path up binds; a private namespace ("0::/") reads the root
    const std::string pc = g_dir + "/proc_cgroup", a = v2 + "/a", ab = a + "/b", abc = ab + "/c";
    for (const std::string& d : {a, ab, abc}) CHECK(mkdir(d.c_str(), 0700) == 0);
    put(v2 + "/cpu.max", "max 100000\n");
    put(a + "/cpu.max", "800000 100000\n");   // 8 CPUs two levels up
    put(ab + "/cpu.max", "max 100000\n");
    put(abc + "/cpu.max", "2400000 100000\n");  // 24 CPUs in the process's own
    put(pc, "0::/a/b/c\n");
    CHECK(cgroup_cpu_quota_self(v2.c_str(), pc.c_str()) == 8.0);
    put(abc + "/cpu.max", "400000 100000\n");  // 4 in its own: tighter
    CHECK(cgroup_cpu_quota_self(v2.c_str(), pc.c_str()) == 4.0);
    put(pc, "0::/\n");
    CHECK(cgroup_cpu_quota_self(v2.c_str(), pc.c_str()) == 0.0);
    put(v2 + "/cpu.max", "1600000 100000\n");
    CHECK(cgroup_cpu_quota_self(v2.c_str(), pc.c_str()) == 16.0);
    put(pc, "0::/a/b\n");
    CHECK(cgroup_cpu_quota_self(v2.c_str(), pc.c_str()) == 8.0);
    // v1: the cpu controller's hierarchy under <root>/cpu
    const std::string v1d = v1c + "/slice";
    CHECK(mkdir(v1d.c_str(), 0700) == 0);
    put(v1d + "/cpu.cfs_quota_us", "300000\n");
    put(v1d + "/cpu.cfs_period_us", "100000\n");
    put(pc, "12:cpuacct,cpu:/slice\n3:memory:/other\n");
    CHECK(cgroup_cpu_quota_self(v1.c_str(), pc.c_str()) == 3.0);
    put(pc, "12:memory:/slice\n");  // no cpu controller line: the root only (unlimited)
    CHECK(cgroup_cpu_quota_self(v1.c_str(), pc.c_str()) == 0.0);
    CHECK(cgroup_cpu_quota_self(none.c_str(), (g_dir + "/no_such_file").c_str()) == 0.0);
    // cpusets: v2 the process's own cgroup, else the mount root; v1 the cpuset hierarchy
    put(v2 + "/cpuset.cpus.effective", "0-255\n");
    put(abc + "/cpuset.cpus.effective", "16-31\n");
    put(pc, "0::/a/b/c\n");
    CHECK(cgroup_cpuset_count(v2.c_str(), pc.c_str()) == 16);
    put(pc, "0::/\n");
    CHECK(cgroup_cpuset_count(v2.c_str(), pc.c_str()) == 256);
    const std::string v1s = v1 + "/cpuset", v1sd = v1s + "/pod";
    CHECK(mkdir(v1s.c_str(), 0700) == 0 && mkdir(v1sd.c_str(), 0700) == 0);
    put(v1sd + "/cpuset.cpus", "0-7,64-71\n");
    put(pc, "7:cpuset:/pod\n12:cpuacct,cpu:/slice\n");
    CHECK(cgroup_cpuset_count(v1.c_str(), pc.c_str()) == 16);
    CHECK(cgroup_cpuset_count(none.c_str(), (g_dir + "/no_such_file").c_str()) == 0);
    unlink((v1sd + "/cpuset.cpus").c_str());
    rmdir(v1sd.c_str());
    rmdir(v1s.c_str());
    unlink((v2 + "/cpuset.cpus.effective").c_str());
    unlink((abc + "/cpuset.cpus.effective").c_str());
    for (const std::string& d : {abc, ab, a}) {
        unlink((d + "/cpu.max").c_str());
        rmdir(d.c_str());
    }
    unlink((v1d + "/cpu.cfs_quota_us").c_str());
    unlink((v1d + "/cpu.cfs_period_us").c_str());
    rmdir(v1d.c_str());
    unlink(pc.c_str());
    for (const std::string& f : {v2 + "/cpu.max", v1c + "/cpu.cfs_quota_us", v1c + "/cpu.cfs_period_us"})
        unlink(f.c_str());
    rmdir(v1c.c_str());
    for (const std::string& d : {v2, v1, none}) rmdir(d.c_str());
    // the override caps every call; the results do not depend on it
    const int resolved = host_cpu_budget();
    CHECK(resolved >= 1);
    CHECK(sd_cas_set_tuning("host_cpu_budget", 3) == SD_OK);
    CHECK(host_cpu_budget() == 3 && cap_host_threads(16) == 3 && cap_host_threads(2) == 2 && cap_host_threads(0) == 1);
    int out[5];
    CHECK(sd_host_cpu_budget(out) == SD_OK && out[0] == 3 && out[4] == 1);
    std::vector<uint8_t> data = content(77, 3 << 20);
    const uint64_t offs[3] = {0, 1 << 20, 2 << 20}, lens[3] = {1 << 20, 12345, (1 << 20) - 1};
    uint8_t h3[96], h1[96];
    CHECK(sd_cpu_checksums(data.data(), offs, lens, 3, h3, 16) == SD_OK);
    CHECK(sd_cas_set_tuning("host_cpu_budget", 0) == SD_OK);
    CHECK(host_cpu_budget() == resolved);
    CHECK(sd_host_cpu_budget(out) == SD_OK && out[0] == resolved && out[4] == 0);
    CHECK(sd_cpu_checksums(data.data(), offs, lens, 3, h1, 1) == SD_OK);
    CHECK(memcmp(h3, h1, 96) == 0);
}

// NUMA placement: a preferred CPU list moves the pools' worker threads onto it (within the
// affinity mask) at their next run, "numa_pin" 0 moves them back, and the caller's own
// thread is never moved
void test_numa_placement() {
    cpu_set_t all;
    CPU_ZERO(&all);
    CHECK(sched_getaffinity(0, sizeof all, &all) == 0);
    if (CPU_COUNT(&all) < 2) return;  // nothing to prefer on one CPU
    int first = -1;
    for (int c = 0; c < CPU_SETSIZE && first < 0; c++)
        if (CPU_ISSET(c, &all)) first = c;
    CHECK(numa_prefer_cpus("") == 0);                 // an empty list prefers nothing
    CHECK(numa_prefer_cpus("100000-100001") == 0);    // nor CPUs outside the mask
    const std::string one = std::to_string(first) + "-" + std::to_string(first) + ",100000\n";
    CHECK(numa_prefer_cpus(one.c_str()) == 1);
    CHECK(numa_placement(nullptr, nullptr) == 0);  // opt-in: nothing placed yet
    CHECK(sd_cas_set_tuning("numa_pin", 1) == SD_OK);
    int ncpu = 0, node = 0;
    CHECK(numa_placement(&ncpu, &node) == 1 && ncpu == 1);
    StagePool pool(4);
    auto workers_on = [&](int want_count) {
        std::mutex mu;
        std::vector<int> counts;
        pool.run(64, [&](size_t) {
            // each task takes a while, so the workers take some of them even where they are
            // slow to wake (under TSan the caller could run all 64 alone)
            std::this_thread::sleep_for(std::chrono::microseconds(500));
            cpu_set_t s;
            CPU_ZERO(&s);
            sched_getaffinity(0, sizeof s, &s);
            std::lock_guard<std::mutex> g(mu);
            counts.push_back(CPU_COUNT(&s));
        });
        cpu_set_t me;
        CPU_ZERO(&me);
        sched_getaffinity(0, sizeof me, &me);
        CHECK(CPU_COUNT(&me) == CPU_COUNT(&all));  // the caller runs tasks too and stays where it was
        bool any = false;
        for (int c : counts) any |= c == want_count;
        return any;
    };
    CHECK(workers_on(1));  // some task ran on a placed worker
    CHECK(sd_cas_set_tuning("numa_pin", 0) == SD_OK);
    CHECK(numa_placement(nullptr, nullptr) == 0);
    CHECK(!workers_on(1));  // every thread back on the whole mask
    // a thread's own narrower mask (a pinned runtime thread, another rank's thread) is never
    // widened or replaced: untouched while "numa_pin" is 0, narrowed only within itself at 1,
    // and given back its own mask -- not the process's -- at 0 again
    int second = -1;
    for (int c = first + 1; c < CPU_SETSIZE && second < 0; c++)
        if (CPU_ISSET(c, &all)) second = c;
    auto mask_is = [](std::initializer_list<int> cpus) {
        cpu_set_t now;
        CPU_ZERO(&now);
        sched_getaffinity(0, sizeof now, &now);
        bool ok = CPU_COUNT(&now) == (int)cpus.size();
        for (int c : cpus) ok = ok && CPU_ISSET(c, &now);
        return ok;
    };
    std::thread([&] {
        cpu_set_t mine;
        CPU_ZERO(&mine);
        CPU_SET(second, &mine);
        CHECK(sched_setaffinity(0, sizeof mine, &mine) == 0);
        CHECK(sd_cas_set_tuning("numa_pin", 0) == SD_OK);  // a new generation: the thread looks again
        library_thread_place();
        CHECK(mask_is({second}));
        CHECK(sd_cas_set_tuning("numa_pin", 1) == SD_OK);
        library_thread_place();  // the preferred {first} holds none of its CPUs: left as it was
        CHECK(mask_is({second}));
        CHECK(sd_cas_set_tuning("numa_pin", 0) == SD_OK);
        library_thread_place();
        CHECK(mask_is({second}));
    }).join();
    std::thread([&] {
        cpu_set_t mine;
        CPU_ZERO(&mine);
        CPU_SET(first, &mine);
        CPU_SET(second, &mine);
        CHECK(sched_setaffinity(0, sizeof mine, &mine) == 0);
        CHECK(sd_cas_set_tuning("numa_pin", 1) == SD_OK);
        library_thread_place();
        CHECK(mask_is({first}));  // placed, within its own mask
        CHECK(sd_cas_set_tuning("numa_pin", 0) == SD_OK);
        library_thread_place();
        CHECK(mask_is({first, second}));  // its own mask back, not the process's
    }).join();
}

// ------------------------------------------------------------------ coalescer
void test_coalescer() {
    std::vector<std::string> names;
    std::vector<uint64_t> sizes;
    std::vector<std::string> want_id, want_ck;
    for (int i = 0; i < 48; i++) {
        const size_t n = i % 3 == 0 ? 150000 + 777 * i : 100 + 913 * i;
        names.push_back(write_file("co" + std::to_string(i), content(900 + i, n)));
        sizes.push_back(n);
        char h17[17], h65[65];
        CHECK(cpu_cas_id_file(names.back().c_str(), n, h17) == SD_FILE_OK);
        CHECK(cpu_checksum_file(names.back().c_str(), h65) == SD_FILE_OK);
        want_id.push_back(h17);
        want_ck.push_back(h65);
    }
    for (int cpu_max : {0, 8, 1000}) {
        CHECK(sd_cas_set_tuning("latency_cpu_max", cpu_max) == SD_OK);
        CHECK(sd_cas_set_tuning("coalesce_window_us", 100) == SD_OK);
        sd_coalescer* c = coalescer_create(reinterpret_cast<sd_cas_ctx*>(0x1));  // never dereferenced here
        std::vector<std::thread> th;
        for (int t = 0; t < 24; t++)
            th.emplace_back([&, t] {
                for (int r = 0; r < 20; r++) {
                    const int i = (t * 7 + r) % 48;
                    char out[65];
                    int32_t st = -1;
                    std::string err;
                    const int kind = r % 2;
                    CHECK(coalescer_submit(c, kind, names[i].c_str(), sizes[i], out, &st, &err) == SD_OK);
                    CHECK(st == SD_FILE_OK);
                    CHECK((kind == 0 ? want_id[i] : want_ck[i]) == out);
                }
            });
        for (auto& t : th) t.join();
        uint64_t stats[4];
        coalescer_stats(c, stats);
        CHECK(stats[0] == 24 * 20);
        if (cpu_max == 0) CHECK(stats[3] == 0 && stats[1] > 0);
        if (cpu_max == 1000) CHECK(stats[3] == 24 * 20);
        coalescer_destroy(c);
    }
    CHECK(sd_cas_set_tuning("latency_cpu_max", 16) == SD_OK);
    CHECK(sd_cas_set_tuning("no_such_knob", 1) == SD_ERR_INVALID);
}

}  // namespace

// ------------------------------------------------------------------ private fd tables
// A pool with private fd tables (stage_pool.h) must not keep the process's descriptors
// alive: its workers drop their copies at start, so a pipe's write end closed by the main
// thread reads as EOF; and its tasks, opening their own files, read them correctly.
void test_private_fd_tables() {
    int p[2];
    CHECK(pipe(p) == 0);
    {
        StagePool pool(6, true);
        const std::string f = g_dir + "/fdtab";
        {
            FILE* w = fopen(f.c_str(), "wb");
            for (int i = 0; i < 4096; i++) fputc(i & 0xFF, w);
            fclose(w);
        }
        std::atomic<int> good{0};
        pool.run(64, [&](size_t i) {
            const int fd = open(f.c_str(), O_RDONLY | O_CLOEXEC);
            uint8_t b = 0;
            if (fd >= 0 && pread(fd, &b, 1, (off_t)i) == 1 && b == (uint8_t)i) good++;
            if (fd >= 0) close(fd);
        });
        CHECK(good.load() == 64);
        close(p[1]);  // the only write end left open anywhere
        fcntl(p[0], F_SETFL, O_NONBLOCK);
        char c;
        CHECK(read(p[0], &c, 1) == 0);  // EOF: no worker kept a copy of the write end
    }
    close(p[0]);
}

// The HIP-thread rule, enforced: a submission step guarded the way
// HIP_CHECK guards every HIP call (sd_api_impl.h) fails with SD_ERR_INTERNAL and a message
// on a private-fd-table worker, and passes on a shared-table pool's workers and the caller.
namespace {
int submit_window_probe() {
    SD_GUARD_BEGIN
    hip_thread_check("hipMemcpyAsync(window)");
    return SD_OK;
    SD_GUARD_END
}
}  // namespace

void test_hip_thread_rule() {
    CHECK(!on_private_fd_table() && submit_window_probe() == SD_OK);
    for (bool priv : {true, false}) {
        StagePool pool(4, priv);
        std::atomic<int> refused{0}, ok{0}, worker_tasks{0};
        std::mutex mu;
        std::string msg;
        const std::thread::id caller = std::this_thread::get_id();
        pool.run(64, [&](size_t) {
            std::this_thread::sleep_for(std::chrono::microseconds(200));  // every worker gets tasks
            if (std::this_thread::get_id() == caller) {  // the caller keeps its shared table
                if (submit_window_probe() == SD_OK) ok++;
                return;
            }
            worker_tasks++;
            const int rc = submit_window_probe();
            if (rc == SD_ERR_INTERNAL) {
                refused++;
                std::lock_guard<std::mutex> g(mu);
                msg = sd_cas_last_error();
            } else if (rc == SD_OK) {
                ok++;
            }
        });
        if (priv) {
            CHECK(refused.load() == worker_tasks.load() && refused.load() > 0);
            CHECK(msg.find("private-fd-table") != std::string::npos && msg.find("hipMemcpyAsync") != std::string::npos);
        } else {
            CHECK(refused.load() == 0 && ok.load() == 64);
        }
    }
    CHECK(!on_private_fd_table() && submit_window_probe() == SD_OK);
}

// ------------------------------------------------------------------ in-process communicator
// sd_comm_group's barrier and slots, as sd_cas_dedup_mgpu uses them: publish, barrier,
// read every peer's slot, barrier -- each rank must see exactly this round's values; and a
// rank that never arrives makes the others fail with SD_ERR_COMM, leaving the group usable.
void test_comm_group() {
    const int R = 5, ROUNDS = 300;
    sd_comm_group g(R);
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int r = 0; r < R; r++)
        th.emplace_back([&, r] {
            for (int k = 0; k < ROUNDS; k++) {
                g.slot_a[r] = (const void*)(uintptr_t)(k * R + r + 1);
                g.barrier();
                for (int p = 0; p < R; p++)
                    if (g.slot_a[p] != (const void*)(uintptr_t)(k * R + p + 1)) bad++;
                g.barrier();
            }
        });
    for (auto& t : th) t.join();
    CHECK(bad == 0);
    sd_comm_group h(3);
    h.timeout_s = 0.2;
    std::atomic<int> comm_errs{0};
    th.clear();
    for (int r = 0; r < 2; r++)  // rank 2 never arrives
        th.emplace_back([&] {
            try {
                h.barrier();
            } catch (const sd_failure& e) {
                if (e.rc == SD_ERR_COMM) comm_errs++;
            }
        });
    for (auto& t : th) t.join();
    CHECK(comm_errs == 2);
    CHECK(h.arrived == 0);
    th.clear();
    h.timeout_s = 30;
    for (int r = 0; r < 3; r++) th.emplace_back([&] { h.barrier(); });  // all three: it completes
    for (auto& t : th) t.join();
    CHECK(h.generation == 1);
}

// ------------------------------------------------------------------ multi-GPU plans
void test_exchange_plan() {
    // 3 ranks: rows [to0, to1, to2, base, n, capacity, valid]
    const int R = 3, W = R + SD_EXCHANGE_ROW_EXTRA;
    std::vector<uint64_t> rows = {5, 1, 0, 0, 10, 100, 6,     // rank 0: files [0, 10)
                                  2, 0, 7, 10, 10, 100, 9,    // rank 1: files [10, 20)
                                  0, 3, 4, 20, 10, 100, 7};   // rank 2: files [20, 30)
    uint64_t sent_to[R][R] = {}, recv_from[R][R] = {};
    for (int me = 0; me < R; me++) {
        const ExchangePlan p = exchange_plan(rows.data(), R, me);
        CHECK(p.fits && p.ascending && p.consistent);
        uint64_t so = 0, ro = 0;
        for (int q = 0; q < R; q++) {
            CHECK(p.send_off[q] == so && p.recv_off[q] == ro);  // destination / source order
            so += p.send_cnt[q];
            ro += p.recv_cnt[q];
            sent_to[me][q] = p.send_cnt[q];
            recv_from[me][q] = p.recv_cnt[q];
        }
        CHECK(p.send_total == so && p.recv_total == ro);
    }
    for (int a = 0; a < R; a++)
        for (int b = 0; b < R; b++) CHECK(sent_to[a][b] == recv_from[b][a]);  // every send has its receive
    CHECK(exchange_plan(rows.data(), R, 0).recv_total == 7 && exchange_plan(rows.data(), R, 2).recv_total == 11);
    // rank 2's capacity short: every rank sees it
    std::vector<uint64_t> tight = rows;
    tight[2 * W + 5] = 10;
    for (int me = 0; me < R; me++) CHECK(!exchange_plan(tight.data(), R, me).fits);
    // rank 1's counts disagree with its valid records: every rank sees it (and stops before
    // the record exchange, so no peer is left waiting in a send or receive)
    std::vector<uint64_t> bad = rows;
    bad[1 * W + 6] = 8;
    for (int me = 0; me < R; me++) CHECK(!exchange_plan(bad.data(), R, me).consistent);
    // overlapping index ranges: no ascending fast path, on any rank
    std::vector<uint64_t> overlap = rows;
    overlap[1 * W + 3] = 5;
    for (int me = 0; me < R; me++) CHECK(!exchange_plan(overlap.data(), R, me).ascending);
    // one file over R ranks: contiguous block ranges covering the file
    for (uint64_t total : {0ull, 1ull, (1ull << 20) + 1, (7ull << 20) + 5})
        for (int r = 1; r <= 5; r++) {
            uint64_t end = 0;
            for (int k = 0; k < r; k++) {
                const SplitPlan sp = split_plan(total, r, k);
                CHECK(sp.off == end);
                end = sp.off + sp.len;
            }
            CHECK(end == total);
        }
}

// sd_checksums' shared range: the range nearest the predicted meeting byte, among the
// ranges of >= 256 MiB
void test_shared_range_pick() {
    const uint64_t M = 1ull << 20, G = 1ull << 30, MIN = 256 * M;
    auto pick = [&](std::vector<uint64_t> l, int h) { return shared_range_pick(l.data(), l.size(), MIN, h, 55.0, 5.5); };
    CHECK(pick({4 * G}, 15) == 0);                                   // one range: it
    CHECK(pick({G, G, G, G}, 15) == 1);                              // meet at 40%: the second
    CHECK(pick({G, G, G, G}, 1) == 3);                               // one host thread: meet at 91%
    CHECK(pick({G, G, G, G}, 0) == 3);                               // no host threads: the end
    CHECK(pick({2 * G + 3, 64 * M, 64 * M, 64 * M, 64 * M}, 15) == 0);  // the GPU's first
    CHECK(pick({64 * M, 100 * M, 200 * M}, 15) == SIZE_MAX);          // none long enough
    CHECK(pick({}, 15) == SIZE_MAX);
    // meet at 40% of 3372 MiB = 1349 MiB: inside the third range (it starts at 1324 MiB)
    CHECK(pick({G, 300 * M, 2 * G}, 15) == 2);
    CHECK(pick({300 * M, 4 * G, 300 * M}, 15) == 1);
    // equally near (meet exactly between two large ranges): the first
    std::vector<uint64_t> two{G, G};
    CHECK(shared_range_pick(two.data(), 2, MIN, 10, 55.0, 5.5) == 0);
}

// sd_file_checksums' learned route (sd_host.h): each route once, then the faster, the other
// every k-th call; a route that slows down loses its place
void test_split_routes() {
    SplitRoutes s;
    std::vector<int> seen;
    auto call = [&](double split_gbps, double cpu_gbps, uint32_t k) {
        const int r = split_route_choose(s, k);
        split_route_record(s, r, r == 0 ? split_gbps : cpu_gbps);
        seen.push_back(r);
        return r;
    };
    CHECK(call(30, 100, 8) == 0);   // first: the split, a warm-up that is not counted
    CHECK(call(120, 100, 8) == 0);  // the split again, counted
    CHECK(call(10, 100, 8) == 1);   // then the CPU path, warm-up
    CHECK(call(120, 100, 8) == 1);  // and counted: now both are known
    int split_calls = 0, cpu_calls = 0;
    for (int i = 0; i < 30; i++) (call(120, 100, 8) == 0 ? split_calls : cpu_calls)++;
    CHECK(split_calls >= 26 && cpu_calls >= 3);  // the faster, and the other every 8th call
    // the host slows the split down (96 against 103): the CPU path takes over
    for (int i = 0; i < 6; i++) call(96, 103, 8);
    int cpu_after = 0;
    for (int i = 0; i < 16; i++) cpu_after += call(96, 103, 8);
    CHECK(cpu_after >= 13);
    // k = 0: no exploring once both are known
    SplitRoutes t;
    for (int r : {0, 0, 1, 1}) split_route_record(t, r, r ? 60 : 50);  // each: a warm-up, then counted
    for (int i = 0; i < 20; i++) CHECK(split_route_choose(t, 0) == 1);
    // seeded with the split slower than the CPU path, after the warm-ups: every call but the
    // explore ones (calls % k == k - 1) takes the CPU path, and those take the split
    SplitRoutes u;
    for (int r : {0, 0, 1, 1}) split_route_record(u, r, r ? 110 : 80);
    for (int i = 0; i < 40; i++) {
        const bool explore = u.calls % 8 == 7;
        const int r = split_route_choose(u, 8);
        CHECK(r == (explore ? 0 : 1));
        split_route_record(u, r, r ? 110 : 80);
    }
    // a change of a key the rates depend on moves the generation; an unchanged value does not
    int keep = 0;
    CHECK(sd_cas_get_tuning("checksum_hybrid_threads", &keep) == SD_OK);
    const uint64_t g0 = split_route_tuning_gen();
    CHECK(sd_cas_set_tuning("checksum_hybrid_threads", keep) == SD_OK && split_route_tuning_gen() == g0);
    CHECK(sd_cas_set_tuning("checksum_hybrid_threads", keep + 1) == SD_OK && split_route_tuning_gen() == g0 + 1);
    CHECK(sd_cas_set_tuning("coalesce_window_us", 200) == SD_OK && split_route_tuning_gen() == g0 + 1);
    CHECK(sd_cas_set_tuning("checksum_hybrid_threads", keep) == SD_OK && split_route_tuning_gen() == g0 + 2);
    // the RCCL exchange's bound on waiting for its peers: 5 minutes by default
    int tmo = 0;
    CHECK(sd_cas_get_tuning("comm_timeout_ms", &tmo) == SD_OK && tmo == 300000);
    // the co-hash cap scales with the budget
    CHECK(checksum_cohash_cap(16) == 13 && checksum_cohash_cap(8) == 6 && checksum_cohash_cap(4) == 3);
    CHECK(checksum_cohash_cap(2) == 1 && checksum_cohash_cap(1) == 0 && checksum_cohash_cap(32) == 26);
}

int main() {
    char tmpl[] = "/tmp/sd_selftest_XXXXXX";
    if (!mkdtemp(tmpl)) return 2;
    g_dir = tmpl;
    test_blake3();
    test_planners();
    test_stager();
    test_readers();
    test_pread_stream();
    test_pool_limit();
    test_pool_growth();
    test_cpu_batches();
    test_cpu_checksums_fd_limit();
    test_cpu_budget();
    test_coalescer();
    test_exchange_plan();
    test_shared_range_pick();
    test_split_routes();
    test_comm_group();
    test_private_fd_tables();
    test_hip_thread_rule();
    test_numa_placement();  // last: it moves the pools' threads
    // clean up the scratch directory
    if (DIR* d = opendir(g_dir.c_str())) {
        while (dirent* e = readdir(d))
            if (e->d_name[0] != '.') unlink((g_dir + "/" + e->d_name).c_str());
        closedir(d);
    }
    rmdir(g_dir.c_str());
    printf("host_selftest: %s (%d failed checks; %d SIMD lanes)\n", g_fail ? "FAILED" : "ok", g_fail.load(),
           cpu_lanes());
    return g_fail ? 1 : 0;
}
