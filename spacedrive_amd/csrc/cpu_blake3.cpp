// cpu_blake3.cpp -- the library's CPU path: BLAKE3 on the host and the sd_cpu_* entry points.
//
// SURVEY.md §8(b) asks for a CPU variant of each export -- for a node without a gfx950
// device, and for the latency path's single-file callers (the location watcher,
// core/src/location/manager/watcher/utils.rs:235,393,438-446, and non_indexed::walk,
// core/src/location/non_indexed.rs:164-187), where one GPU round trip per file costs more
// than hashing the file on the calling thread.  It reads files with the same semantics as
// the GPU path (sd_host.cpp: stage_one, MsgSource) and hashes with:
//   * whole 1 KiB chunks many at a time, one chunk per SIMD lane (cpu_b3_lanes.inc:
//     AVX-512 16 lanes, AVX2 8, SSE2 4 -- chosen at run time);
//   * the BLAKE3 spec's incremental structure: the last chunk of the input stays buffered
//     until more input arrives, complete chunks push their CV on a stack that merges
//     every completed subtree, finalize merges the stack into the root (ROOT on the
//     final compression).
#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "sd_host.h"
#include "stage_pool.h"

void cpu_hash_chunks_x16(const uint8_t* const* in, int n, uint64_t ctr0, uint32_t (*cv)[8]);
void cpu_hash_chunks_x8(const uint8_t* const* in, int n, uint64_t ctr0, uint32_t (*cv)[8]);
void cpu_hash_chunks_x4(const uint8_t* const* in, int n, uint64_t ctr0, uint32_t (*cv)[8]);
void cpu_hash_parents_x16(const uint32_t (*cvs)[8], int n, uint32_t (*out)[8]);
void cpu_hash_parents_x8(const uint32_t (*cvs)[8], int n, uint32_t (*out)[8]);
void cpu_hash_parents_x4(const uint32_t (*cvs)[8], int n, uint32_t (*out)[8]);
void cpu_hash_chunks_var_x16(const uint8_t* const* in, const uint32_t* len, const uint64_t* ctr, const uint8_t* root,
                             int n, uint32_t (*cv)[8]);
void cpu_hash_chunks_var_x8(const uint8_t* const* in, const uint32_t* len, const uint64_t* ctr, const uint8_t* root,
                            int n, uint32_t (*cv)[8]);
void cpu_hash_chunks_var_x4(const uint8_t* const* in, const uint32_t* len, const uint64_t* ctr, const uint8_t* root,
                            int n, uint32_t (*cv)[8]);

namespace {

constexpr uint32_t CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8;
constexpr uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                            0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
constexpr uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// one compression: cv <- first 8 words of compress(cv, m, counter, len, flags)
void compress1(uint32_t cv[8], const uint32_t m_in[16], uint64_t counter, uint32_t len, uint32_t flags) {
    uint32_t m[16], s[16];
    memcpy(m, m_in, 64);
    for (int i = 0; i < 8; i++) s[i] = cv[i];
    for (int i = 0; i < 4; i++) s[8 + i] = IV[i];
    s[12] = (uint32_t)counter;
    s[13] = (uint32_t)(counter >> 32);
    s[14] = len;
    s[15] = flags;
    auto g = [&](int a, int b, int c, int d, uint32_t x, uint32_t y) {
        s[a] = s[a] + s[b] + x; s[d] = rotr(s[d] ^ s[a], 16);
        s[c] = s[c] + s[d];     s[b] = rotr(s[b] ^ s[c], 12);
        s[a] = s[a] + s[b] + y; s[d] = rotr(s[d] ^ s[a], 8);
        s[c] = s[c] + s[d];     s[b] = rotr(s[b] ^ s[c], 7);
    };
    for (int r = 0; r < 7; r++) {
        g(0, 4, 8, 12, m[0], m[1]);
        g(1, 5, 9, 13, m[2], m[3]);
        g(2, 6, 10, 14, m[4], m[5]);
        g(3, 7, 11, 15, m[6], m[7]);
        g(0, 5, 10, 15, m[8], m[9]);
        g(1, 6, 11, 12, m[10], m[11]);
        g(2, 7, 8, 13, m[12], m[13]);
        g(3, 4, 9, 14, m[14], m[15]);
        uint32_t t[16];
        for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
        memcpy(m, t, 64);
    }
    for (int i = 0; i < 8; i++) cv[i] = s[i] ^ s[i + 8];
}

void parent_cv(const uint32_t l[8], const uint32_t r[8], uint32_t extra, uint32_t out[8]) {
    uint32_t m[16];
    memcpy(m, l, 32);
    memcpy(m + 8, r, 32);
    memcpy(out, IV, 32);
    compress1(out, m, 0, 64, PARENT | extra);
}

// CV of one chunk of len (0..1024) bytes, chunk index counter; ROOT on its last block
void chunk_cv(const uint8_t* p, uint32_t len, uint64_t counter, bool root, uint32_t cv[8]) {
    memcpy(cv, IV, 32);
    const uint32_t nb = len == 0 ? 1 : (len + 63) / 64;
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t bl = b + 1 < nb ? 64 : len - 64 * b;
        uint8_t blk[64] = {0};
        memcpy(blk, p + 64 * b, bl);
        uint32_t m[16];
        memcpy(m, blk, 64);  // little-endian host
        const uint32_t fl = (b == 0 ? CHUNK_START : 0) | (b + 1 == nb ? CHUNK_END : 0) | (root && b + 1 == nb ? ROOT : 0);
        compress1(cv, m, counter, bl, fl);
    }
}

using chunks_fn = void (*)(const uint8_t* const*, int, uint64_t, uint32_t (*)[8]);
using parents_fn = void (*)(const uint32_t (*)[8], int, uint32_t (*)[8]);
using var_fn = void (*)(const uint8_t* const*, const uint32_t*, const uint64_t*, const uint8_t*, int, uint32_t (*)[8]);
struct Simd {
    chunks_fn fn;
    int lanes;
    parents_fn parents;
    var_fn var;  // chunks of any length, one per lane (cpu_blake3_batch)
};
Simd pick_simd() {
    __builtin_cpu_init();
    // SD_CPU_LANES=4/8 caps the width (tests run every width the CPU has)
    const char* cap = getenv("SD_CPU_LANES");
    const int lim = cap ? atoi(cap) : 16;
    if (lim >= 16 && __builtin_cpu_supports("avx512f"))
        return {cpu_hash_chunks_x16, 16, cpu_hash_parents_x16, cpu_hash_chunks_var_x16};
    if (lim >= 8 && __builtin_cpu_supports("avx2"))
        return {cpu_hash_chunks_x8, 8, cpu_hash_parents_x8, cpu_hash_chunks_var_x8};
    return {cpu_hash_chunks_x4, 4, cpu_hash_parents_x4, cpu_hash_chunks_var_x4};
}
const Simd& simd() {
    static const Simd s = pick_simd();
    return s;
}

// n >= 2 CVs merged level-wise (pairs left to right, the odd node carried up: BLAKE3's tree
// over power-of-two aligned groups), the pairs of a level SIMD_LANES at a time; ROOT on the
// final parent when `root`.  cv[] is overwritten.
void merge_levels(uint32_t (*cv)[8], uint64_t n, bool root, uint32_t out[8]) {
    const Simd& s = simd();
    uint32_t tmp[16][8];
    while (n > 2) {
        const uint64_t P = n / 2;
        for (uint64_t i = 0; i < P; i += (uint64_t)s.lanes) {
            const int g = (int)std::min<uint64_t>((uint64_t)s.lanes, P - i);
            s.parents(cv + 2 * i, g, tmp);  // reads pairs [2i, 2i + 2g) before any write
            memcpy(cv + i, tmp, 32 * (size_t)g);
        }
        if (n & 1) memmove(cv + P, cv + n - 1, 32);
        n = P + (n & 1);
    }
    parent_cv(cv[0], cv[1], root ? ROOT : 0, out);
}

}  // namespace

int cpu_lanes() { return simd().lanes; }

CpuHasher::CpuHasher() {}
CpuHasher::CpuHasher(uint64_t chunk0) : ctr0_(chunk0) {}

void CpuHasher::push_chunk_cv(const uint32_t cv[8]) {
    if (nblk_ == SMALL_CHUNKS && !big_) {
        big_.reset(new uint32_t[BLOCK_CHUNKS][8]);
        memcpy(big_.get(), small_, sizeof small_);
    }
    memcpy(blk()[nblk_++], cv, 32);
    chunks_++;
    if (nblk_ < BLOCK_CHUNKS) return;
    // a complete 1 MiB block (never the message's last: its last chunk stays buffered)
    uint32_t cur[8];
    merge_levels(blk(), nblk_, false, cur);
    nblk_ = 0;
    uint64_t total = ++blocks_;
    while ((total & 1) == 0) {  // this block completes a subtree: merge it with its left half
        parent_cv(stack_[--sp_], cur, 0, cur);
        total >>= 1;
    }
    memcpy(stack_[sp_++], cur, 32);
}

void CpuHasher::update(const uint8_t* p, size_t n) {
    const Simd& s = simd();
    while (n) {
        if (buf_len_ == 1024) {  // the buffered chunk is not the last one: push it
            uint32_t cv[8];
            chunk_cv(buf_, 1024, ctr0_ + chunks_, false, cv);
            push_chunk_cv(cv);
            buf_len_ = 0;
        }
        if (buf_len_ == 0 && n > 1024) {  // whole chunks straight from the input, keeping >= 1 byte back
            size_t k = (n - 1) / 1024;
            const uint8_t* ptrs[16];
            uint32_t cvs[16][8];
            while (k) {
                const int g = (int)std::min<size_t>(k, (size_t)s.lanes);
                for (int i = 0; i < g; i++) ptrs[i] = p + 1024 * (size_t)i;
                s.fn(ptrs, g, ctr0_ + chunks_, cvs);
                for (int i = 0; i < g; i++) push_chunk_cv(cvs[i]);
                p += 1024 * (size_t)g;
                n -= 1024 * (size_t)g;
                k -= (size_t)g;
            }
            continue;
        }
        const size_t take = std::min<size_t>(1024 - buf_len_, n);
        memcpy(buf_ + buf_len_, p, take);
        buf_len_ += (uint32_t)take;
        p += take;
        n -= take;
    }
}

void CpuHasher::finish(uint8_t out[32], bool root) const {
    uint32_t cur[8];
    if (chunks_ == 0) {  // one chunk: it is the message (ROOT on its last block)
        chunk_cv(buf_, buf_len_, ctr0_, root, cur);
        memcpy(out, cur, 32);  // little-endian words = the hash bytes
        return;
    }
    // the last block: its chunk CVs and the buffered last chunk, merged level-wise
    const uint32_t (*cv)[8] = blk();
    uint32_t last[8];
    chunk_cv(buf_, buf_len_, ctr0_ + chunks_, false, last);
    const bool whole = sp_ == 0;  // the message is this one block
    if (nblk_ == 0) {
        memcpy(cur, last, 32);
    } else {
        // finish() is const: merge a copy (on the stack for the short messages of cas_ids)
        uint32_t small[128][8];
        std::vector<uint32_t> big;
        uint32_t(*t)[8] = small;
        if (nblk_ + 1 > 128) {
            big.resize((size_t)(nblk_ + 1) * 8);
            t = reinterpret_cast<uint32_t(*)[8]>(big.data());
        }
        memcpy(t, cv, 32 * (size_t)nblk_);
        memcpy(t[nblk_], last, 32);
        merge_levels(t, nblk_ + 1, root && whole, cur);
    }
    if (!whole) {  // then the complete blocks' subtrees, right to left
        for (int i = sp_ - 1; i >= 1; i--) parent_cv(stack_[i], cur, 0, cur);
        parent_cv(stack_[0], cur, root ? ROOT : 0, cur);
    }
    memcpy(out, cur, 32);
}

void CpuHasher::finalize(uint8_t out[32]) const { finish(out, true); }
void CpuHasher::finalize_cv(uint8_t out[32]) const { finish(out, false); }

// BLAKE3 root from nb >= 2 consecutive 1 MiB block CVs (the split checksum)
void cpu_root_from_cvs(const uint8_t* cvs, uint64_t nb, uint8_t out[32]) {
    std::vector<uint32_t> lvl(nb * 8);
    memcpy(lvl.data(), cvs, nb * 32);
    uint32_t o[8];
    merge_levels(reinterpret_cast<uint32_t(*)[8]>(lvl.data()), nb, true, o);
    memcpy(out, o, 32);
}

void cpu_blake3(const uint8_t* p, size_t n, uint8_t out[32]) {
    CpuHasher h;
    h.update(p, n);
    h.finalize(out);
}

// BLAKE3 of n messages at once.  A message of a few chunks fills few SIMD lanes on its own
// (most cas messages: 60% of a library's small files are one partial chunk, a sampled
// message is 56 chunks and an 8-byte one), so the chunks of all n messages are packed
// across the lanes: every chunk is a job (its bytes, its counter in its message, ROOT if it
// is its message's only chunk), jobs are grouped by block count, full chunks first, and
// each message's chunk CVs are then merged into its root.  A message over 1 MiB goes
// through CpuHasher on its own.
void cpu_blake3_batch(const uint8_t* const* msg, const uint64_t* len, size_t n, uint8_t (*out)[32]) {
    constexpr uint64_t BATCH_MAX = 1ull << 20;
    const Simd& s = simd();
    std::vector<uint64_t> first(n + 1);  // message i's chunk CVs: slots [first[i], first[i + 1])
    uint64_t total = 0;
    size_t per_nb[17] = {0};  // jobs by block count (1..16)
    for (size_t i = 0; i < n; i++) {
        first[i] = total;
        if (len[i] > BATCH_MAX) continue;
        const uint64_t C = len[i] == 0 ? 1 : (len[i] + 1023) / 1024;
        per_nb[16] += C - 1;  // the chunks before the last are full
        const uint64_t last = len[i] - 1024 * (C - 1);
        per_nb[last == 0 ? 1 : (last + 63) / 64]++;
        total += C;
    }
    first[n] = total;
    struct Job {
        const uint8_t* p;
        uint64_t ctr, slot;
        uint32_t len;
        uint8_t root;
    };
    std::vector<Job> jobs(total);
    size_t at[17];
    for (size_t k = 16, pos = 0; k >= 1; k--) {  // longest first
        at[k] = pos;
        pos += per_nb[k];
    }
    for (size_t i = 0; i < n; i++) {
        if (len[i] > BATCH_MAX) continue;
        const uint64_t C = first[i + 1] - first[i];
        for (uint64_t c = 0; c < C; c++) {
            const uint32_t L = (uint32_t)(c + 1 < C ? 1024 : len[i] - 1024 * c);
            const size_t k = L == 0 ? 1 : (L + 63) / 64;
            jobs[at[k]++] = Job{msg[i] + 1024 * c, c, first[i] + c, L, (uint8_t)(C == 1)};
        }
    }
    std::vector<uint32_t> cvbuf(total * 8);
    auto cvs = reinterpret_cast<uint32_t(*)[8]>(cvbuf.data());
    for (size_t j = 0; j < total; j += (size_t)s.lanes) {
        const int g = (int)std::min<size_t>((size_t)s.lanes, total - j);
        const uint8_t* ptr[16];
        uint32_t lens[16];
        uint64_t ctr[16];
        uint8_t root[16];
        uint32_t tmp[16][8];
        for (int l = 0; l < g; l++) {
            const Job& b = jobs[j + (size_t)l];
            ptr[l] = b.p;
            lens[l] = b.len;
            ctr[l] = b.ctr;
            root[l] = b.root;
        }
        s.var(ptr, lens, ctr, root, g, tmp);
        for (int l = 0; l < g; l++) memcpy(cvs[jobs[j + (size_t)l].slot], tmp[l], 32);
    }
    for (size_t i = 0; i < n; i++) {
        if (len[i] > BATCH_MAX) {
            cpu_blake3(msg[i], len[i], out[i]);
            continue;
        }
        const uint64_t C = first[i + 1] - first[i];
        if (C == 1) {  // its one chunk, hashed with ROOT
            memcpy(out[i], cvs[first[i]], 32);
            continue;
        }
        uint32_t o[8];
        merge_levels(cvs + first[i], C, true, o);
        memcpy(out[i], o, 32);
    }
}

void hex_lower(const uint8_t* h, int nbytes, char* out) {
    static const char HEX[] = "0123456789abcdef";
    for (int i = 0; i < nbytes; i++) {
        out[2 * i] = HEX[h[i] >> 4];
        out[2 * i + 1] = HEX[h[i] & 15];
    }
    out[2 * nbytes] = 0;
}

namespace {
struct Fd {
    int fd;
    ~Fd() {
        if (fd >= 0) close(fd);
    }
};

// hashes a MsgSource to its end; SD_FILE_OK or io_status
int32_t hash_source(MsgSource& src, uint8_t* buf, uint64_t bufsz, uint8_t out[32]) {
    CpuHasher h;
    for (;;) {
        const uint64_t got = src.read(buf, bufsz);
        if (src.err) return io_status(src.err);
        h.update(buf, got);
        if (src.done) break;
    }
    h.finalize(out);
    return SD_FILE_OK;
}
}  // namespace

// per-thread read buffers, allocated once (a fresh, zeroed 128 KiB or 1 MiB buffer per file
// costs more than reading a small file)
static uint8_t* scratch(size_t bytes) {
    thread_local std::unique_ptr<uint8_t[]> buf;
    thread_local size_t have = 0;
    if (have < bytes) {
        buf.reset(new uint8_t[bytes]);
        have = bytes;
    }
    return buf.get();
}

int32_t cpu_cas_id_file(const char* path, uint64_t size, char out_hex17[17]) {
    uint8_t h[32];
    if (size > SD_MINIMUM_FILE_SIZE) {  // cas.rs:30-58: the 57 352 B sampled message
        uint8_t* msg = scratch(sd_align_up(SD_SAMPLED_MSG_LEN, SD_STAGE_PAD));
        sd_extent e = plan_extent(size, 0);
        const int32_t st = stage_one(path, e, msg);
        if (st != SD_FILE_OK) return st;
        cpu_blake3(msg, e.msg_len, h);
    } else {  // cas.rs:25-29: le64(size) || fs::read
        Fd f{open(path, O_RDONLY | O_CLOEXEC)};
        if (f.fd < 0) return io_status(errno);
        {
            // a seekable file in one call (as stage_one): le64(size), then up to the buffer's
            // room.  Exactly `size` bytes back (the file holds what its stat said) is the
            // file; any other count -- a longer or shorter file, a filesystem that returns
            // short counts -- or a pipe (ESPIPE, nothing consumed) takes the streaming read
            // below, which reads until a read returns 0 as fs::read does.
            constexpr uint64_t ROOM = (128 << 10) - 8;
            uint8_t* msg = scratch(128 << 10);
            for (int i = 0; i < 8; i++) msg[i] = (uint8_t)(size >> (8 * i));
            ssize_t r;
            do {
                r = pread(f.fd, msg + 8, ROOM, 0);
            } while (r < 0 && errno == EINTR);
            if (r >= 0 && (uint64_t)r == size) {
                cpu_blake3(msg, 8 + (size_t)r, h);
                hex_lower(h, 8, out_hex17);  // cas.rs:61 to_hex()[..16]
                return SD_FILE_OK;
            }
            if (r < 0 && errno != ESPIPE) return io_status(errno);
        }
        MsgSource src(f.fd, MsgSource::READ_TO_EOF);
        src.set_prefix_le64(size);
        const int32_t st = hash_source(src, scratch(128 << 10), 128 << 10, h);
        if (st != SD_FILE_OK) return st;
    }
    hex_lower(h, 8, out_hex17);  // cas.rs:61 to_hex()[..16]
    return SD_FILE_OK;
}

bool cpu_block_cv_fd(int fd, uint64_t file_len, uint64_t block, uint8_t cv[32]) {
    const uint64_t off = block * SD_CK_BLOCK;
    if (off >= file_len) return false;
    const uint64_t want = std::min<uint64_t>(SD_CK_BLOCK, file_len - off);
    // "cpu_read_piece_kib" p > 0: the block is read and hashed p KiB at a time, so each
    // piece is hashed while it is still in this core's L2 (0: one 1 MiB read, then the hash)
    const int pk = tuning_get(SD_TUNE_CPU_READ_PIECE_KIB);
    const uint64_t piece = pk > 0 ? std::min<uint64_t>(SD_CK_BLOCK, (uint64_t)pk << 10) : SD_CK_BLOCK;
    uint8_t* buf = scratch(piece);
    CpuHasher h(block * (SD_CK_BLOCK / 1024));
    for (uint64_t o = 0; o < want; o += piece) {
        const uint64_t n = std::min(piece, want - o);
        if (pread_full(fd, buf, n, off + o) != (int64_t)n) return false;
        h.update(buf, n);
    }
    h.finalize_cv(cv);
    return true;
}

int32_t cpu_checksum_file(const char* path, char out_hex65[65]) {
    Fd f{open(path, O_RDONLY | O_CLOEXEC)};  // hash.rs:11
    if (f.fd < 0) return io_status(errno);
    MsgSource src(f.fd, MsgSource::CHECKSUM_READS);
    uint8_t h[32];
    const int32_t st = hash_source(src, scratch(SD_CK_BLOCK), SD_CK_BLOCK, h);
    if (st != SD_FILE_OK) return st;
    hex_lower(h, 32, out_hex65);  // hash.rs:21-23
    return SD_FILE_OK;
}

namespace {
// fn(i) for i in [0, n) on up to nthreads threads (the caller's included)
template <class F>
void parallel_for(size_t n, int nthreads, F fn) {
    // never more threads than the process's host budget (sd_host.h), the caller's included
    nthreads = std::max(1, std::min<int>(cap_host_threads(nthreads), (int)std::min<size_t>(n, 256)));
    if (nthreads == 1) {
        for (size_t i = 0; i < n; i++) fn(i);
        return;
    }
    // worker threads persist across calls in pools keyed by thread count (creating the
    // threads per call cost a 16-file call ~0.4 ms, most of its time); a pool serves one
    // call at a time, so concurrent callers take separate pools.  The workers run on
    // private fd tables (stage_pool.h): every task opens and closes its own files
    static std::mutex mu;
    static std::vector<std::unique_ptr<StagePool>> idle[257];
    std::unique_ptr<StagePool> pool;
    {
        std::lock_guard<std::mutex> g(mu);
        if (!idle[nthreads].empty()) {
            pool = std::move(idle[nthreads].back());
            idle[nthreads].pop_back();
        }
    }
    if (!pool) pool = std::make_unique<StagePool>(nthreads, true);  // tasks open their own files
    struct Back {
        std::unique_ptr<StagePool>& p;
        int k;
        ~Back() {
            std::lock_guard<std::mutex> g(mu);
            idle[k].push_back(std::move(p));
        }
    } back{pool, nthreads};
    pool->run(n, std::function<void(size_t)>(fn));
}
}  // namespace

// ============================================================================ C ABI
extern "C" {

int sd_cpu_simd_lanes(void) { return cpu_lanes(); }

int sd_cpu_cas_ids(const uint8_t* staged, uint64_t staged_bytes, const sd_extent* extents, size_t n, char* out_hex17,
                   int32_t* status, int nthreads) {
    SD_GUARD_BEGIN
    if (n && (!staged || !extents || !out_hex17)) throw sd_failure(SD_ERR_INVALID, "null argument");
    for (size_t i = 0; i < n; i++) {
        validate_extent(extents[i], i);
        if (extents[i].msg_offset + extents[i].msg_len > staged_bytes)
            throw sd_failure(SD_ERR_INVALID, "extent beyond staged_bytes");
    }
    // groups of up to 64 messages, their chunks packed across the SIMD lanes together
    // (cpu_blake3_batch); at least ~4 groups per thread
    const size_t G = std::max<size_t>(1, std::min<size_t>(64, n / ((size_t)std::max(1, nthreads) * 4)));
    parallel_for((n + G - 1) / G, nthreads, [&](size_t t) {
        const size_t a = t * G, b = std::min(n, a + G);
        const uint8_t* m[64] = {};
        uint64_t l[64] = {};
        size_t idx[64], k = 0;
        for (size_t i = a; i < b; i++) {
            if (status && status[i] != SD_FILE_OK) continue;
            m[k] = staged + extents[i].msg_offset;
            l[k] = extents[i].msg_len;
            idx[k++] = i;
        }
        uint8_t h[64][32];
        cpu_blake3_batch(m, l, k, h);
        for (size_t q = 0; q < k; q++) hex_lower(h[q], 8, out_hex17 + 17 * idx[q]);
    });
    return SD_OK;
    SD_GUARD_END
}

int sd_cpu_cas_ids_files(const char* const* paths, const uint64_t* sizes, size_t n, char* out_hex17, int32_t* status,
                         int nthreads) {
    SD_GUARD_BEGIN
    if (n && (!paths || !sizes || !out_hex17 || !status)) throw sd_failure(SD_ERR_INVALID, "null argument");
    parallel_for(n, nthreads, [&](size_t i) { status[i] = cpu_cas_id_file(paths[i], sizes[i], out_hex17 + 17 * i); });
    return SD_OK;
    SD_GUARD_END
}

int sd_cpu_checksums(const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, size_t n, uint8_t* out_hash32,
                     int nthreads) {
    SD_GUARD_BEGIN
    if (n && (!data || !offsets || !lens || !out_hash32)) throw sd_failure(SD_ERR_INVALID, "null argument");
    // a range of 8 MiB or more is hashed block-parallel (as sd_cpu_file_checksums below): its
    // 1 MiB blocks are tasks of their own beside the small ranges' tasks, and its root is
    // merged from the block CVs -- else one huge range ran on one thread
    constexpr uint64_t SPLIT_MIN = 8ull << 20;
    struct Task {
        size_t range;
        uint64_t block;  // UINT64_MAX: the whole range
    };
    std::vector<Task> tasks;
    std::vector<size_t> big;
    std::vector<std::vector<uint8_t>> cvs;
    tasks.reserve(n);
    for (size_t i = 0; i < n; i++) {
        if (nthreads > 1 && lens[i] >= SPLIT_MIN) {
            const uint64_t nb = (lens[i] + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
            for (uint64_t b = 0; b < nb; b++) tasks.push_back({big.size(), b});
            big.push_back(i);
            cvs.emplace_back(nb * 32);
        } else {
            tasks.push_back({i, UINT64_MAX});
        }
    }
    parallel_for(tasks.size(), nthreads, [&](size_t t) {
        const Task& k = tasks[t];
        if (k.block == UINT64_MAX) {
            cpu_blake3(data + offsets[k.range], lens[k.range], out_hash32 + 32 * k.range);
            return;
        }
        const size_t i = big[k.range];
        const uint64_t pos = k.block * SD_CK_BLOCK, len = std::min<uint64_t>(SD_CK_BLOCK, lens[i] - pos);
        CpuHasher h(k.block * (SD_CK_BLOCK / 1024));
        h.update(data + offsets[i] + pos, len);
        h.finalize_cv(cvs[k.range].data() + 32 * k.block);
    });
    for (size_t q = 0; q < big.size(); q++) cpu_root_from_cvs(cvs[q].data(), cvs[q].size() / 32, out_hash32 + 32 * big[q]);
    return SD_OK;
    SD_GUARD_END
}

// file_checksum (hash.rs:10-24) for n paths on the host.  A regular file of at least
// CPU_SPLIT_MIN bytes is hashed block-parallel: its 1 MiB blocks are tasks of their own
// (a block's chaining value depends only on its bytes and its chunk counter), so a batch
// of a few large files keeps every thread busy; its root is merged from the block CVs.
// For a regular file the 1 MiB reads of hash.rs are exactly its bytes up to EOF; if the
// file turns out shorter or longer than its stat length while it is read, it is hashed
// again with the sequential read loop.  Other files: one task each, the read loop.
constexpr uint64_t CPU_SPLIT_MIN = 8ull << 20;

int sd_cpu_file_checksums(const char* const* paths, size_t n, char* out_hex65, int32_t* status, int nthreads) {
    SD_GUARD_BEGIN
    if (n && (!paths || !out_hex65 || !status)) throw sd_failure(SD_ERR_INVALID, "null argument");
    struct Big {
        size_t file;
        uint64_t len, nb;
        std::vector<uint8_t> cvs;
        std::atomic<bool> failed{false};
    };
    std::vector<uint64_t> len(n, 0);
    std::vector<uint8_t> split(n, 0);
    if (nthreads > 1)
        parallel_for(n, nthreads, [&](size_t i) {
            struct stat st;
            if (stat(paths[i], &st) == 0 && S_ISREG(st.st_mode) && (uint64_t)st.st_size >= CPU_SPLIT_MIN) {
                len[i] = (uint64_t)st.st_size;
                split[i] = 1;
            }
        });
    std::vector<std::unique_ptr<Big>> big;
    struct Task {
        size_t file;    // a whole file (block == UINT64_MAX) ...
        uint64_t block; // ... or one 1 MiB block of big[file]
    };
    std::vector<Task> tasks;
    for (size_t i = 0; i < n; i++) {
        if (!split[i]) {
            tasks.push_back({i, UINT64_MAX});
            continue;
        }
        // no descriptor is held across the call (a call of many large files would otherwise
        // hold one per file and could exhaust RLIMIT_NOFILE for the whole process): every
        // block task opens the path itself, and the end-of-file check reopens it
        auto b = std::make_unique<Big>();
        b->file = i;
        b->len = len[i];
        b->nb = (len[i] + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
        b->cvs.resize(b->nb * 32);
        for (uint64_t k = 0; k < b->nb; k++) tasks.push_back({big.size(), k});
        big.push_back(std::move(b));
    }
    parallel_for(tasks.size(), nthreads, [&](size_t t) {
        const Task& task = tasks[t];
        if (task.block == UINT64_MAX) {
            status[task.file] = cpu_checksum_file(paths[task.file], out_hex65 + 65 * task.file);
            return;
        }
        Big& b = *big[task.file];
        if (b.failed.load(std::memory_order_relaxed)) return;
        // the task's own descriptor: pool workers have private fd tables (stage_pool.h)
        const int fd = open(paths[b.file], O_RDONLY | O_CLOEXEC);
        const bool ok = fd >= 0 && cpu_block_cv_fd(fd, b.len, task.block, b.cvs.data() + 32 * task.block);
        if (fd >= 0) close(fd);
        if (!ok)  // shrank, replaced, unopenable: the read loop below reports it
            b.failed.store(true, std::memory_order_relaxed);
    });
    for (auto& bp : big) {
        Big& b = *bp;
        bool at_end = false;
        if (!b.failed.load()) {  // nothing past the stat length: the blocks were the whole file
            Fd f{open(paths[b.file], O_RDONLY | O_CLOEXEC)};
            uint8_t probe;
            at_end = f.fd >= 0 && pread_full(f.fd, &probe, 1, b.len) == 0;
        }
        if (at_end) {
            uint8_t h[32];
            cpu_root_from_cvs(b.cvs.data(), b.nb, h);
            hex_lower(h, 32, out_hex65 + 65 * b.file);  // hash.rs:21-23
            status[b.file] = SD_FILE_OK;
        } else {  // the file changed while it was read: hash.rs's sequential loop, to EOF
            status[b.file] = cpu_checksum_file(paths[b.file], out_hex65 + 65 * b.file);
        }
    }
    return SD_OK;
    SD_GUARD_END
}

int sd_cpu_cas_id_path(const char* path, uint64_t size, char* out_hex17, int32_t* status) {
    SD_GUARD_BEGIN
    if (!path || !out_hex17 || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    *status = cpu_cas_id_file(path, size, out_hex17);
    return SD_OK;
    SD_GUARD_END
}

}  // extern "C"

void cpu_block_cvs(const uint8_t* msg, uint64_t total_len, uint64_t b0, uint64_t b1, uint8_t* cvs, int nthreads) {
    parallel_for(b1 - b0, nthreads, [&](size_t k) {
        const uint64_t b = b0 + k;
        const uint64_t len = std::min<uint64_t>(SD_CK_BLOCK, total_len - b * SD_CK_BLOCK);
        CpuHasher h(b * (SD_CK_BLOCK / 1024));
        h.update(msg + b * SD_CK_BLOCK, len);
        h.finalize_cv(cvs + 32 * b);
    });
}

extern "C" {

int sd_cpu_split_leaves(const uint8_t* slice, uint64_t total_len, int nranks, int rank, uint8_t* cvs,
                        int nthreads) {
    SD_GUARD_BEGIN
    const SplitPlan p = split_plan(total_len, nranks, rank);
    if (!cvs || (p.len && !slice)) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (p.nb == 1) {  // one block: rank 0 holds the file and slot 0 its root hash
        if (rank == 0) cpu_blake3(slice, p.len, cvs);
        return SD_OK;
    }
    parallel_for(p.b1 - p.b0, nthreads, [&](size_t k) {
        const uint64_t b = p.b0 + k;
        const uint64_t off = b * SD_CK_BLOCK - p.off;
        const uint64_t len = std::min<uint64_t>(SD_CK_BLOCK, p.total - b * SD_CK_BLOCK);
        CpuHasher h(b * (SD_CK_BLOCK / 1024));
        h.update(slice + off, len);
        h.finalize_cv(cvs + 32 * b);
    });
    return SD_OK;
    SD_GUARD_END
}

int sd_cpu_split_root(const uint8_t* cvs, uint64_t total_len, uint8_t* out_hash32) {
    SD_GUARD_BEGIN
    if (!cvs || !out_hash32) throw sd_failure(SD_ERR_INVALID, "null argument");
    const SplitPlan p = split_plan(total_len, 1, 0);
    if (p.nb == 1) memcpy(out_hash32, cvs, 32);
    else cpu_root_from_cvs(cvs, p.nb, out_hash32);
    return SD_OK;
    SD_GUARD_END
}

int sd_cpu_file_checksum_path(const char* path, char* out_hex65, int32_t* status) {
    SD_GUARD_BEGIN
    if (!path || !out_hex65 || !status) throw sd_failure(SD_ERR_INVALID, "null argument");
    *status = cpu_checksum_file(path, out_hex65);
    return SD_OK;
    SD_GUARD_END
}

}  // extern "C"
