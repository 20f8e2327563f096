// sd_host.h -- the GPU-free half of libsdcas: batch planners, the file stager with the
// reference's read semantics, the sequential message reader, error plumbing.
//
// Nothing here includes HIP, so this code (sd_host.cpp, cpu_blake3.cpp, stage_pool.h) is
// also built with g++ under ASan/UBSan and TSan by `make sanitize` (csrc/host_selftest.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sd_cas.h"
#include "stage_pool.h"

// ------------------------------------------------------------------ errors
struct sd_failure : std::runtime_error {
    int rc;
    sd_failure(int r, const std::string& m) : std::runtime_error(m), rc(r) {}
};
void sd_set_err(const char* fmt, ...);

// The HIP-thread rule: a thread that ran private_fd_table() has closed its
// copies of the HIP runtime's device descriptors, so a HIP call from it faults the process
// (round 5's first block split did exactly that).  Every HIP_CHECK (sd_api_impl.h) asks
// this first and throws SD_ERR_INTERNAL with `what` named instead of calling HIP there.
bool on_private_fd_table();
void hip_thread_check(const char* what);

// every extern "C" entry point: no C++ exception crosses the ABI (the reference FFI fences
// panics with catch_unwind, apps/mobile/modules/sd-core/ios/crate/src/lib.rs:41,60)
#define SD_GUARD_BEGIN try {
#define SD_GUARD_END                                   \
    }                                                  \
    catch (const sd_failure& f) {                      \
        sd_set_err("%s", f.what());                    \
        return f.rc;                                   \
    }                                                  \
    catch (const std::bad_alloc&) {                    \
        sd_set_err("host allocation failed");          \
        return SD_ERR_NOMEM;                           \
    }                                                  \
    catch (const std::exception& ex) {                 \
        sd_set_err("internal error: %s", ex.what());   \
        return SD_ERR_INTERNAL;                        \
    }                                                  \
    catch (...) {                                      \
        sd_set_err("internal error");                  \
        return SD_ERR_INTERNAL;                        \
    }

// process-wide tuning knobs (sd_cas_set_tuning, defined in sd_host.cpp); read at call time
enum sd_tune_key {
    SD_TUNE_COALESCE_US = 0,      // latency path: GPU batch collection window (us)
    SD_TUNE_COALESCE_MAX = 1,     // latency path: largest coalesced GPU batch
    SD_TUNE_FILES_WINDOW_MB = 2,  // sd_cas_ids_files: pinned staging window (MiB)
    SD_TUNE_DEDUP_VARIANT = 3,    // sd_dedup_group: 0 = radix sort, 1 = LDS buckets (radix on overflow)
    SD_TUNE_LATENCY_CPU_MAX = 4,  // latency path: hash on the CPU while fewer calls are in flight
    SD_TUNE_READ_THREADS = 5,     // sd_file_checksums: parallel preads of regular files
    SD_TUNE_SAMPLED_WAVE_MAX = 6, // batches of at most this many sampled files: one wave per file (latency)
    SD_TUNE_WHOLE_WAVE_MAX = 7,   // batches of at most this many whole-kind files: one workgroup per file
    SD_TUNE_BATCH_CPU_MAX = 8,    // sd_cas_ids_files: calls of at most this many files take the CPU path
    SD_TUNE_FILES_RING = 9,       // sd_cas_ids_files: pinned window buffers the readers may fill ahead
    SD_TUNE_CHECKSUM_CPU_MAX = 10,  // sd_file_checksums: calls of at most this many files take the CPU path
    SD_TUNE_FILES_STAGE_HOT = 11,   // sd_cas_ids_files: read into a per-thread buffer, stream-copy to the window
    SD_TUNE_CHECKSUM_HYBRID_THREADS = 12,  // sd_file_checksums: reader threads of the GPU route in a hybrid call
    SD_TUNE_HOST_COHASH_THREADS = 13,      // sd_cas_ids: host threads hashing beside the GPU (large calls)
    SD_TUNE_HOST_CPU_BUDGET = 14,          // cap on the host threads one call starts (0 = resolve it)
    SD_TUNE_CHECKSUM_STAGE_HOT = 15,       // sd_file_checksums' GPU route: pread_stream into the windows
    SD_TUNE_NUMA_PIN = 16,                 // library threads on the GPU's NUMA node (0 = float)
    SD_TUNE_CPU_READ_PIECE_KIB = 17,       // CPU path: a 1 MiB block read and hashed in pieces of this size
    SD_TUNE_CHECKSUM_SPLIT_BLOCKS = 18,    // sd_file_checksums' split: 1 = claims by blocks, 0 = by files
    SD_TUNE_CHECKSUM_SPLIT_ADAPT = 19,     // split-eligible calls: 0 = always split, k = learn the faster route
    SD_TUNE_COMM_TIMEOUT_MS = 20,          // sd_cas_dedup_mgpu over RCCL: longest wait for the peers (0 = none)
    SD_TUNE_NKEYS = 21
};
int tuning_get(int key);

// ------------------------------------------------------------------ host thread budget
// The host threads one call of this process may run at once, at least
// 1: min(the affinity share, the quota share), where
//   * the affinity share is the CPUs in the process's affinity mask -- divided by the GPU
//     ranks sharing the node (LOCAL_WORLD_SIZE, which torch.distributed.run sets; 1 when
//     absent) only when the mask holds every online CPU; a narrower mask is a per-rank
//     binding and already this rank's own;
//   * the quota share is the cgroup CPU bandwidth quota, rounded up, divided by those
//     ranks: every rank of the container draws on the one quota.  The quota is the
//     tightest limit on the path from the process's own cgroup (/proc/self/cgroup) up to
//     the mount root.
// "host_cpu_budget" > 0 replaces the resolved value (a Rust host that knows its own share
// sets it).  Every pool size, reader count and co-hash thread count is capped by it.
struct CpuBudget {
    int budget = 1;       // the cap
    int affinity = 1;     // CPUs in sched_getaffinity
    int online = 1;       // CPUs the process's container may use: online, or its cpuset when smaller
    int quota_milli = 0;  // cgroup CPU quota in milli-CPUs (0 = no limit)
    int local_world = 1;  // ranks per node sharing the host
    int overridden = 0;   // 1 when "host_cpu_budget" set the cap
};
// pure arithmetic of the rule (host_selftest checks it with fake masks, quotas and world sizes)
CpuBudget cpu_budget_resolve(int affinity, int online, double quota_cpus, int local_world);
// the CPU bandwidth limit of the cgroup directory `root` (v2 cpu.max, else v1
// cpu/cpu.cfs_quota_us / cpu.cfs_period_us), in CPUs; 0 when unlimited or unreadable
double cgroup_cpu_quota(const char* root);
// the tightest limit over the mount root and every directory from the process's own cgroup
// (read from `proc_cgroup`, default /proc/self/cgroup) up to it; `root` defaults to
// /sys/fs/cgroup.  0 when none is set
double cgroup_cpu_quota_self(const char* root, const char* proc_cgroup);
// CPUs in the process's cgroup cpuset (v2 cpuset.cpus.effective of its own cgroup, else the
// mount root's; v1 cpuset/<path>/cpuset.effective_cpus or cpuset.cpus), 0 when unreadable:
// a container pinned with --cpuset-cpus and no quota shows the host's CPUs online, and an
// affinity mask of the whole cpuset is then shared by the node's ranks, not one rank's binding
int cgroup_cpuset_count(const char* root, const char* proc_cgroup);
// CPUs in a cpuset list ("0-15,32,40-47"); 0 when malformed
int cpulist_count(const char* list);
CpuBudget host_cpu_budget_detail();  // resolved once per process, then the override applied
int host_cpu_budget();
inline int cap_host_threads(int n) {
    const int b = host_cpu_budget();
    return n < 1 ? 1 : (n > b ? b : n);
}

// ------------------------------------------------------------------ NUMA placement
// With "numa_pin" 1 (opt-in) the library's own threads (pool workers, co-hashing threads)
// run on the CPUs of the GPU's NUMA node, within each thread's own affinity mask; with 0 a
// thread is never touched, and one placed earlier gets its own mask back.  When the
// files' page cache was written on that node too, it pays (scripts/numa_probe.sh: the CPU
// path 90 vs 77 GB/s, the split checksum 106 vs 100 GB/s); with the page cache where an
// unplaced writer left it -- the usual case -- it measured neutral (0.93-1.04x,
// scripts/numa_lib_probe.py), so it is off by default.  `node_cpulist` is the node's sysfs
// cpulist ("0-63,128-191"); the first context sets the preference.  Returns the CPUs kept.
int numa_prefer_cpus(const char* node_cpulist);
// the node of a PCI device ("0000:23:00.0") from sysfs, or -1
int pci_numa_node(const char* bdf);
// the sysfs cpulist of a NUMA node ("" when absent)
std::string numa_node_cpulist(int node);
// 1 when library threads are placed on a preferred CPU set; the set's CPU count in *ncpus,
// the first context's device node in *node (-1 unknown)
int numa_placement(int* ncpus, int* node);
void numa_note_node(int node);

// latency path (coalesce.cpp): single-file calls, CPU route or coalesced GPU batches
struct sd_coalescer;
sd_coalescer* coalescer_create(sd_cas_ctx* ctx);
void coalescer_destroy(sd_coalescer* c);
int coalescer_submit(sd_coalescer* c, int kind, const char* path, uint64_t size, char* out, int32_t* status,
                     std::string* err);
void coalescer_stats(sd_coalescer* c, uint64_t out[4]);

inline uint64_t sd_align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
// sd_file_status IO_ERROR with the errno in the high 16 bits
inline int32_t io_status(int err) { return (int32_t)(SD_FILE_IO_ERROR | ((uint32_t)(err & 0xFFFF) << 16)); }

// What the kernels need of a staged message: a 16-byte aligned start (validate_extent) and
// zero padding up to the next 64-byte boundary.  The planner places messages on
// SD_STAGE_ALIGN (128, whole cache lines) but callers' own layouts only need this.
constexpr uint64_t SD_STAGE_PAD = 64;
// Whole-file cas messages up to this length (8 + 102400: every file the reference hashes
// whole when its length equals `size`) go through the work-list kernels; longer ones (a
// file that grew past the size it was planned with) through the chunk-parallel checksum
// kernels -- a message is just bytes.
constexpr uint32_t SD_WHOLE_ITEMS_MAX = 8 + SD_MINIMUM_FILE_SIZE;
// hash.rs:8 BLOCK_LEN: file_checksum reads 1 MiB per read call; also the checksum
// kernels' leaf block (1024 chunks per workgroup)
constexpr uint64_t SD_CK_BLOCK = 1ull << 20;

// ------------------------------------------------------------------ device tables
struct sd_u32x2 { uint32_t x, y; };        // layout of HIP's uint2
struct sd_u32x4 { uint32_t x, y, z, w; };  // layout of HIP's uint4

// one message of a checksum batch
struct ck_file {
    uint64_t offset;   // byte offset in the data buffer
    uint64_t len;      // message length
    uint64_t cv_base;  // first slot of this message's 1 MiB block CVs in the level-0 CV buffer
};

// one workgroup of a checksum reduce pass
struct ck_reduce_wg {
    uint64_t src_base;   // first CV (index into the source level) of this group
    uint64_t dst_index;  // CV slot in the destination level
    uint32_t count;      // CVs in this group (1..256)
    uint32_t file;       // file index (for the root output)
    uint32_t is_root;    // the group is the file's whole level: ROOT on the final parent
    uint32_t pad;
};

// ------------------------------------------------------------------ planners
// cas.rs:25-58 message layout of a file of `size` bytes at `off`: le64(size) || the whole
// file (size <= 102400, cas.rs:27 -- inclusive) or head / 4 samples / tail (57 352 B)
sd_extent plan_extent(uint64_t size, uint64_t off);
// the kind follows the size argument (cas.rs:27); a sampled message is 57 352 B; a whole
// message is le64(size) + the bytes the file held when read (any count, cas.rs:29)
void validate_extent(const sd_extent& e, size_t i);
uint32_t msg_chunks(uint32_t msg_len);
// BLAKE3 compressions of a message: block compressions of every chunk + parents
uint64_t msg_compressions(uint64_t len);

// whole-file work lists (item formats: cas_kernels.hip, k_whole_items / k_whole_merge8)
struct WholePlan {
    std::vector<sd_u32x4> full, tail, merge_a, merge_b;
    uint32_t n_cv = 0, n_cv2 = 0;  // pair-node CV slots, pass-A output slots
};
void plan_whole_items(WholePlan& p, const sd_extent* ext, size_t n);

// checksum batch plan: per-message tables, leaf workgroups, reduce passes
struct CkPlan {
    std::vector<ck_file> files;
    std::vector<sd_u32x2> wg_map;                 // leaf workgroup -> (message, 1 MiB block)
    std::vector<std::vector<ck_reduce_wg>> passes;  // reduce passes, level 0 -> 1 -> 0 ...
    uint64_t lvl_cap[2] = {0, 0};                 // CVs each level buffer must hold
    uint64_t total_bytes = 0, compressions = 0, blocks = 0;
};
void plan_checksum(CkPlan& p, const uint64_t* offsets, const uint64_t* lens, size_t n);

// One file over R ranks (sd_split_range, include/sd_cas.h): nb = max(1, ceil(total / 1 MiB))
// blocks, rank r holds blocks [b0, b1) = [r*q, min((r+1)*q, nb)), q = ceil(nb / R), i.e.
// file bytes [off, off + len).  Throws SD_ERR_INVALID on a bad rank / rank count.
struct SplitPlan {
    uint64_t total = 0, nb = 1, q = 1, b0 = 0, b1 = 0, off = 0, len = 0;
    int nranks = 1, rank = 0;
    uint64_t cv_bytes() const { return (uint64_t)nranks * q * 32; }
};
SplitPlan split_plan(uint64_t total, int nranks, int rank);

// The multi-GPU dedup exchange (sd_cas_dedup_mgpu) as seen by rank `me` from the gathered
// rows of all R ranks, row r = [count to rank 0 .. count to rank R-1, index base, file
// count, output capacity, valid records].  Every rank derives `fits`, `consistent` and
// `ascending` from the same matrix, so all ranks take the same branch.  Records go out in destination order (the partition's
// order) and come in in source-rank order.
struct ExchangePlan {
    std::vector<uint64_t> send_cnt, send_off, recv_cnt, recv_off;  // per peer, in records
    uint64_t send_total = 0, recv_total = 0;
    bool fits = true;        // every rank's capacity holds what it receives
    bool consistent = true;  // every rank's counts add up to its valid records
    bool ascending = true;   // the ranks' index ranges ascend with the rank
};
constexpr int SD_EXCHANGE_ROW_EXTRA = 4;
ExchangePlan exchange_plan(const uint64_t* rows, int R, int me);

// The in-process communicator's rendezvous (sd_comm_group_create, dedup_mgpu.cpp): its
// ranks are threads of one process.  A generation barrier plus one published pointer pair
// per rank: a rank writes its slots before a barrier and reads its peers' after it, the
// barrier's mutex ordering the two.  A rank that never arrives (its thread failed) makes
// the others throw SD_ERR_COMM after `timeout_s` rather than hang.
struct sd_comm_group {
    int nranks = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<const void*> slot_a, slot_b;
    std::vector<int> joined;
    double timeout_s = 120.0;
    explicit sd_comm_group(int n) : nranks(n), slot_a(n, nullptr), slot_b(n, nullptr), joined(n, 0) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == nranks) {
            arrived = 0;
            generation++;
            cv.notify_all();
            return;
        }
        // a system_clock deadline: libstdc++ waits on it with pthread_cond_timedwait, which
        // TSan intercepts (a steady_clock wait_for goes to pthread_cond_clockwait, which GCC
        // 11's TSan does not, and reads as a double lock); a clock step only moves a timeout
        const auto deadline = std::chrono::system_clock::now() +
                              std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                  std::chrono::duration<double>(timeout_s));
        if (!cv.wait_until(lk, deadline, [&] { return generation != gen; })) {
            arrived--;
            throw sd_failure(SD_ERR_COMM, "in-process group: a rank did not reach the barrier in time");
        }
    }
};

// ------------------------------------------------------------------ file reading
// Reads one file's cas message into staged + e.msg_offset exactly as generate_cas_id reads
// it (cas.rs:25-58) and zero-pads it to the next 64-byte boundary.  Returns an
// sd_file_status:
//   whole kind: every byte read() returns until EOF (fs::read, cas.rs:29); e.msg_len is
//     set to 8 + that count.  SD_FILE_CHANGED if the file holds more bytes than the
//     extent's planned room (e.msg_len - 8 on entry): the reference would hash them all.
//     With `capture`, a file that is not a regular file (a pipe, a character device: its
//     bytes cannot be read a second time) is read to its end instead, all its bytes
//     (the room's, then the rest) going to *capture; the status is still SD_FILE_CHANGED
//     and the caller hashes le64(size) || *capture.  A regular file that grew is left
//     for the caller to re-read (it may be large).
//   sampled kind: read_exact of the head and the samples at their traced offsets
//     (SHORT_READ past EOF), then the footer at seek(End(-8192)) -- the file's real end,
//     EINVAL when it is shorter than 8192 bytes.
int32_t stage_one(const char* path, sd_extent& e, uint8_t* staged, std::vector<uint8_t>* capture = nullptr);
// pread until n bytes or EOF; returns the count, or -errno
int64_t pread_full(int fd, uint8_t* dst, uint64_t n, uint64_t off);
// pread_full's result, delivered through this thread's cache-resident 256 KiB buffer and
// streamed (non-temporal stores) into dst: the page-cache copy lands in L2 and the
// destination -- a pinned window the GPU will DMA -- is written without being read first.
// On the MI355X box's host this costs 0.068 ns/B against 0.087 for pread straight into the
// pinned window and 0.172 for pread + BLAKE3 (scripts/ck_host_cost.cpp,
// profiles/r4/r4b_ck_host_cost.jsonl).  Same return convention as pread_full.
int64_t pread_stream(int fd, uint8_t* dst, uint64_t n, uint64_t off);

// A message read front to back from a file: optional le64 prefix (a cas message's size
// header), optional bytes already read from the file, then the file itself.
class MsgSource {
public:
    enum Mode {
        READ_TO_EOF,     // fs::read (cas.rs:29): read() until it returns 0
        CHECKSUM_READS,  // hash.rs:14-20: one read() of 1 MiB per call until one returns fewer
    };
    static constexpr uint64_t CHECKSUM_READ = SD_CK_BLOCK;
    MsgSource(int fd, Mode m) : fd_(fd), mode_(m) {}
    void set_prefix_le64(uint64_t v);
    // a message held in memory: after the prefix, exactly these bytes, then the end
    void set_memory(const uint8_t* p, uint64_t n) {
        pend_ = p;
        pend_len_ = n;
        mem_only_ = true;
    }
    // the file's first n bytes, already taken from it (whole 1 MiB reads in CHECKSUM_READS mode)
    void set_pending(const uint8_t* p, uint64_t n) {
        pend_ = p;
        pend_len_ = n;
        file_pos_ = n;
    }
    // A regular file (S_ISREG) read in CHECKSUM_READS mode: hash.rs's 1 MiB reads until a
    // short one return exactly the bytes up to EOF, so each window is filled with 1 MiB
    // preads at their offsets in parallel on `pool`, and ends at the first short piece.
    // At most `threads` of the pool's threads read one window; `stream` delivers the pieces
    // through pread_stream (a pinned destination) instead of pread straight into dst.
    void set_parallel(StagePool* pool, int threads = 1 << 30, bool stream = false) {
        pool_ = pool;
        par_threads_ = threads;
        par_stream_ = stream;
    }
    // A regular file's stat length: when the reads reach exactly that many file bytes, one
    // 1-byte pread past it decides whether the message has ended (a read there returns 0,
    // as the reference's next read would), so a reader of W-byte windows learns the end
    // with the last full window instead of from an extra, empty one.  A file that grew
    // keeps going: nothing is consumed by the probe.
    void set_eof_hint(uint64_t file_len) {
        eof_hint_ = file_len;
        has_eof_hint_ = true;
    }
    // Writes up to n message bytes to dst and returns the count; fewer than n only at the
    // end of the message (done) or on an error (err = errno).  CHECKSUM_READS: n is a
    // multiple of 1 MiB.
    uint64_t read(uint8_t* dst, uint64_t n);
    bool done = false;
    int err = 0;

private:
    uint64_t read_parallel(uint8_t* dst, uint64_t n);
    uint64_t read_impl(uint8_t* dst, uint64_t n);
    int fd_;
    Mode mode_;
    StagePool* pool_ = nullptr;
    int par_threads_ = 1 << 30;
    bool par_stream_ = false;
    uint64_t file_pos_ = 0;  // bytes taken from the file so far
    uint8_t prefix_[8] = {};
    uint32_t prefix_len_ = 0, prefix_pos_ = 0;
    const uint8_t* pend_ = nullptr;
    uint64_t pend_len_ = 0;
    uint64_t eof_hint_ = 0;
    bool has_eof_hint_ = false;
    bool mem_only_ = false;
};

// ------------------------------------------------------------------ CPU BLAKE3 (cpu_blake3.cpp)
// The library's own CPU hasher: the BLAKE3 spec's incremental chunk / CV-stack structure,
// with whole chunks hashed many at a time across SIMD lanes (AVX-512 16-way, AVX2 8-way,
// portable 1-way, picked at run time).  Used by the sd_cpu_* entry points and the
// latency path's CPU route.
class CpuHasher {
public:
    CpuHasher();
    // a subtree whose first chunk has index chunk0 (a 1 MiB block of a longer message)
    explicit CpuHasher(uint64_t chunk0);
    void update(const uint8_t* p, size_t n);
    void finalize(uint8_t out[32]) const;
    // the subtree's chaining value: no ROOT flag (a block of a message of several blocks)
    void finalize_cv(uint8_t out[32]) const;

private:
    static constexpr uint32_t BLOCK_CHUNKS = 1024;  // 1 MiB: the unit merged level-wise
    void push_chunk_cv(const uint32_t cv[8]);
    void finish(uint8_t out[32], bool root) const;
    // chunk CVs of the current 1 MiB block, merged level-wise (SIMD parents) when it is
    // complete; complete blocks' CVs on a stack that merges every completed subtree
    // (the first SMALL_CHUNKS CVs inline: a cas message never needs the heap -- a 32 KiB
    // allocation per message cost the 16-thread CPU path a third of its rate)
    static constexpr uint32_t SMALL_CHUNKS = 128;
    uint32_t (*blk())[8] { return big_ ? big_.get() : small_; }
    const uint32_t (*blk() const)[8] { return big_ ? big_.get() : small_; }
    uint32_t small_[SMALL_CHUNKS][8];
    std::unique_ptr<uint32_t[][8]> big_;  // BLOCK_CHUNKS entries, once a message outgrows small_
    uint32_t nblk_ = 0;
    uint32_t stack_[48][8];
    int sp_ = 0;
    uint64_t blocks_ = 0;  // complete blocks pushed so far
    uint64_t ctr0_ = 0;    // chunk index of the first chunk
    uint64_t chunks_ = 0;  // complete chunks pushed so far
    uint8_t buf_[1024];
    uint32_t buf_len_ = 0;
};
void cpu_blake3(const uint8_t* p, size_t n, uint8_t out[32]);
// BLAKE3 of n messages, the chunks of all of them packed across the SIMD lanes together
// (cas messages of a few chunks each); out[i] = the hash of msg[i][0, len[i])
void cpu_blake3_batch(const uint8_t* const* msg, const uint64_t* len, size_t n, uint8_t (*out)[32]);
// BLAKE3 root of a message from its nb >= 2 consecutive 1 MiB block CVs (32 B each)
void cpu_root_from_cvs(const uint8_t* cvs, uint64_t nb, uint8_t out[32]);
// the (non-root) chaining values of 1 MiB blocks [b0, b1) of a message of total_len >= 2
// blocks, on nthreads threads: block b's 32 bytes at cvs + 32 * b
void cpu_block_cvs(const uint8_t* msg, uint64_t total_len, uint64_t b0, uint64_t b1, uint8_t* cvs, int nthreads);
// sd_checksums' co-hashing: the index of the range of >= min_len bytes
// nearest the byte where the GPU (gpu_gbps, from the front) and host_threads host threads
// (thread_gbps each, from the back) are predicted to meet; the first of equally near ones;
// SIZE_MAX if no range is that long
size_t shared_range_pick(const uint64_t* lens, size_t n, uint64_t min_len, int host_threads, double gpu_gbps,
                         double thread_gbps);
// lanes of the SIMD chunk hasher this CPU runs (16, 8 or 1)
int cpu_lanes();
// generate_cas_id / file_checksum of one file on the calling thread -> sd_file_status
int32_t cpu_cas_id_file(const char* path, uint64_t size, char out_hex17[17]);
int32_t cpu_checksum_file(const char* path, char out_hex65[65]);
// the (non-root) chaining value of 1 MiB block `block` of a regular file of file_len >= 2
// blocks, read from fd at its offset ("cpu_read_piece_kib" pieces); false on a short read
bool cpu_block_cv_fd(int fd, uint64_t file_len, uint64_t block, uint8_t cv[32]);

// sd_file_checksums' route for a call the split applies to, learned per context (round 5:
// the split lost 7 % to the CPU path alone on a host whose CPU path read and hashed 103 GB/s
// from files, and won 34 % on one at 78).  rate[r] is the EWMA of GB/s of
// route r's past calls (0 = the split, 1 = the CPU path alone), n[r] how many were counted
// -- a route's first call in the context is not (it pays for its pinned windows and pools:
// a split's first call ran at 82 GB/s against 100+ after) -- and each route runs until one
// call is counted, then the faster one, and every explore_every-th call the other (0 = never).
struct SplitRoutes {
    double rate[2] = {0.0, 0.0};
    uint32_t n[2] = {0, 0};
    uint32_t seen[2] = {0, 0};  // calls recorded per route, the uncounted first included
    uint64_t calls = 0;         // counted calls
};
int split_route_choose(const SplitRoutes& s, uint32_t explore_every);
void split_route_record(SplitRoutes& s, int route, double gbps);
// bumped by sd_cas_set_tuning when a key either route's rate depends on changes value
// (read_threads, checksum_hybrid_threads, host_cpu_budget, checksum_split_blocks,
// cpu_read_piece_kib, checksum_stage_hot, numa_pin, host_cohash_threads): a context's
// learned rates from before are dropped at its next eligible call
uint64_t split_route_tuning_gen();
// co-hashing threads of a sd_checksums call under a host budget of b: b less 3/16 of it, at
// least one less (16 -> 13, 8 -> 6, 4 -> 3, 2 -> 1, 1 -> 0)
inline int checksum_cohash_cap(int b) { return b <= 1 ? 0 : b - std::max(1, (3 * b + 8) / 16); }
void hex_lower(const uint8_t* h, int nbytes, char* out);
