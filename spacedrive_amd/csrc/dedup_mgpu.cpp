// dedup_mgpu.cpp -- the multi-GPU post-hash step behind the C ABI.
//
// Reference semantics: identifier_job_step links every file_path to the Object that owns
// an equal cas_id, creating Objects otherwise (core/src/object/file_identifier/mod.rs:
// 136-333).  With the library sharded by file index over one process per GPU, the only
// exchange is the one that brings equal cas_ids together: each rank partitions its
// records (cas_id as big-endian u64, global index) by cas_id prefix into contiguous
// destination ranges, and an all-to-all over RCCL (xGMI on MI355X) delivers every record
// to the rank that owns its prefix range, which groups and assigns Objects locally.
//
// One call per rank, all on the caller's stream:
//   1. sd_dedup_partition: stable partition by destination, per-destination counts;
//   2. ncclAllGather of one row per rank -- its counts, index range and output capacity --
//      so every rank knows the whole count matrix: the receive sizes, a capacity check
//      that every rank evaluates identically (so an undersized rank makes all ranks
//      return before the record exchange rather than leave peers hanging), and whether
//      the shards' index ranges ascend with the rank (the received records are then in
//      index order, and the grouping skips one sort);
//   3. grouped ncclSend / ncclRecv of the 16-byte records (one pair per peer, self
//      included), the all-to-all;
//   4. sd_dedup_group + sd_dedup_owners on the received records.
// A Rust host drives this through sd_comm_id (ncclGetUniqueId on one rank, the 128 bytes
// passed to the others out of band) and sd_comm_create (ncclCommInitRank).
//
// The same calls also run over an in-process group (sd_comm_group_create +
// sd_comm_create_local): ranks are threads of one process, on one device or several, and
// steps 2 and 3 become device-to-device copies between the ranks' buffers, ordered by a
// host barrier.  It serves one process driving several GPUs, and it rehearses N ranks on
// one GPU, which RCCL refuses ("Duplicate GPU detected") -- the partition, the gathered
// plan, the per-peer offsets and the grouping are the same code either way.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sd_internal.h"

struct sd_comm {
    ncclComm_t comm = nullptr;
    sd_comm_group* group = nullptr;  // in-process transport instead of RCCL
    int nranks = 0, rank = 0, device = 0;
    // device scratch, grown on demand: the partitioned send records, the all-gather rows
    // (send row + nranks rows)
    void* d_send = nullptr;
    size_t send_bytes = 0;
    void* d_rows = nullptr;
    void* d_part_scratch = nullptr;  // sdk::dedup_partition's scratch; its last u64 = valid records
    uint64_t* h_rows = nullptr;      // pinned: this rank's row extras, then all rows
    // sd_comm_set_timing: events around the phases of the last sd_cas_dedup_mgpu call
    bool timing = false;
    bool timed = false;  // the last call recorded all of ev[]
    hipEvent_t ev[SD_DEDUP_PHASES + 1] = {};
    // A wait for the peers outlasted "comm_timeout_ms" (wait_peers): work may still be queued
    // or spinning on the stream against these buffers and this RCCL communicator, so every
    // later call fails and destruction releases nothing (the host is expected to exit; its
    // process teardown frees the device state).
    bool broken = false;
    std::string broken_why;
    ~sd_comm() {
        if (broken) {
            if (group) {
                std::lock_guard<std::mutex> lk(group->mu);
                group->joined[rank] = 0;
            }
            return;
        }
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (d_part_scratch) (void)hipFree(d_part_scratch);
        if (d_send) (void)hipFree(d_send);
        if (d_rows) (void)hipFree(d_rows);
        if (h_rows) (void)hipHostFree(h_rows);
        if (comm) (void)ncclCommDestroy(comm);
        if (group) {
            std::lock_guard<std::mutex> lk(group->mu);
            group->joined[rank] = 0;
        }
    }
};

namespace {

#define HIP_OK(expr)                                                                                    \
    do {                                                                                                \
        hip_thread_check(#expr); /* the HIP-thread rule (sd_host.h) */                                  \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            throw sd_failure(e_ == hipErrorOutOfMemory ? SD_ERR_NOMEM : SD_ERR_DEVICE,                 \
                             std::string(#expr) + ": " + hipGetErrorString(e_));                       \
    } while (0)

#define NCCL_OK(expr)                                                                                   \
    do {                                                                                                \
        hip_thread_check(#expr);                                                                        \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess) throw sd_failure(SD_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

void check_rc(int rc) {
    if (rc != SD_OK) throw sd_failure(rc, sd_cas_last_error());
}

// row layout of the all-gather: counts[nranks], index base, local file count, capacity,
// valid records (the partition's own total, so the consistency check is collective)
constexpr int ROW_EXTRA = SD_EXCHANGE_ROW_EXTRA;
static_assert(ROW_EXTRA == 4, "row = counts, base, n, capacity, valid");

// phase boundary k of the current call, when timing is on
void mark(sd_comm* c, int k, hipStream_t s) {
    if (!c->timing) return;
    if (!c->ev[k]) HIP_OK(hipEventCreate(&c->ev[k]));
    HIP_OK(hipEventRecord(c->ev[k], s));
}

// Waits for the work queued on `s` -- this call's collectives among it -- for at most
// "comm_timeout_ms" (0 = no bound).  An RCCL kernel waits for its peers without limit, so a
// peer rank that died or hung would otherwise keep this rank's host thread, and its GPU,
// waiting forever.  On RCCL's asynchronous error or the deadline this rank reports
// SD_ERR_COMM naming the step, and the communicator is marked broken (see sd_comm).  It is
// not aborted: ncclCommAbort frees resources that kernels still queued behind the wait
// would use.  The in-process transport has its own bounded barrier.
void wait_peers(sd_comm* c, hipStream_t s, const char* step) {
    const int ms = tuning_get(SD_TUNE_COMM_TIMEOUT_MS);
    if (c->group || ms <= 0) {
        HIP_OK(hipStreamSynchronize(s));
        return;
    }
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int spin = 0;; spin++) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) HIP_OK(e);
        ncclResult_t r = ncclSuccess;
        NCCL_OK(ncclCommGetAsyncError(c->comm, &r));
        const bool late = clk::now() - t0 > std::chrono::milliseconds(ms);
        if ((r != ncclSuccess && r != ncclInProgress) || late) {
            c->broken = true;
            c->broken_why = std::string(step) + ": " +
                            (late ? "the peers did not complete within comm_timeout_ms = " + std::to_string(ms)
                                  : std::string("RCCL reported ") + ncclGetErrorString(r));
            throw sd_failure(SD_ERR_COMM, "sd_cas_dedup_mgpu: " + c->broken_why +
                                              " (the communicator is unusable from now on)");
        }
        // a short exchange finishes within microseconds: poll first, then sleep between polls
        if (spin < 256) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

void check_usable(const sd_comm* c) {
    if (c->broken) throw sd_failure(SD_ERR_COMM, "communicator broken by an earlier call (" + c->broken_why + ")");
}

// In-process all-gather of `bytes` per rank: rank p's block at `src` lands at dst + p * bytes
// (host or device memory) for every p.  In place when src == dst + rank * bytes.
void local_allgather(sd_comm* c, const void* src, void* dst, size_t bytes, hipStream_t s) {
    sd_comm_group* g = c->group;
    HIP_OK(hipStreamSynchronize(s));  // this rank's block is complete
    g->slot_a[c->rank] = src;
    g->barrier();
    for (int p = 0; p < c->nranks; p++) {
        uint8_t* to = (uint8_t*)dst + (size_t)p * bytes;
        if (bytes && to != g->slot_a[p]) HIP_OK(hipMemcpyAsync(to, g->slot_a[p], bytes, hipMemcpyDefault, s));
    }
    HIP_OK(hipStreamSynchronize(s));
    g->barrier();  // every rank holds every block: the sources may change again
}

}  // namespace

extern "C" {

int sd_comm_group_create(int nranks, sd_comm_group** out) {
    SD_GUARD_BEGIN
    if (!out) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (nranks < 1 || nranks > 64) throw sd_failure(SD_ERR_INVALID, "nranks out of range (1..64)");
    *out = new sd_comm_group(nranks);
    return SD_OK;
    SD_GUARD_END
}

void sd_comm_group_destroy(sd_comm_group* group) { delete group; }

int sd_comm_create_local(sd_cas_ctx* ctx, sd_comm_group* group, int rank, sd_comm** out) {
    SD_GUARD_BEGIN
    if (!ctx || !group || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (rank < 0 || rank >= group->nranks) throw sd_failure(SD_ERR_INVALID, "rank out of range");
    *out = nullptr;
    {
        std::lock_guard<std::mutex> lk(group->mu);
        if (group->joined[rank]) throw sd_failure(SD_ERR_INVALID, "rank already joined this group");
        group->joined[rank] = 1;
    }
    auto c = std::make_unique<sd_comm>();
    c->group = group;
    c->nranks = group->nranks;
    c->rank = rank;
    c->device = sd_ctx_device(ctx);
    HIP_OK(hipSetDevice(c->device));
    const size_t row = (size_t)c->nranks + ROW_EXTRA;
    HIP_OK(hipMalloc(&c->d_rows, sizeof(uint64_t) * row * (c->nranks + 1)));
    HIP_OK(hipMalloc(&c->d_part_scratch, sdk::dedup_partition_scratch(c->nranks)));
    HIP_OK(hipHostMalloc((void**)&c->h_rows, sizeof(uint64_t) * (row * (c->nranks + 1) + 1), hipHostMallocDefault));
    *out = c.release();
    return SD_OK;
    SD_GUARD_END
}

int sd_comm_id(uint8_t* out_id) {
    SD_GUARD_BEGIN
    if (!out_id) throw sd_failure(SD_ERR_INVALID, "null argument");
    static_assert(sizeof(ncclUniqueId) == SD_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    NCCL_OK(ncclGetUniqueId(&id));
    memcpy(out_id, &id, SD_COMM_ID_BYTES);
    return SD_OK;
    SD_GUARD_END
}

int sd_comm_create(sd_cas_ctx* ctx, const uint8_t* id, int nranks, int rank, sd_comm** out) {
    SD_GUARD_BEGIN
    if (!ctx || !id || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks)
        throw sd_failure(SD_ERR_INVALID, "rank / nranks out of range (1..64 ranks)");
    *out = nullptr;
    auto c = std::make_unique<sd_comm>();
    c->nranks = nranks;
    c->rank = rank;
    c->device = sd_ctx_device(ctx);
    HIP_OK(hipSetDevice(c->device));
    ncclUniqueId uid;
    memcpy(&uid, id, SD_COMM_ID_BYTES);
    NCCL_OK(ncclCommInitRank(&c->comm, nranks, uid, rank));
    const size_t row = (size_t)nranks + ROW_EXTRA;
    HIP_OK(hipMalloc(&c->d_rows, sizeof(uint64_t) * row * (nranks + 1)));
    HIP_OK(hipMalloc(&c->d_part_scratch, sdk::dedup_partition_scratch(nranks)));
    HIP_OK(hipHostMalloc((void**)&c->h_rows, sizeof(uint64_t) * (row * (nranks + 1) + 1), hipHostMallocDefault));
    *out = c.release();
    return SD_OK;
    SD_GUARD_END
}

void sd_comm_destroy(sd_comm* comm) {
    try {
        if (comm) (void)hipSetDevice(comm->device);
        delete comm;
    } catch (...) {
    }
}

int sd_cas_dedup_mgpu(sd_cas_ctx* ctx, sd_comm* comm, const uint8_t* d_hash32, const uint8_t* d_valid, uint64_t n,
                      uint64_t global_index_base, uint64_t chunk_size, uint64_t* d_records_out, uint64_t* d_rep_out,
                      uint64_t* d_owner_out, uint64_t capacity, uint64_t* m_out, uint64_t* n_groups_out,
                      void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !comm || !m_out || !n_groups_out || (n && !d_hash32) ||
        (capacity && (!d_records_out || !d_rep_out || !d_owner_out)))
        throw sd_failure(SD_ERR_INVALID, "null argument");
    if (chunk_size == 0) throw sd_failure(SD_ERR_INVALID, "chunk_size must be positive");
    check_usable(comm);
    HIP_OK(hipSetDevice(comm->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int R = comm->nranks, me = comm->rank;
    const size_t row = (size_t)R + ROW_EXTRA;
    // 1. partition this rank's records by destination rank
    if (comm->send_bytes < 16 * n || !comm->d_send) {
        if (comm->d_send) HIP_OK(hipFree(comm->d_send));
        comm->d_send = nullptr;
        comm->send_bytes = 16 * (n ? n : 1);
        HIP_OK(hipMalloc(&comm->d_send, comm->send_bytes));
    }
    // (the partition counts go straight into this rank's all-gather row; no host sync here)
    uint64_t* d_row = (uint64_t*)comm->d_rows;
    uint64_t* d_all = d_row + row;
    const size_t psb = sdk::dedup_partition_scratch(R);
    uint64_t* pscratch = (uint64_t*)comm->d_part_scratch;
    comm->timed = false;
    mark(comm, 0, s);
    HIP_OK(sdk::dedup_partition(d_hash32, d_valid, n, global_index_base, R, d_row, (uint64_t*)comm->d_send, pscratch,
                                s));
    mark(comm, 1, s);
    // 2. all-gather of (counts, index base, file count, capacity, valid records)
    uint64_t* h_row = comm->h_rows;
    h_row[R] = global_index_base;
    h_row[R + 1] = n;
    h_row[R + 2] = capacity;
    HIP_OK(hipMemcpyAsync(d_row + R, h_row + R, sizeof(uint64_t) * 3, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(d_row + R + 3, pscratch + psb / sizeof(uint64_t) - 1, sizeof(uint64_t),
                          hipMemcpyDeviceToDevice, s));
    uint64_t* all = comm->h_rows + row;
    if (comm->group) {  // in-process: every rank's row straight into this rank's host table
        comm->group->slot_b[me] = comm->d_send;  // read by the peers after the barriers below
        local_allgather(comm, d_row, all, sizeof(uint64_t) * row, s);
        mark(comm, 2, s);
    } else {
        NCCL_OK(ncclAllGather(d_row, d_all, row, ncclUint64, comm->comm, s));
        HIP_OK(hipMemcpyAsync(all, d_all, sizeof(uint64_t) * row * R, hipMemcpyDeviceToHost, s));
        mark(comm, 2, s);
    }
    wait_peers(comm, s, "all-gather of the count rows");  // the sync before the exchange: every rank's row
    const ExchangePlan plan = exchange_plan(all, R, me);
    *m_out = plan.recv_total;
    *n_groups_out = 0;
    // every rank sees the same matrix, so every rank stops here together, before any record
    // moves (a rank that stopped alone would leave its peers waiting in the send/receive)
    if (!plan.fits)
        throw sd_failure(SD_ERR_CAPACITY, "an output capacity is smaller than the records its rank receives "
                                         "(*m_out = this rank's requirement)");
    if (!plan.consistent) throw sd_failure(SD_ERR_INTERNAL, "a rank's partition counts disagree with its valid records");
    // 3. the all-to-all of the 16-byte records: one send and one receive per peer
    mark(comm, 3, s);
    const uint64_t* send = (const uint64_t*)comm->d_send;
    if (comm->group) {
        // in-process: pull what each peer sends here from its partitioned records, which
        // start at the sum of its counts to the ranks before this one
        sd_comm_group* g = comm->group;
        for (int p = 0; p < R; p++) {
            if (!plan.recv_cnt[p]) continue;
            uint64_t off = 0;
            for (int q = 0; q < me; q++) off += all[(size_t)p * row + q];
            HIP_OK(hipMemcpyAsync(d_records_out + 2 * plan.recv_off[p], (const uint64_t*)g->slot_b[p] + 2 * off,
                                  16 * plan.recv_cnt[p], hipMemcpyDefault, s));
        }
        HIP_OK(hipStreamSynchronize(s));
        g->barrier();  // every rank has its records: the send buffers may be reused
    } else {
        NCCL_OK(ncclGroupStart());
        for (int p = 0; p < R; p++) {
            if (plan.send_cnt[p])
                NCCL_OK(ncclSend(send + 2 * plan.send_off[p], 2 * plan.send_cnt[p], ncclUint64, p, comm->comm, s));
            if (plan.recv_cnt[p])
                NCCL_OK(ncclRecv(d_records_out + 2 * plan.recv_off[p], 2 * plan.recv_cnt[p], ncclUint64, p,
                                 comm->comm, s));
        }
        NCCL_OK(ncclGroupEnd());
    }
    mark(comm, 4, s);
    // bounded, before the grouping's own (unbounded) sync for the group count
    if (!comm->group) wait_peers(comm, s, "send/receive of the records");
    // 4. group by cas_id and assign Objects (chunk-of-100 rule) on the received records
    uint64_t ng = 0;
    dedup_group_owners(ctx, d_records_out, *m_out, plan.ascending ? SD_DEDUP_INDEX_SORTED : 0, d_rep_out, chunk_size,
                       d_owner_out, &ng, s);
    mark(comm, 5, s);
    comm->timed = comm->timing;
    *n_groups_out = ng;
    return SD_OK;
    SD_GUARD_END
}

int sd_comm_rccl_info(int* version, char* path_out, size_t path_cap) {
    SD_GUARD_BEGIN
    if (!version) throw sd_failure(SD_ERR_INVALID, "null argument");
    NCCL_OK(ncclGetVersion(version));
    if (path_out && path_cap) {
        // the file the dynamic linker bound this library's RCCL symbols to: librccl.so.1 is
        // one soname, so a process that loaded another copy first (torch's) serves it here
        Dl_info di{};
        const char* f = dladdr(reinterpret_cast<void*>(&ncclGetVersion), &di) && di.dli_fname ? di.dli_fname : "";
        snprintf(path_out, path_cap, "%s", f);
    }
    return SD_OK;
    SD_GUARD_END
}

int sd_comm_set_timing(sd_comm* comm, int on) {
    SD_GUARD_BEGIN
    if (!comm) throw sd_failure(SD_ERR_INVALID, "null argument");
    comm->timing = on != 0;
    comm->timed = false;
    return SD_OK;
    SD_GUARD_END
}

int sd_comm_last_phases(sd_comm* comm, float* ms_out) {
    SD_GUARD_BEGIN
    if (!comm || !ms_out) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (!comm->timed) throw sd_failure(SD_ERR_INVALID, "no timed sd_cas_dedup_mgpu call (sd_comm_set_timing)");
    HIP_OK(hipSetDevice(comm->device));
    HIP_OK(hipEventSynchronize(comm->ev[SD_DEDUP_PHASES]));
    for (int k = 0; k < SD_DEDUP_PHASES; k++) HIP_OK(hipEventElapsedTime(&ms_out[k], comm->ev[k], comm->ev[k + 1]));
    return SD_OK;
    SD_GUARD_END
}

// One file over the ranks (include/sd_cas.h): each rank's block CVs, then an in-place
// all-gather of the CV slots -- rank r's q slots sit at r * q, so the gathered buffer is the
// file's block CVs in order (the padding past nb is never read) --, then the reduce.
int sd_split_checksum_mgpu(sd_cas_ctx* ctx, sd_comm* comm, sd_split_checksum* split, const uint8_t* d_slice,
                           uint8_t* d_cvs, uint8_t* d_hash32, void* stream) {
    SD_GUARD_BEGIN
    if (!ctx || !comm || !split || !d_cvs || !d_hash32) throw sd_failure(SD_ERR_INVALID, "null argument");
    const SplitPlan& p = sd_split_plan_of(split);
    if (p.nranks != comm->nranks || p.rank != comm->rank)
        throw sd_failure(SD_ERR_INVALID, "the split's nranks / rank differ from the communicator's");
    check_usable(comm);
    HIP_OK(hipSetDevice(comm->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    check_rc(sd_split_checksum_leaves(ctx, split, d_slice, d_cvs, stream));
    // over RCCL the all-gather runs at any rank count (one rank: an in-place copy of its own
    // slots), so a one-GPU run drives the same collective an 8-GPU node does
    if (comm->nranks > 1 || !comm->group) {
        const size_t slot_bytes = (size_t)p.q * 32;
        if (comm->group) local_allgather(comm, d_cvs + (size_t)p.rank * slot_bytes, d_cvs, slot_bytes, s);
        else NCCL_OK(ncclAllGather(d_cvs + (size_t)p.rank * slot_bytes, d_cvs, slot_bytes, ncclUint8, comm->comm, s));
    }
    check_rc(sd_split_checksum_root(ctx, split, d_cvs, d_hash32, stream));
    return SD_OK;
    SD_GUARD_END
}

}  // extern "C"
