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
// This file: the context, staging and device batches, the latency path, dedup, synthetic
// data and device utilities; the file-reading pipelines and the streaming hash are in
// sd_files.cpp, the types both share in sd_api_impl.h.
#include <ctype.h>
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

#include "sd_api_impl.h"

namespace sdi {

// ----------------------------------------------------------- checksum batches (device)
// (Re)plans `b` for these byte ranges reusing its device buffers (grow-only).  With a
// stream, the small uploads are async on it and read from b's host copies, which stay
// valid until the next rebuild of `b` (the caller syncs the stream before that).
void plan_checksum_batch(sd_checksum_batch* b, const uint64_t* offsets, const uint64_t* lens, size_t n,
                         hipStream_t stream) {
    plan_checksum(b->plan, offsets, lens, n);
    b->n = n;
    b->tab.begin();
    b->o_files = b->tab.add(b->plan.files);
    b->o_map = b->tab.add(b->plan.wg_map);
    b->o_pass.clear();
    for (const auto& ps : b->plan.passes) b->o_pass.push_back(b->tab.add(ps));
    b->tab.upload(stream);
    b->lvl[0].ensure(b->plan.lvl_cap[0] * 32);
    b->lvl[1].ensure(b->plan.lvl_cap[1] * 32);
}

void run_checksum_reduce(const sd_checksum_batch* b, uint32_t* out, hipStream_t s) {
    for (size_t k = 0; k < b->plan.passes.size(); k++) {
        const int src = (int)(k & 1);  // level 0 -> 1 -> 0 ...
        HIP_CHECK(sdk::launch_ck_reduce(b->lvl[src].as<uint32_t>(), b->lvl[1 - src].as<uint32_t>(),
                                        b->d_pass(k), (uint32_t)b->plan.passes[k].size(), out,
                                        s));
    }
}

void run_checksum_batch(const sd_checksum_batch* b, const uint8_t* d_data, uint8_t* d_hash32, hipStream_t s) {
    uint32_t* out = reinterpret_cast<uint32_t*>(d_hash32);
    HIP_CHECK(sdk::launch_ck_leaf(d_data, 0, 0, b->d_files(), b->d_map(),
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
    b->h_wrows.clear();
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
    b->whole_wave = b->n_whole <= (uint32_t)std::max(0, tuning_get(SD_TUNE_WHOLE_WAVE_MAX));
    if (b->whole_wave) {  // small batch: one workgroup per whole-kind message, no work lists
        b->whole = WholePlan{};
        for (size_t i = 0; i < n; i++) {
            const sd_extent& e = ext[i];
            if (e.kind != SD_KIND_SAMPLED && e.msg_len <= SD_WHOLE_ITEMS_MAX)
                b->h_wrows.push_back({(uint32_t)e.msg_offset, (uint32_t)(e.msg_offset >> 32), e.msg_len, (uint32_t)i});
        }
    } else {
        plan_whole_items(b->whole, ext, n);
    }
    b->tab.begin();
    b->o_sidx = b->tab.add(b->h_sidx);
    b->o_soff = b->tab.add(b->h_soff);
    b->o_full = b->tab.add(b->whole.full);
    b->o_tail = b->tab.add(b->whole.tail);
    b->o_ma = b->tab.add(b->whole.merge_a);
    b->o_mb = b->tab.add(b->whole.merge_b);
    b->o_lidx = b->tab.add(b->h_long_idx);
    b->o_wrows = b->tab.add(b->h_wrows);
    b->tab.upload(stream);
    b->cvbuf.ensure((size_t)b->whole.n_cv * 32);
    b->cv2.ensure((size_t)b->whole.n_cv2 * 32);
    b->sampled_wave = b->n_sampled <= (uint32_t)std::max(0, tuning_get(SD_TUNE_SAMPLED_WAVE_MAX));
    if (!b->sampled_wave) b->srows.ensure(sdk::cas_sampled_rows_bytes(b->n_sampled));
    if (b->n_long) {
        plan_checksum_batch(&b->lng, loff.data(), llen.data(), b->n_long, stream);
        b->compressions += b->lng.plan.compressions;
        b->long_out.ensure((size_t)b->n_long * 32);
    }
}

void run_cas_batch(const sd_cas_batch* b, const uint8_t* d_staged, uint8_t* d_hash32, hipStream_t s, int parts) {
    uint32_t* out = reinterpret_cast<uint32_t*>(d_hash32);
    // small batches take the latency kernels (one wave / workgroup per file), large ones the
    // throughput kernels; the plan chose ("sampled_wave_max", "whole_wave_max")
    if ((parts & SD_PART_SAMPLED) && b->sampled_wave)
        HIP_CHECK(sdk::launch_cas_sampled_wave(d_staged, b->d_soff(), b->d_sidx(), b->n_sampled, out, s));
    else if (parts & SD_PART_SAMPLED)
        HIP_CHECK(sdk::launch_cas_sampled(d_staged, b->d_soff(), b->d_sidx(), b->n_sampled, b->srows.as<uint32_t>(),
                                          out, s));
    if (parts & SD_PART_WHOLE) {
        const WholePlan& w = b->whole;
        if (b->whole_wave)
            HIP_CHECK(sdk::launch_whole_wave(d_staged, b->d_wrows(), (uint32_t)b->h_wrows.size(), out, s));
        else
            HIP_CHECK(sdk::launch_whole_items(d_staged, b->d_full(), (uint32_t)w.full.size(), b->d_tail(),
                                              (uint32_t)w.tail.size(), b->d_ma(), (uint32_t)w.merge_a.size(),
                                              b->d_mb(), (uint32_t)w.merge_b.size(), b->cvbuf.as<uint32_t>(),
                                              b->cv2.as<uint32_t>(), out, s));
        if (b->n_long) {
            run_checksum_batch(&b->lng, d_staged, b->long_out.as<uint8_t>(), s);
            HIP_CHECK(sdk::launch_scatter_hash(b->long_out.as<uint32_t>(), b->d_lidx(), b->n_long, out,
                                               s));
        }
    }
}

}  // namespace sdi

using namespace sdi;


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
    {  // the library's threads go to the device's NUMA node (sd_host.h, "numa_pin")
        char bdf[64] = {0};
        if (hipDeviceGetPCIBusId(bdf, sizeof bdf, device) == hipSuccess) {
            for (char* q = bdf; *q; q++) *q = (char)tolower(*q);
            const int node = pci_numa_node(bdf);
            numa_note_node(node);
            const std::string cpus = numa_node_cpulist(node);
            if (!cpus.empty()) numa_prefer_cpus(cpus.c_str());
        }
    }
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
    nthreads = cap_host_threads(nthreads);  // the process's host budget (sd_host.h)
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    std::atomic<size_t> cursor{0};
    auto work = [&](bool own_table) {
        if (own_table) private_fd_table();  // a thread of this call: its own fd table (stage_pool.h)
        for (;;) {
            const size_t i = cursor.fetch_add(1, std::memory_order_relaxed);
            if (i >= n) break;
            status[i] = stage_one(paths[i], extents[i], staged);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; t++) pool.emplace_back(work, true);
    work(false);
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
    // every live extent is checked before anything is hashed, whichever side will hash it
    for (size_t i : live) {
        validate_extent(extents[i], i);
        if (extents[i].msg_offset + extents[i].msg_len > staged_bytes)
            throw sd_failure(SD_ERR_INVALID, "extent beyond staged_bytes");
    }
    // windows of files (index order) whose staged span fits WINDOW bytes; two slots
    // alternate so window k+1's H2D copy overlaps window k's kernels
    const uint64_t WINDOW = 512ull << 20;
    struct Win {
        size_t gi = 0, gj = 0;
        bool busy = false;
    };
    SlotPair slots(ctx);
    Win wins[2];
    auto harvest = [&](int k) {
        if (!wins[k].busy) return;
        slots[k].sync();
        const uint8_t* h = slots[k].host_hashes.u8();
        for (size_t q = wins[k].gi; q < wins[k].gj; q++) {
            to_hex(h + (q - wins[k].gi) * 32, 8, out_hex17 + live[q] * 17);  // cas.rs:61 to_hex()[..16]
            if (status) status[live[q]] = SD_FILE_OK;
        }
        wins[k].busy = false;
    };
    // Co-hashing ("host_cohash_threads" h > 0, calls of >= 8192 files): the messages are
    // already in host memory, so feeding the GPU costs the host almost nothing (DMA), and the
    // call is bound by PCIe; h host threads hash files from the END of the list on the CPU
    // path meanwhile, claiming chunks of files, while the windows for the GPU are claimed
    // from the front -- under one lock, so the two meet wherever their rates put them.
    // (never more host threads than the process's host budget, less one for this thread)
    const int cohash = std::max(0, std::min({64, tuning_get(SD_TUNE_HOST_COHASH_THREADS), host_cpu_budget() - 1}));
    constexpr size_t COHASH_MIN = 8192, COHASH_CHUNK = 256;
    std::mutex claim_mu;
    size_t back = live.size();  // live[back, end) is claimed by the host threads
    size_t front = 0;           // live[0, front) is claimed by the GPU windows
    std::atomic<uint64_t> host_files{0};
    std::vector<std::thread> hosts;
    struct Join {
        std::vector<std::thread>& t;
        std::mutex& mu;
        size_t& back;
        ~Join() {  // on an exception below: stop claiming, then wait
            {
                std::lock_guard<std::mutex> g(mu);
                back = 0;
            }
            for (auto& x : t)
                if (x.joinable()) x.join();
        }
    } join_hosts{hosts, claim_mu, back};  // declared after everything the threads touch
    // while co-hashing, the GPU claims 128 MiB windows (~2 ms of PCIe each), so a mid-size
    // call is not taken whole by its first window before the host threads have started
    uint64_t window = WINDOW;
    if (cohash > 0 && live.size() >= COHASH_MIN) {
        window = 128ull << 20;
        for (int t = 0; t < cohash; t++)
            hosts.emplace_back([&] {
                library_thread_place();  // the device's NUMA node (sd_host.h)
                for (;;) {
                    size_t a, b;
                    {
                        std::lock_guard<std::mutex> g(claim_mu);
                        if (back <= front) return;
                        b = back;
                        a = b - std::min(COHASH_CHUNK, b - front);
                        back = a;
                    }
                    // 64 files at a time, their chunks packed across the SIMD lanes together
                    for (size_t q0 = a; q0 < b; q0 += 64) {
                        const size_t k = std::min<size_t>(64, b - q0);
                        const uint8_t* m[64];
                        uint64_t l[64];
                        uint8_t h[64][32];
                        for (size_t q = 0; q < k; q++) {
                            const sd_extent& e = extents[live[q0 + q]];  // validated above
                            m[q] = staged + e.msg_offset;
                            l[q] = e.msg_len;
                        }
                        cpu_blake3_batch(m, l, k, h);
                        for (size_t q = 0; q < k; q++) {
                            to_hex(h[q], 8, out_hex17 + live[q0 + q] * 17);  // cas.rs:61 to_hex()[..16]
                            if (status) status[live[q0 + q]] = SD_FILE_OK;
                        }
                    }
                    host_files.fetch_add(b - a, std::memory_order_relaxed);
                }
            });
    }
    std::vector<sd_extent> ext;
    size_t gi = 0;
    for (int w = 0;; w ^= 1) {
        harvest(w);  // frees slot w (its previous window is done)
        uint64_t lo = UINT64_MAX, hi = 0;
        size_t gj = gi;
        {
            std::lock_guard<std::mutex> g(claim_mu);
            while (gj < back) {
                const sd_extent& e = extents[live[gj]];
                const uint64_t nlo = std::min(lo, e.msg_offset);
                const uint64_t nhi = std::max(hi, align_up(e.msg_offset + e.msg_len, SD_STAGE_PAD));
                if (gj > gi && nhi - nlo > window) break;
                lo = nlo;
                hi = nhi;
                gj++;
            }
            front = gj;
        }
        if (gj == gi) break;  // the host threads hold the rest
        if (hi > staged_bytes) throw sd_failure(SD_ERR_INVALID, "extent beyond staged_bytes");
        ext.clear();
        for (size_t q = gi; q < gj; q++) {
            sd_extent e = extents[live[q]];
            e.msg_offset -= lo;
            ext.push_back(e);
        }
        Slot& sl = slots[w];
        plan_cas_batch(&sl.cas, ext.data(), ext.size(), sl.stream);
        sl.staged.ensure(hi - lo);
        sl.hashes.ensure(ext.size() * 32);
        sl.host_hashes.ensure(ext.size() * 32);
        HIP_CHECK(hipMemcpyAsync(sl.staged.p, staged + lo, hi - lo, hipMemcpyHostToDevice, sl.stream));
        run_cas_batch(&sl.cas, sl.staged.as<uint8_t>(), sl.hashes.as<uint8_t>(), sl.stream);
        HIP_CHECK(hipMemcpyAsync(sl.host_hashes.p, sl.hashes.p, ext.size() * 32, hipMemcpyDeviceToHost, sl.stream));
        wins[w] = Win{gi, gj, true};
        gi = gj;
    }
    harvest(0);
    harvest(1);
    for (auto& t : hosts) t.join();
    ctx->cas_ids_gpu_files.fetch_add(gi, std::memory_order_relaxed);
    ctx->cas_ids_host_files.fetch_add(host_files.load(), std::memory_order_relaxed);
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_ids_stats(sd_cas_ctx* ctx, uint64_t out[2]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = ctx->cas_ids_gpu_files.load(std::memory_order_relaxed);
    out[1] = ctx->cas_ids_host_files.load(std::memory_order_relaxed);
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

int sd_cas_ids_files_stats(sd_cas_ctx* ctx, uint64_t out[2]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = ctx->files_calls_cpu.load(std::memory_order_relaxed);
    out[1] = ctx->files_calls_gpu.load(std::memory_order_relaxed);
    return SD_OK;
    SD_GUARD_END
}

int sd_file_checksums_stats(sd_cas_ctx* ctx, uint64_t out[2]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = ctx->checksum_calls_cpu.load(std::memory_order_relaxed);
    out[1] = ctx->checksum_calls_gpu.load(std::memory_order_relaxed);
    return SD_OK;
    SD_GUARD_END
}

int sd_file_checksums_routes(sd_cas_ctx* ctx, uint64_t out[3]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = ctx->checksum_calls_cpu.load(std::memory_order_relaxed);
    out[1] = ctx->checksum_calls_gpu.load(std::memory_order_relaxed);
    out[2] = ctx->checksum_calls_hybrid.load(std::memory_order_relaxed);
    return SD_OK;
    SD_GUARD_END
}

int sd_file_checksums_bytes(sd_cas_ctx* ctx, uint64_t out[2]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = ctx->checksum_bytes_gpu.load(std::memory_order_relaxed);
    out[1] = ctx->checksum_bytes_cpu_split.load(std::memory_order_relaxed);
    return SD_OK;
    SD_GUARD_END
}

int sd_file_checksums_learned(sd_cas_ctx* ctx, double out[4]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> g(ctx->split_mu);
    const SplitRoutes& r = ctx->split_routes;
    out[0] = r.rate[0];
    out[1] = r.rate[1];
    out[2] = (double)r.n[0];
    out[3] = (double)r.n[1];
    return SD_OK;
    SD_GUARD_END
}

int sd_checksums_learned(sd_cas_ctx* ctx, double out[4]) {
    SD_GUARD_BEGIN
    if (!ctx || !out) throw sd_failure(SD_ERR_INVALID, "null argument");
    std::lock_guard<std::mutex> g(ctx->split_mu);
    const SplitRoutes& r = ctx->cohash_routes;
    out[0] = r.rate[0];
    out[1] = r.rate[1];
    out[2] = (double)r.n[0];
    out[3] = (double)r.n[1];
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
        HIP_CHECK(sdk::launch_ck_leaf(d_slice, p.off, 0, x->plan.d_files(),
                                      x->plan.d_map() + p.b0, (uint32_t)(p.b1 - p.b0), cvs, cvs,
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
    const uint32_t iters = 1024;  // ~5 ms a launch: the launch ramp is < 1%
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
    const double ops = (double)reps * grid * 256.0 * iters * sdk::VALU_PEAK_OPS_PER_ITER;
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
