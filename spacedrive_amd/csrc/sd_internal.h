// sd_internal.h -- types shared between the host-side C ABI and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sd_cas.h"

// one file of a checksum batch (device table)
struct ck_file {
    uint64_t offset;   // byte offset in the data buffer
    uint64_t len;      // file length
    uint64_t cv_base;  // first slot of this file's 1 MiB block CVs in the level-0 CV buffer
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

// process-wide tuning knobs (sd_cas_set_tuning); read at launch time
enum sd_tune_key {
    SD_TUNE_SAMPLED_VARIANT = 0,
    SD_TUNE_WHOLE_VARIANT = 1,
    SD_TUNE_CK_VARIANT = 2,
    SD_TUNE_COALESCE_US = 3,
    SD_TUNE_COALESCE_MAX = 4,
    SD_TUNE_FILES_WINDOW_MB = 5,
    SD_TUNE_WHOLE_LDS_KB = 6,  // dynamic LDS per k_whole_items workgroup (occupancy A/B; 0 = none)
    SD_TUNE_DEDUP_VARIANT = 7,  // sd_dedup_group: 0 = radix sort, 1 = LDS buckets (radix on overflow)
    SD_TUNE_NKEYS = 8
};
int tuning_get(int key);
// What the kernels need of a staged message: a 16-byte aligned start (validate_extent) and
// zero padding up to the next 64-byte boundary.  The planner places messages on
// SD_STAGE_ALIGN (128, whole cache lines) but callers' own layouts only need this.
constexpr uint64_t SD_STAGE_PAD = 64;

// latency path (coalesce.cpp)
#include <string>
struct sd_coalescer;
sd_coalescer* coalescer_create(sd_cas_ctx* ctx);
void coalescer_destroy(sd_coalescer* c);
int coalescer_submit(sd_coalescer* c, int kind, const char* path, uint64_t size, char* out, int32_t* status,
                     std::string* err);
void coalescer_stats(sd_coalescer* c, uint64_t out[3]);

namespace sdk {
hipError_t launch_cas_sampled(const uint8_t* staged, const sd_extent* ext, const uint32_t* idx, uint32_t n,
                              uint32_t* out, hipStream_t s);
hipError_t launch_cas_mixed(const uint8_t* staged, const sd_extent* ext, const uint32_t* sidx, uint32_t n_sampled,
                            const uint32_t* order, const uint2* groups, uint32_t n_groups, uint32_t* out,
                            hipStream_t s, bool pairpf);
hipError_t launch_whole_forest(const uint32_t* order, const uint32_t* pair_prefix, const uint2* groups,
                               uint32_t n_groups, const uint32_t* cvbuf, uint32_t* out, hipStream_t s);
hipError_t launch_whole_pair_leaf(const uint8_t* staged, const sd_extent* ext, const uint32_t* order,
                                  const uint32_t* pair_prefix, const uint32_t* hint, uint32_t nw, uint32_t total_pairs,
                                  uint32_t* cvbuf, uint32_t* out, hipStream_t s);
hipError_t launch_whole_leaf(const uint8_t* staged, const sd_extent* ext, const uint32_t* order,
                             const uint32_t* chunk_prefix, const uint32_t* hint, uint32_t nw, uint32_t total_chunks,
                             uint32_t* cvbuf, uint32_t* out, hipStream_t s);
hipError_t launch_whole_tree(const uint32_t* order, const uint32_t* chunk_prefix, uint32_t n_multi, uint32_t* cvbuf,
                             uint32_t* out, hipStream_t s);
hipError_t launch_whole(const uint8_t* staged, const sd_extent* ext, const uint32_t* order,
                        const uint32_t* chunk_prefix, const uint32_t* hint, uint32_t nw, uint32_t total_chunks,
                        uint32_t n_multi, uint32_t* cvbuf, uint32_t* out, hipStream_t s);
// variant 6: full-pair items, cost-sorted tail items, two merge8 passes (cv2 = pass-A output)
hipError_t launch_whole_items(const uint8_t* staged, const uint4* full, uint32_t n_full, const uint4* tail,
                              uint32_t n_tail, const uint4* merge_a, uint32_t n_a, const uint4* merge_b, uint32_t n_b,
                              uint32_t* cvbuf, uint32_t* cv2, uint32_t* out, hipStream_t s, bool combined, int pf);
hipError_t launch_ck_leaf(const uint8_t* data, uint64_t shift, const ck_file* files, const uint2* wg_map,
                          uint32_t n_wg, uint32_t* cvbuf, uint32_t* out, hipStream_t s);
hipError_t launch_ck_reduce(const uint32_t* src, uint32_t* dst, const ck_reduce_wg* wgs, uint32_t n_wg,
                            uint32_t* out, hipStream_t s);
hipError_t launch_synth_stage_cas(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins,
                                  const sd_extent* ext, uint32_t n, uint8_t* staged, hipStream_t s);
hipError_t launch_synth_fill(uint64_t cid, uint32_t twin, uint64_t len, uint8_t* out, hipStream_t s);
hipError_t launch_read_probe(const uint8_t* buf, uint64_t bytes, int pattern, hipStream_t s);
hipError_t launch_valu_peak(uint32_t* sink, uint32_t iters, uint32_t grid, hipStream_t s);
// dedup
hipError_t dedup_partition(const uint8_t* hash32, const uint8_t* valid, uint64_t n, uint64_t base, int nparts,
                           uint64_t* counts, uint64_t* records, uint64_t* scratch, hipStream_t s);
// device scratch bytes dedup_partition needs; the valid-record total is its last u64
size_t dedup_partition_scratch(int nparts);
hipError_t dedup_group(uint64_t* records, uint64_t m, int flags, uint64_t* rep, uint64_t* n_groups_dev,
                       void* scratch, size_t* scratch_bytes, hipStream_t s);
// bucket grouping (dedup_variant 1): same outputs as dedup_group for m < 2^31 unless
// state[1] (overflow) comes back nonzero -- then records hold a permutation of the input
// and dedup_group (without SD_DEDUP_INDEX_SORTED) must run.  state: 6 device u64, state[0]
// = the group count.
size_t dedup_group_buckets_scratch(uint64_t m);
hipError_t dedup_group_buckets(uint64_t* records, uint64_t m, uint64_t* rep, uint64_t* state, void* scratch,
                               size_t scratch_bytes, hipStream_t s);
hipError_t dedup_owners(const uint64_t* records, uint64_t m, const uint64_t* rep, uint64_t chunk, uint64_t* owner,
                        hipStream_t s);
}  // namespace sdk
