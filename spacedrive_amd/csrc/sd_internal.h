// sd_internal.h -- types shared between the host-side C ABI and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sd_cas.h"
#include "sd_host.h"

// the device a context was created on
int sd_ctx_device(const sd_cas_ctx* ctx);
// sd_dedup_group followed by sd_dedup_owners (owner_chunk > 0) with a single host sync
void dedup_group_owners(sd_cas_ctx* ctx, uint64_t* d_records, uint64_t m, int flags, uint64_t* d_rep,
                        uint64_t owner_chunk, uint64_t* d_owner, uint64_t* n_groups, hipStream_t s);
// the block partition of a split-file checksum object
const SplitPlan& sd_split_plan_of(const sd_split_checksum* x);
namespace sdk {
// soff[i] = msg_offset of sampled file i, idx[i] = its index in the batch (the output slot)
// sampled cas (two kernels: lanes of 8 chunks, then the per-file merge) through `rows`
uint64_t cas_sampled_rows_bytes(uint32_t n);
hipError_t launch_cas_sampled(const uint8_t* staged, const uint64_t* soff, const uint32_t* idx, uint32_t n,
                              uint32_t* rows, uint32_t* out, hipStream_t s);
// the same for small batches: one wave per file, 16 + 6 dependent compressions (latency)
hipError_t launch_cas_sampled_wave(const uint8_t* staged, const uint64_t* soff, const uint32_t* idx, uint32_t n,
                                   uint32_t* out, hipStream_t s);
// whole-kind messages of <= 101 chunks, small batches: one workgroup per message (latency);
// rows = (u64 message offset, length, output row)
hipError_t launch_whole_wave(const uint8_t* staged, const uint4* rows, uint32_t n, uint32_t* out, hipStream_t s);
// whole-file work lists: full-pair items, cost-sorted tail items, two merge8 passes (cv2 =
// pass-A output)
hipError_t launch_whole_items(const uint8_t* staged, const uint4* full, uint32_t n_full, const uint4* tail,
                              uint32_t n_tail, const uint4* merge_a, uint32_t n_a, const uint4* merge_b, uint32_t n_b,
                              uint32_t* cvbuf, uint32_t* cv2, uint32_t* out, hipStream_t s);
hipError_t launch_scatter_hash(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* out, hipStream_t s);
hipError_t launch_ck_leaf(const uint8_t* data, uint64_t shift, uint32_t blk_base, const ck_file* files,
                          const uint2* wg_map, uint32_t n_wg, uint32_t* cvbuf, uint32_t* out, hipStream_t s);
hipError_t launch_ck_reduce(const uint32_t* src, uint32_t* dst, const ck_reduce_wg* wgs, uint32_t n_wg,
                            uint32_t* out, hipStream_t s);
hipError_t launch_synth_stage_cas(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins,
                                  const sd_extent* ext, uint32_t n, uint8_t* staged, hipStream_t s);
hipError_t launch_synth_fill(uint64_t cid, uint32_t twin, uint64_t offset, uint64_t len, uint8_t* out,
                             hipStream_t s);
hipError_t launch_read_probe(const uint8_t* buf, uint64_t bytes, int pattern, hipStream_t s);
constexpr uint32_t VALU_PEAK_OPS_PER_ITER = 384;  // k_valu_peak: VALU instructions per wave per iteration
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
