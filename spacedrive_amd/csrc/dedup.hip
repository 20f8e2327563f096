// dedup.hip -- post-hash duplicate grouping (the cas_id -> Object link step).
//
// Reference semantics: identifier_job_step links each file_path to an Object owning an
// equal cas_id and otherwise creates one (core/src/object/file_identifier/mod.rs:136-333);
// size-0 files never take part (:80-88).  Here, per SURVEY.md §8(e): records
// (cas_id as a big-endian u64 of the first 8 hash bytes = the 16-hex string's order,
// global file index) are bucketed by the top bits of the cas_id for an all-to-all
// exchange across ranks, then each rank sorts its bucket and maps every record to the
// smallest file index of its equal-cas_id group (the Object-link candidate).
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cstring>
#include <utility>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "sd_internal.h"

namespace {

__device__ __forceinline__ uint64_t cas_key(const uint8_t* h) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(h);
    // bytes h[0..7] as a big-endian number == lexicographic order of the hex cas_id
    return ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
}

__device__ __forceinline__ uint32_t dest_of(uint64_t key, int nparts) {
    return (uint32_t)(((key >> 48) * (uint64_t)nparts) >> 16);  // top 16 bits scaled: contiguous ranges
}

// Deterministic, contention-free partition in two passes over a fixed grid of PART_BLOCKS
// workgroups, each owning one contiguous slice of the input:
//   count:   per (destination, block) histogram, wave-aggregated into LDS;
//   scan:    one workgroup turns the histogram into destination-major offsets;
//   scatter: each block walks its slice again in order; a record's position is its
//            block's offset for its destination + its rank among earlier records of the
//            same destination (ballot/popcount inside a wave, LDS counts across waves).
// Output is stable: grouped by destination, in input order within a destination.
constexpr uint32_t PART_BLOCKS = 1024;
constexpr uint32_t PART_MAXD = 64;

struct slice_t { uint64_t lo, hi; };
__device__ __forceinline__ slice_t slice_of(uint64_t n, uint32_t b) {
    const uint64_t per = (n + PART_BLOCKS - 1) / PART_BLOCKS;
    uint64_t lo = (uint64_t)b * per, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    return {lo, hi};
}

// rank of this lane among active lanes with the same destination, and that group's size
__device__ __forceinline__ void wave_match(bool active, uint32_t d, uint32_t& rank, uint32_t& size, bool& leader) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t remaining = __ballot(active);
    rank = 0; size = 0; leader = false;
    while (remaining) {
        const uint32_t first = __builtin_ctzll(remaining);
        const uint32_t dl = __shfl(d, first);
        const uint64_t m = __ballot(active && d == dl);
        if (active && d == dl) {
            rank = __popcll(m & ((1ull << lane) - 1));
            size = __popcll(m);
            leader = lane == first;
        }
        remaining &= ~m;
    }
}

__global__ __launch_bounds__(256) void k_part_count(const uint8_t* __restrict__ hash32,
                                                    const uint8_t* __restrict__ valid, uint64_t n, int nparts,
                                                    uint32_t* __restrict__ hist) {
    __shared__ uint32_t local[PART_MAXD];
    if (threadIdx.x < PART_MAXD) local[threadIdx.x] = 0;
    __syncthreads();
    const slice_t sl = slice_of(n, blockIdx.x);
    for (uint64_t base = sl.lo; base < sl.hi; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const bool act = i < sl.hi && (!valid || valid[i]);
        const uint32_t d = act ? dest_of(cas_key(hash32 + i * 32), nparts) : 0;
        uint32_t rank, size;
        bool leader;
        wave_match(act, d, rank, size, leader);
        if (leader) atomicAdd(&local[d], size);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)nparts) hist[threadIdx.x * PART_BLOCKS + blockIdx.x] = local[threadIdx.x];
}

// exclusive scan of hist[nparts * PART_BLOCKS] (destination-major) -> offs; counts[d]
__global__ __launch_bounds__(1024) void k_part_scan(const uint32_t* __restrict__ hist, int nparts,
                                                    uint64_t* __restrict__ offs,
                                                    unsigned long long* __restrict__ counts,
                                                    unsigned long long* __restrict__ total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int d = 0; d < nparts; d++) {
        const uint64_t v = hist[d * PART_BLOCKS + threadIdx.x];
        uint64_t x = v;  // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint64_t before = carry;
        for (uint32_t k = 0; k < w; k++) before += wsum[k];
        offs[d * PART_BLOCKS + threadIdx.x] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) {
            counts[d] = before + x - carry;
            carry = before + x;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void k_part_scatter(const uint8_t* __restrict__ hash32,
                                                      const uint8_t* __restrict__ valid, uint64_t n, uint64_t base_idx,
                                                      int nparts, const uint64_t* __restrict__ offs,
                                                      uint64_t* __restrict__ records) {
    __shared__ uint64_t run[PART_MAXD];
    __shared__ uint32_t wcnt[4][PART_MAXD];
    const uint32_t w = threadIdx.x >> 6;
    if (threadIdx.x < (unsigned)nparts) run[threadIdx.x] = offs[threadIdx.x * PART_BLOCKS + blockIdx.x];
    for (uint32_t k = threadIdx.x; k < 4 * PART_MAXD; k += blockDim.x) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    const slice_t sl = slice_of(n, blockIdx.x);
    for (uint64_t base = sl.lo; base < sl.hi; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const bool act = i < sl.hi && (!valid || valid[i]);
        const uint64_t key = act ? cas_key(hash32 + i * 32) : 0;
        const uint32_t d = act ? dest_of(key, nparts) : 0;
        uint32_t rank, size;
        bool leader;
        wave_match(act, d, rank, size, leader);
        if (leader) wcnt[w][d] = size;
        __syncthreads();
        if (act) {
            uint64_t pos = run[d] + rank;
            for (uint32_t k = 0; k < w; k++) pos += wcnt[k][d];
            records[2 * pos] = key;
            records[2 * pos + 1] = base_idx + i;
        }
        __syncthreads();
        if (threadIdx.x < (unsigned)nparts)
            run[threadIdx.x] += wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] + wcnt[3][threadIdx.x];
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < 4 * PART_MAXD; k += blockDim.x) (&wcnt[0][0])[k] = 0;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_split(const uint64_t* __restrict__ rec, uint64_t m, uint64_t* __restrict__ keys,
                                               uint64_t* __restrict__ idx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        keys[i] = rec[2 * i];
        idx[i] = rec[2 * i + 1];
    }
}

// after the (idx, then stable key) sorts: head positions, then max-scan -> group head
__global__ __launch_bounds__(256) void k_heads(const uint64_t* __restrict__ keys, uint64_t m,
                                               uint64_t* __restrict__ headpos, uint64_t* __restrict__ nheads) {
    __shared__ unsigned long long cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    unsigned long long mine = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const bool head = i == 0 || keys[i] != keys[i - 1];
        headpos[i] = head ? i : 0;
        mine += head;
    }
    atomicAdd(&cnt, mine);
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(nheads), cnt);
}

__global__ __launch_bounds__(256) void k_join(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ idx,
                                              const uint64_t* __restrict__ headscan, uint64_t m,
                                              uint64_t* __restrict__ rec, uint64_t* __restrict__ rep) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        rec[2 * i] = keys[i];
        rec[2 * i + 1] = idx[i];
        rep[i] = idx[headscan[i]];
    }
}

uint32_t grid_for(uint64_t n) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (uint32_t)g;
}

}  // namespace

namespace sdk {

hipError_t dedup_partition(const uint8_t* hash32, const uint8_t* valid, uint64_t n, uint64_t base, int nparts,
                           uint64_t* counts, uint64_t* records, uint64_t* scratch, hipStream_t s) {
    // scratch: hist (u32 nparts x PART_BLOCKS), offs (u64 nparts x PART_BLOCKS), total (u64)
    uint32_t* hist = reinterpret_cast<uint32_t*>(scratch);
    uint64_t* offs = scratch + (size_t)nparts * PART_BLOCKS / 2 + 1;
    auto* total = reinterpret_cast<unsigned long long*>(offs + (size_t)nparts * PART_BLOCKS);
    hipLaunchKernelGGL(k_part_count, dim3(PART_BLOCKS), dim3(256), 0, s, hash32, valid, n, nparts, hist);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(1024), 0, s, hist, nparts, offs,
                       reinterpret_cast<unsigned long long*>(counts), total);
    hipLaunchKernelGGL(k_part_scatter, dim3(PART_BLOCKS), dim3(256), 0, s, hash32, valid, n, base, nparts, offs,
                       records);
    return hipGetLastError();
}

size_t dedup_partition_scratch(int nparts) {
    return ((size_t)nparts * PART_BLOCKS / 2 + 1 + (size_t)nparts * PART_BLOCKS + 1) * sizeof(uint64_t);
}

// scratch layout: keys[m], idx[m], keys2[m], idx2[m], heads[m], then rocprim temp storage
hipError_t dedup_group(uint64_t* records, uint64_t m, int flags, uint64_t* rep, uint64_t* n_groups_dev,
                       void* scratch, size_t* scratch_bytes, hipStream_t s) {
    size_t sort_bytes = 0, scan_bytes = 0;
    uint64_t* nul = nullptr;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, sort_bytes, nul, nul, nul, nul, (size_t)m, 0, 64, s);
    if (e != hipSuccess) return e;
    e = rocprim::inclusive_scan(nullptr, scan_bytes, nul, nul, (size_t)m, rocprim::maximum<uint64_t>(), s);
    if (e != hipSuccess) return e;
    const size_t arrays = 5 * m * sizeof(uint64_t);
    size_t temp = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
    temp = (temp + 255) & ~size_t(255);
    const size_t need = arrays + temp + 256;
    if (scratch == nullptr) { *scratch_bytes = need; return hipSuccess; }
    if (*scratch_bytes < need) return hipErrorInvalidValue;
    uint64_t* keys = reinterpret_cast<uint64_t*>(scratch);
    uint64_t* idx = keys + m;
    uint64_t* keys2 = idx + m;
    uint64_t* idx2 = keys2 + m;
    uint64_t* heads = idx2 + m;
    void* tmp = reinterpret_cast<void*>(((uintptr_t)(heads + m) + 255) & ~uintptr_t(255));
    e = hipMemsetAsync(n_groups_dev, 0, sizeof(uint64_t), s);
    if (e != hipSuccess || m == 0) return e;
    hipLaunchKernelGGL(k_split, dim3(grid_for(m)), dim3(256), 0, s, records, m, keys, idx);
    size_t tb = temp;
    if (!(flags & SD_DEDUP_INDEX_SORTED)) {
        // sort by index first, so the stable cas_id sort below leaves equal cas_ids in
        // ascending index order
        e = rocprim::radix_sort_pairs(tmp, tb, idx, idx2, keys, keys2, (size_t)m, 0, 64, s);
        if (e != hipSuccess) return e;
        std::swap(keys, keys2);
        std::swap(idx, idx2);
        tb = temp;
    }
    e = rocprim::radix_sort_pairs(tmp, tb, keys, keys2, idx, idx2, (size_t)m, 0, 64, s);
    if (e != hipSuccess) return e;
    // grid-stride over at most 1024 workgroups: one global atomic per workgroup, so the
    // count does not serialise ~m/256 atomics on one L2 line
    hipLaunchKernelGGL(k_heads, dim3(std::min<unsigned>(grid_for(m), 1024u)), dim3(256), 0, s, keys2, m, heads,
                       n_groups_dev);
    tb = temp;
    e = rocprim::inclusive_scan(tmp, tb, heads, keys, (size_t)m, rocprim::maximum<uint64_t>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_join, dim3(grid_for(m)), dim3(256), 0, s, keys2, idx2, keys, m, records, rep);
    return hipGetLastError();
}

}  // namespace sdk
