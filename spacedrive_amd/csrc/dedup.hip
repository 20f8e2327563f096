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

#include <cstring>

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

__global__ __launch_bounds__(256) void k_part_count(const uint8_t* __restrict__ hash32,
                                                    const uint8_t* __restrict__ valid, uint64_t n, int nparts,
                                                    unsigned long long* __restrict__ counts) {
    __shared__ unsigned long long local[64];
    if (threadIdx.x < 64) local[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (valid && !valid[i]) continue;
        atomicAdd(&local[dest_of(cas_key(hash32 + i * 32), nparts)], 1ull);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)nparts && local[threadIdx.x]) atomicAdd(&counts[threadIdx.x], local[threadIdx.x]);
}

// cursor[d] starts at the exclusive prefix of counts; records land grouped by destination
__global__ __launch_bounds__(256) void k_part_scatter(const uint8_t* __restrict__ hash32,
                                                      const uint8_t* __restrict__ valid, uint64_t n, uint64_t base,
                                                      int nparts, unsigned long long* __restrict__ cursor,
                                                      uint64_t* __restrict__ records) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (valid && !valid[i]) continue;
        const uint64_t key = cas_key(hash32 + i * 32);
        const unsigned long long pos = atomicAdd(&cursor[dest_of(key, nparts)], 1ull);
        records[2 * pos] = key;
        records[2 * pos + 1] = base + i;
    }
}

__global__ void k_prefix_small(const unsigned long long* counts, int nparts, unsigned long long* cursor) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        unsigned long long acc = 0;
        for (int d = 0; d < nparts; d++) { cursor[d] = acc; acc += counts[d]; }
        cursor[nparts] = acc;
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
                           uint64_t* counts, uint64_t* records, uint64_t* cursor_scratch, hipStream_t s) {
    auto* c = reinterpret_cast<unsigned long long*>(counts);
    auto* cur = reinterpret_cast<unsigned long long*>(cursor_scratch);
    hipError_t e = hipMemsetAsync(c, 0, sizeof(uint64_t) * nparts, s);
    if (e != hipSuccess) return e;
    if (n) hipLaunchKernelGGL(k_part_count, dim3(grid_for(n)), dim3(256), 0, s, hash32, valid, n, nparts, c);
    hipLaunchKernelGGL(k_prefix_small, dim3(1), dim3(64), 0, s, c, nparts, cur);
    if (n) hipLaunchKernelGGL(k_part_scatter, dim3(grid_for(n)), dim3(256), 0, s, hash32, valid, n, base, nparts, cur,
                              records);
    return hipGetLastError();
}

// scratch layout: keys[m], idx[m], keys2[m], idx2[m], heads[m], then rocprim temp storage
hipError_t dedup_group(uint64_t* records, uint64_t m, uint64_t* rep, uint64_t* n_groups_dev, void* scratch,
                       size_t* scratch_bytes, hipStream_t s) {
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
    // sort by index, then stable by cas_id: equal cas_ids end up in ascending index order
    size_t tb = temp;
    e = rocprim::radix_sort_pairs(tmp, tb, idx, idx2, keys, keys2, (size_t)m, 0, 64, s);
    if (e != hipSuccess) return e;
    tb = temp;
    e = rocprim::radix_sort_pairs(tmp, tb, keys2, keys, idx2, idx, (size_t)m, 0, 64, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_heads, dim3(grid_for(m)), dim3(256), 0, s, keys, m, heads, n_groups_dev);
    tb = temp;
    e = rocprim::inclusive_scan(tmp, tb, heads, keys2, (size_t)m, rocprim::maximum<uint64_t>(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_join, dim3(grid_for(m)), dim3(256), 0, s, keys, idx, keys2, m, records, rep);
    return hipGetLastError();
}

}  // namespace sdk
