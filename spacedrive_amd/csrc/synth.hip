// synth.hip -- device-side synthetic file generator and the VALU
// microbenchmark.  Not on the hashing path: it produces benchmark / parity inputs
// directly in HBM so multi-GB libraries never cross PCIe, bit-identical to the CPU
// generator in oracle/sd_oracle.c (sdo_synth_fill / sdo_synth_cas_message).
//
// byte o of content (cid, twin) = byte (o & 7) of splitmix64(SEED ^ cid*GOLDEN ^ (o >> 3)),
// and a twin XORs byte 18432 with (twin & 0xFF) | 1 -- outside every sample window of
// cas.rs:35-58, so twins share a cas_id but not a checksum.
#include <hip/hip_runtime.h>

#include "sd_internal.h"

namespace {

constexpr uint64_t SEED = 0x5D5DCA51Dull;
constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ull;
constexpr uint64_t TWIN_OFFSET = SD_HEADER_OR_FOOTER_SIZE + SD_SAMPLE_SIZE;

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// 8 content bytes starting at content offset o (any alignment), little-endian packed
__device__ __forceinline__ uint64_t content8(uint64_t key, uint64_t o, uint32_t twin) {
    const uint32_t sh = (uint32_t)(o & 7) * 8;
    uint64_t v = splitmix64(key ^ (o >> 3));
    if (sh) v = (v >> sh) | (splitmix64(key ^ ((o >> 3) + 1)) << (64 - sh));
    if (twin && o <= TWIN_OFFSET && TWIN_OFFSET < o + 8)
        v ^= (uint64_t)((twin & 0xFFu) | 1u) << (8 * (TWIN_OFFSET - o));
    return v;
}

// message position q (multiple of 8, q >= 8) -> content offset for a sampled message
__device__ __forceinline__ uint64_t sampled_src(uint64_t size, uint64_t q) {
    const uint64_t m = q - 8;  // position inside head||samples||tail
    const uint64_t H = SD_HEADER_OR_FOOTER_SIZE, S = SD_SAMPLE_SIZE;
    if (m < H) return m;
    if (m < H + 4 * S) {
        const uint64_t k = (m - H) / S;
        const uint64_t jump = (size - 2 * H) / SD_SAMPLE_COUNT;
        return H + k * jump + (m - H - k * S);
    }
    return size - H + (m - H - 4 * S);
}

__global__ __launch_bounds__(256) void k_synth_stage_cas(const uint64_t* __restrict__ sizes,
                                                         const uint64_t* __restrict__ cids,
                                                         const uint32_t* __restrict__ twins,
                                                         const sd_extent* __restrict__ ext, uint32_t n,
                                                         uint8_t* __restrict__ staged) {
    const uint32_t f = blockIdx.x;
    if (f >= n) return;
    const sd_extent e = ext[f];
    const uint64_t size = sizes[f];
    const uint64_t key = SEED ^ (cids[f] * GOLDEN);
    const uint32_t twin = twins ? twins[f] : 0u;
    const uint32_t padded = (e.msg_len + SD_STAGE_ALIGN - 1) & ~(SD_STAGE_ALIGN - 1);
    uint64_t* dst = reinterpret_cast<uint64_t*>(staged + e.msg_offset);
    for (uint32_t w = threadIdx.x; w < padded / 8; w += blockDim.x) {
        const uint64_t q = (uint64_t)w * 8;
        uint64_t v;
        if (q == 0) v = size;                         // cas.rs:25 le64(size)
        else if (q >= e.msg_len) v = 0;               // zero padding
        else {
            const uint64_t src = e.kind == SD_KIND_SAMPLED ? sampled_src(size, q) : q - 8;
            v = content8(key, src, twin);
            const uint64_t valid = e.msg_len - q;     // whole files: cut at the message end
            if (valid < 8) v &= (1ull << (8 * valid)) - 1;
        }
        dst[w] = v;
    }
}

__global__ __launch_bounds__(256) void k_synth_fill(uint64_t key, uint32_t twin, uint64_t offset, uint64_t len,
                                                    uint8_t* __restrict__ out) {
    const uint64_t words = (len + 7) / 8;
    uint64_t* o = reinterpret_cast<uint64_t*>(out);
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t v = content8(key, offset + w * 8, twin);
        if (w == words - 1 && (len & 7)) v &= (1ull << (8 * (len & 7))) - 1;
        o[w] = v;
    }
}

// VALU integer microbenchmark: 4 independent BLAKE3-style ARX chains per lane; each
// iteration is 12 ops x 4 chains (add3, add, xor, alignbit mix like one G function).
__global__ __launch_bounds__(256) void k_valu_peak(uint32_t* sink, uint32_t iters) {
    uint32_t a0 = threadIdx.x, b0 = blockIdx.x, c0 = 0x6A09E667u, d0 = 0xBB67AE85u;
    uint32_t a1 = a0 ^ 1, b1 = b0 ^ 3, c1 = c0 ^ 5, d1 = d0 ^ 7;
    uint32_t a2 = a0 ^ 11, b2 = b0 ^ 13, c2 = c0 ^ 17, d2 = d0 ^ 19;
    uint32_t a3 = a0 ^ 23, b3 = b0 ^ 29, c3 = c0 ^ 31, d3 = d0 ^ 37;
    const uint32_t mx = iters * 7u, my = iters * 13u;
#define VG(a, b, c, d)                                                          \
    a = a + b + mx; d = __builtin_amdgcn_alignbit(d ^ a, d ^ a, 16);            \
    c = c + d;      b = __builtin_amdgcn_alignbit(b ^ c, b ^ c, 12);            \
    a = a + b + my; d = __builtin_amdgcn_alignbit(d ^ a, d ^ a, 8);             \
    c = c + d;      b = __builtin_amdgcn_alignbit(b ^ c, b ^ c, 7);
    for (uint32_t i = 0; i < iters; i++) {
        VG(a0, b0, c0, d0) VG(a1, b1, c1, d1) VG(a2, b2, c2, d2) VG(a3, b3, c3, d3)
        VG(a0, b0, c0, d0) VG(a1, b1, c1, d1) VG(a2, b2, c2, d2) VG(a3, b3, c3, d3)
    }
#undef VG
    const uint32_t r = a0 ^ b0 ^ c0 ^ d0 ^ a1 ^ b1 ^ c1 ^ d1 ^ a2 ^ b2 ^ c2 ^ d2 ^ a3 ^ b3 ^ c3 ^ d3;
    if (r == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// Read probe: XOR-reduces the buffer so nothing is dead-code eliminated; writes one word
// per workgroup only if the reduction hits a sentinel (never, in practice).
__global__ __launch_bounds__(256) void k_read_probe(const uint8_t* __restrict__ buf, uint64_t bytes, int pattern,
                                                    uint32_t* __restrict__ sink) {
    const uint4* b = reinterpret_cast<const uint4*>(buf);
    uint32_t acc = 0;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    if (pattern == 0) {
        for (uint64_t i = tid; i < bytes / 16; i += nthreads) {
            const uint4 v = b[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    } else {
        const uint32_t per = pattern == 2 ? 2048u : 1024u;  // bytes per lane
        for (uint64_t lane = tid; lane < bytes / per; lane += nthreads) {
            const uint4* q = b + lane * (per / 16);
            for (uint32_t blk = 0; blk < per / 64; blk++) {
                for (int k = 0; k < 4; k++) {
                    const uint4 v = q[blk * 4 + k];
                    acc ^= v.x ^ v.y ^ v.z ^ v.w;
                }
            }
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

}  // namespace

namespace sdk {

hipError_t launch_read_probe(const uint8_t* buf, uint64_t bytes, int pattern, hipStream_t s) {
    static uint32_t* sink = nullptr;
    if (!sink) {
        hipError_t e = hipMalloc(&sink, 4096 * sizeof(uint32_t));
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_read_probe, dim3(4096), dim3(256), 0, s, buf, bytes, pattern, sink);
    return hipGetLastError();
}

hipError_t launch_synth_stage_cas(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins,
                                  const sd_extent* ext, uint32_t n, uint8_t* staged, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth_stage_cas, dim3(n), dim3(256), 0, s, sizes, cids, twins, ext, n, staged);
    return hipGetLastError();
}

hipError_t launch_synth_fill(uint64_t cid, uint32_t twin, uint64_t offset, uint64_t len, uint8_t* out,
                             hipStream_t s) {
    if (len == 0) return hipSuccess;
    const uint64_t words = (len + 7) / 8;
    uint64_t grid = (words + 255) / 256;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(k_synth_fill, dim3((uint32_t)grid), dim3(256), 0, s, SEED ^ (cid * GOLDEN), twin, offset, len,
                       out);
    return hipGetLastError();
}

hipError_t launch_valu_peak(uint32_t* sink, uint32_t iters, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(k_valu_peak, dim3(grid), dim3(256), 0, s, sink, iters);
    return hipGetLastError();
}

}  // namespace sdk
