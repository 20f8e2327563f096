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

// VALU ceiling of BLAKE3's G as the kernels issue it (blake3_device.h: 2x v_add3_u32,
// rotr16 as two crosswise v_xor_b32_sdwa, 2x v_add_u32, 3x v_xor_b32, 3x v_alignbit_b32),
// written in asm on hard-named VGPRs (v8..v35: <= 64 allocated, so 8 waves per SIMD fit)
// with no memory operation: 4 independent G columns per lane, interleaved op by op, the
// state fed back round after round.  scripts/valu_probe7.hip runs the same block beside
// per-op controls (profiles/r3/r3c_valu_probe7.txt).
#define VR(n) "v" #n
#define G_ADD3(a, b, m) "v_add3_u32 " VR(a) ", " VR(a) ", " VR(b) ", " VR(m) "\n"
#define G_R16A(t, d, a) "v_xor_b32_sdwa " VR(t) ", " VR(d) ", " VR(a) " dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n"
#define G_R16B(t, d, a) "v_xor_b32_sdwa " VR(t) ", " VR(d) ", " VR(a) " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define G_ADD(c, d) "v_add_u32 " VR(c) ", " VR(c) ", " VR(d) "\n"
#define G_XOR(x, y, z) "v_xor_b32 " VR(x) ", " VR(y) ", " VR(z) "\n"
#define G_ROT(x, n) "v_alignbit_b32 " VR(x) ", " VR(x) ", " VR(x) ", " #n "\n"
// column k: a = v(8+k), b = v(12+k), c = v(16+k), d = v(20+k), m0 = v(24+k), m1 = v(28+k), t = v(32+k)
#define G_COLS(OP, ...) OP(8, 12, 16, 20, 24, 28, 32) OP(9, 13, 17, 21, 25, 29, 33) OP(10, 14, 18, 22, 26, 30, 34) \
    OP(11, 15, 19, 23, 27, 31, 35)
#define S1(a, b, c, d, m0, m1, t) G_ADD3(a, b, m0)
#define S2(a, b, c, d, m0, m1, t) G_R16A(t, d, a)
#define S3(a, b, c, d, m0, m1, t) G_R16B(t, d, a)
#define S4(a, b, c, d, m0, m1, t) G_ADD(c, t)
#define S5(a, b, c, d, m0, m1, t) G_XOR(b, b, c)
#define S6(a, b, c, d, m0, m1, t) G_ROT(b, 12)
#define S7(a, b, c, d, m0, m1, t) G_ADD3(a, b, m1)
#define S8(a, b, c, d, m0, m1, t) G_XOR(d, t, a)
#define S9(a, b, c, d, m0, m1, t) G_ROT(d, 8)
#define S10(a, b, c, d, m0, m1, t) G_ADD(c, d)
#define S11(a, b, c, d, m0, m1, t) G_XOR(b, b, c)
#define S12(a, b, c, d, m0, m1, t) G_ROT(b, 7)
#define G_BLOCK                                                                                              \
    G_COLS(S1) G_COLS(S2) G_COLS(S3) G_COLS(S4) G_COLS(S5) G_COLS(S6) G_COLS(S7) G_COLS(S8) G_COLS(S9) \
        G_COLS(S10) G_COLS(S11) G_COLS(S12)
#define G_CLOB                                                                                                 \
    "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", \
        "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35"
static_assert(sdk::VALU_PEAK_OPS_PER_ITER == 8 * 48, "8 G blocks of 4 columns x 12 ops per iteration");
__global__ __launch_bounds__(256) void k_valu_peak(uint32_t* sink, uint32_t iters) {
    asm volatile(
        "v_mov_b32 v8, 1\nv_mov_b32 v9, 2\nv_mov_b32 v10, 3\nv_mov_b32 v11, 4\nv_mov_b32 v12, 5\nv_mov_b32 v13, 6\n"
        "v_mov_b32 v14, 7\nv_mov_b32 v15, 8\nv_mov_b32 v16, 9\nv_mov_b32 v17, 10\nv_mov_b32 v18, 11\nv_mov_b32 v19, 12\n"
        "v_mov_b32 v20, 13\nv_mov_b32 v21, 14\nv_mov_b32 v22, 15\nv_mov_b32 v23, 16\nv_mov_b32 v24, 17\nv_mov_b32 v25, 18\n"
        "v_mov_b32 v26, 19\nv_mov_b32 v27, 20\nv_mov_b32 v28, 21\nv_mov_b32 v29, 22\nv_mov_b32 v30, 23\nv_mov_b32 v31, 24\n"
        "v_mov_b32 v32, 0\nv_mov_b32 v33, 0\nv_mov_b32 v34, 0\nv_mov_b32 v35, 0" ::: G_CLOB);
    for (uint32_t i = 0; i < iters; i++) {
        asm volatile(G_BLOCK G_BLOCK G_BLOCK G_BLOCK ::: G_CLOB);
        asm volatile(G_BLOCK G_BLOCK G_BLOCK G_BLOCK ::: G_CLOB);
    }
    uint32_t r;
    asm volatile("v_xor_b32 %0, v8, v20" : "=v"(r));
    if (r == 0x12345678u && iters == 7) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
#undef G_BLOCK

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
    } else if (pattern == 3) {  // the same coalesced read, loads marked non-temporal (power per byte)
        for (uint64_t i = tid; i < bytes / 16; i += nthreads) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + i);
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
