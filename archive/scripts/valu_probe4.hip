// VALU issue probe, part 4: can BLAKE3's rotr16 leave the 3-source issue path?
// xor + v_alignbit(x,x,16) (one fast + one slow op) vs two VOP2-SDWA xors that write
// the two 16-bit halves crosswise (both 2-source ops).  Same four independent G columns
// as valu_probe3 (batched by step); every variant computes the same state, checked below.
// Build: hipcc --offload-arch=gfx950 -O3 -w -o scripts/valu_probe4 scripts/valu_probe4.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP 8
#define BODY0 "v_add3_u32 %0, %0, %4, %20\nv_add3_u32 %1, %1, %5, %20\nv_add3_u32 %2, %2, %6, %20\nv_add3_u32 %3, %3, %7, %20\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 16\nv_alignbit_b32 %13, %13, %13, 16\nv_alignbit_b32 %14, %14, %14, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %0, %0, %4, %21\nv_add3_u32 %1, %1, %5, %21\nv_add3_u32 %2, %2, %6, %21\nv_add3_u32 %3, %3, %7, %21\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY1 "v_add3_u32 %0, %0, %4, %20\nv_add3_u32 %1, %1, %5, %20\nv_add3_u32 %2, %2, %6, %20\nv_add3_u32 %3, %3, %7, %20\nv_xor_b32_sdwa %16, %12, %0 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %13, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %14, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %3 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %16, %12, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %17, %13, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %18, %14, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %19, %15, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_add_u32 %8, %8, %16\nv_add_u32 %9, %9, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %11, %11, %19\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %0, %0, %4, %21\nv_add3_u32 %1, %1, %5, %21\nv_add3_u32 %2, %2, %6, %21\nv_add3_u32 %3, %3, %7, %21\nv_xor_b32 %12, %16, %0\nv_xor_b32 %13, %17, %1\nv_xor_b32 %14, %18, %2\nv_xor_b32 %15, %19, %3\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY2 "v_add3_u32 %0, %0, %4, %20\nv_add3_u32 %1, %1, %5, %20\nv_add3_u32 %2, %2, %6, %20\nv_add3_u32 %3, %3, %7, %20\nv_xor_b32_sdwa %16, %12, %0 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %13, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %14, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %3 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %12, %12, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %13, %13, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %14, %14, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %15, %15, %3 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_or_b32 %16, %16, %12\nv_or_b32 %17, %17, %13\nv_or_b32 %18, %18, %14\nv_or_b32 %19, %19, %15\nv_add_u32 %8, %8, %16\nv_add_u32 %9, %9, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %11, %11, %19\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %0, %0, %4, %21\nv_add3_u32 %1, %1, %5, %21\nv_add3_u32 %2, %2, %6, %21\nv_add3_u32 %3, %3, %7, %21\nv_xor_b32 %12, %16, %0\nv_xor_b32 %13, %17, %1\nv_xor_b32 %14, %18, %2\nv_xor_b32 %15, %19, %3\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY3 "v_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %5\nv_add_u32 %2, %2, %6\nv_add_u32 %3, %3, %7\nv_add_u32 %0, %0, %20\nv_add_u32 %1, %1, %20\nv_add_u32 %2, %2, %20\nv_add_u32 %3, %3, %20\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 16\nv_alignbit_b32 %13, %13, %13, 16\nv_alignbit_b32 %14, %14, %14, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %5\nv_add_u32 %2, %2, %6\nv_add_u32 %3, %3, %7\nv_add_u32 %0, %0, %21\nv_add_u32 %1, %1, %21\nv_add_u32 %2, %2, %21\nv_add_u32 %3, %3, %21\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY4 "v_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %5\nv_add_u32 %2, %2, %6\nv_add_u32 %3, %3, %7\nv_add_u32 %0, %0, %20\nv_add_u32 %1, %1, %20\nv_add_u32 %2, %2, %20\nv_add_u32 %3, %3, %20\nv_xor_b32_sdwa %16, %12, %0 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %13, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %14, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %3 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %16, %12, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %17, %13, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %18, %14, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %19, %15, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_add_u32 %8, %8, %16\nv_add_u32 %9, %9, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %11, %11, %19\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %5\nv_add_u32 %2, %2, %6\nv_add_u32 %3, %3, %7\nv_add_u32 %0, %0, %21\nv_add_u32 %1, %1, %21\nv_add_u32 %2, %2, %21\nv_add_u32 %3, %3, %21\nv_xor_b32 %12, %16, %0\nv_xor_b32 %13, %17, %1\nv_xor_b32 %14, %18, %2\nv_xor_b32 %15, %19, %3\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"

template <int KIND>
__global__ __launch_bounds__(256) void k_mix(uint32_t* sink, uint32_t iters, uint32_t* out) {
    const uint32_t mx = threadIdx.x * 0x9E3779B9u + blockIdx.x, my = mx ^ 0x5bd1e995u;
    uint32_t a0 = mx, a1 = mx + 1, a2 = mx + 2, a3 = mx + 3, b0 = my, b1 = my * 3, b2 = my * 5, b3 = my * 7;
    uint32_t c0 = mx ^ 77, c1 = mx ^ 78, c2 = mx ^ 79, c3 = mx ^ 80, d0 = my + 1, d1 = my + 2, d2 = my + 3, d3 = my + 4;
    uint32_t t0 = mx ^ 1, t1 = mx ^ 2, t2 = mx ^ 3, t3 = mx ^ 4;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#define ASM(S)                                                                                            \
    asm volatile(S : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(c0), \
                 "+v"(c1), "+v"(c2), "+v"(c3), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3),    \
                 "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3)                                               \
                 : "v"(mx), "v"(my))
            if (KIND == 0) ASM(BODY0);
            if (KIND == 1) ASM(BODY1);
            if (KIND == 2) ASM(BODY2);
            if (KIND == 3) ASM(BODY3);
            if (KIND == 4) ASM(BODY4);
#undef ASM
        }
    }
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ b0 ^ b1 ^ b2 ^ b3 ^ c0 ^ c1 ^ c2 ^ c3 ^ d0 ^ d1 ^ d2 ^ d3;
    if (out) out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (r == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    void (*fns[])(uint32_t*, uint32_t, uint32_t*) = {k_mix<0>, k_mix<1>, k_mix<2>, k_mix<3>, k_mix<4>};
    const char* names[] = {"baseline: xor + alignbit16", "sdwa xor lo/hi (PRESERVE)", "sdwa xor lo, hi + v_or", "add3 as two v_add", "two v_add + sdwa PRESERVE"};
    uint32_t *sink, *chk;
    (void)hipMalloc(&chk, 5 * 256 * 4);
    uint32_t host[5][256];
    for (int k = 0; k < 5; k++) {
        hipLaunchKernelGGL(fns[k], dim3(1), dim3(256), 0, 0, chk, 3, chk + k * 256);
        (void)hipMemcpy(host[k], chk + k * 256, 1024, hipMemcpyDeviceToHost);
    }
    for (int k = 1; k < 5; k++) {
        int bad = 0;
        for (int i = 0; i < 256; i++) bad += host[k][i] != host[0][i];
        printf("%-30s state equal to baseline: %s (%d lanes differ)\n", names[k], bad ? "NO" : "yes", bad);
    }
    for (int wps : {4, 8}) {
        const int grid = p.multiProcessorCount * wps;
        (void)hipMalloc(&sink, (size_t)grid * 256 * 4);
        const uint32_t iters = 256;
        for (int pass = 0; pass < 2; pass++)
            for (int k = 0; k < 5; k++) {
                hipEvent_t e0, e1;
                (void)hipEventCreate(&e0);
                (void)hipEventCreate(&e1);
                for (int w = 0; w < 20; w++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, sink, iters, nullptr);
                (void)hipEventRecord(e0);
                for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, sink, iters, nullptr);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                const double blocks = 5.0 * grid * 256.0 * iters * REP;
                // 48 = the baseline's instruction count for 4 G: BLAKE3 work rate in baseline lane-ops
                printf("waves/SIMD %d pass %d  %-30s %6.2f T baseline lane-ops/s  %.3f ms\n", wps, pass, names[k],
                       blocks * 48 / (ms * 1e-3) / 1e12, ms);
                (void)hipEventDestroy(e0);
                (void)hipEventDestroy(e1);
            }
        (void)hipFree(sink);
    }
    return 0;
}
