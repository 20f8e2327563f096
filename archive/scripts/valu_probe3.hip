// VALU issue probe, part 3: does the ORDER of independent fast (2-source VOP2) and slow
// (3-source) ops change the issue rate on gfx950?  Four independent columns per lane (the
// four G functions of a BLAKE3 round are independent), emitted column by column or batched
// by step.  Generated op lists; each kernel runs one asm block of 4 columns per REP.
// Build: hipcc --offload-arch=gfx950 -O3 -w -o scripts/valu_probe3 scripts/valu_probe3.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP 8
#define BODY0 "v_add3_u32 %0, %0, %4, %16\nv_xor_b32 %12, %12, %0\nv_alignbit_b32 %12, %12, %12, 16\nv_add_u32 %8, %8, %12\nv_xor_b32 %4, %4, %8\nv_alignbit_b32 %4, %4, %4, 12\nv_add3_u32 %0, %0, %4, %17\nv_xor_b32 %12, %12, %0\nv_alignbit_b32 %12, %12, %12, 8\nv_add_u32 %8, %8, %12\nv_xor_b32 %4, %4, %8\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %1, %1, %5, %16\nv_xor_b32 %13, %13, %1\nv_alignbit_b32 %13, %13, %13, 16\nv_add_u32 %9, %9, %13\nv_xor_b32 %5, %5, %9\nv_alignbit_b32 %5, %5, %5, 12\nv_add3_u32 %1, %1, %5, %17\nv_xor_b32 %13, %13, %1\nv_alignbit_b32 %13, %13, %13, 8\nv_add_u32 %9, %9, %13\nv_xor_b32 %5, %5, %9\nv_alignbit_b32 %5, %5, %5, 7\nv_add3_u32 %2, %2, %6, %16\nv_xor_b32 %14, %14, %2\nv_alignbit_b32 %14, %14, %14, 16\nv_add_u32 %10, %10, %14\nv_xor_b32 %6, %6, %10\nv_alignbit_b32 %6, %6, %6, 12\nv_add3_u32 %2, %2, %6, %17\nv_xor_b32 %14, %14, %2\nv_alignbit_b32 %14, %14, %14, 8\nv_add_u32 %10, %10, %14\nv_xor_b32 %6, %6, %10\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %3, %3, %7, %16\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %11, %11, %15\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %3, %3, %7, %17\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %11, %11, %15\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY1 "v_add3_u32 %0, %0, %4, %16\nv_add3_u32 %1, %1, %5, %16\nv_add3_u32 %2, %2, %6, %16\nv_add3_u32 %3, %3, %7, %16\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 16\nv_alignbit_b32 %13, %13, %13, 16\nv_alignbit_b32 %14, %14, %14, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %0, %0, %4, %17\nv_add3_u32 %1, %1, %5, %17\nv_add3_u32 %2, %2, %6, %17\nv_add3_u32 %3, %3, %7, %17\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY2 "v_add3_u32 %0, %0, %4, %16\nv_add3_u32 %1, %1, %5, %16\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_alignbit_b32 %12, %12, %12, 16\nv_alignbit_b32 %13, %13, %13, 16\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_add3_u32 %0, %0, %4, %17\nv_add3_u32 %1, %1, %5, %17\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_alignbit_b32 %12, %12, %12, 8\nv_alignbit_b32 %13, %13, %13, 8\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_add3_u32 %2, %2, %6, %16\nv_add3_u32 %3, %3, %7, %16\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %14, %14, %14, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %2, %2, %6, %17\nv_add3_u32 %3, %3, %7, %17\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %14, %14, %14, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"
#define BODY3 "v_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7\n"
#define BODY4 "v_xor_b32 %4, %4, %8\nv_alignbit_b32 %13, %13, %13, 7\nv_xor_b32 %5, %5, %9\nv_alignbit_b32 %14, %14, %14, 7\nv_xor_b32 %6, %6, %10\nv_alignbit_b32 %15, %15, %15, 7\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %12, %12, %12, 7\n"
#define BODY5 "v_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\n"
#define BODY6 "v_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7\nv_add3_u32 %0, %0, %4, %16\nv_add3_u32 %1, %1, %5, %16\nv_add3_u32 %2, %2, %6, %16\nv_add3_u32 %3, %3, %7, %16\n"
#define BODY7 "v_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7\n"
#define BODY8 "v_add3_u32 %0, %0, %4, %16\nv_add3_u32 %1, %1, %5, %16\nv_add3_u32 %2, %2, %6, %16\nv_add3_u32 %3, %3, %7, %16\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_perm_b32 %12, %12, %12, %18\nv_perm_b32 %13, %13, %13, %18\nv_perm_b32 %14, %14, %14, %18\nv_perm_b32 %15, %15, %15, %18\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %6, %6, %6, 12\nv_alignbit_b32 %7, %7, %7, 12\nv_add3_u32 %0, %0, %4, %17\nv_add3_u32 %1, %1, %5, %17\nv_add3_u32 %2, %2, %6, %17\nv_add3_u32 %3, %3, %7, %17\nv_xor_b32 %12, %12, %0\nv_xor_b32 %13, %13, %1\nv_xor_b32 %14, %14, %2\nv_xor_b32 %15, %15, %3\nv_perm_b32 %12, %12, %12, %19\nv_perm_b32 %13, %13, %13, %19\nv_perm_b32 %14, %14, %14, %19\nv_perm_b32 %15, %15, %15, %19\nv_add_u32 %8, %8, %12\nv_add_u32 %9, %9, %13\nv_add_u32 %10, %10, %14\nv_add_u32 %11, %11, %15\nv_xor_b32 %4, %4, %8\nv_xor_b32 %5, %5, %9\nv_xor_b32 %6, %6, %10\nv_xor_b32 %7, %7, %11\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\n"

template <int KIND>
__global__ __launch_bounds__(256) void k_mix(uint32_t* sink, uint32_t iters) {
    const uint32_t mx = threadIdx.x * 0x9E3779B9u + blockIdx.x, my = mx ^ 0x5bd1e995u;
    const uint32_t sel16 = 0x01000302u + (iters >> 30), sel8 = 0x00030201u + (iters >> 30);  // byte selects: rotr 16, rotr 8
    uint32_t a0 = mx, a1 = mx + 1, a2 = mx + 2, a3 = mx + 3, b0 = my, b1 = my * 3, b2 = my * 5, b3 = my * 7;
    uint32_t c0 = mx ^ 77, c1 = mx ^ 78, c2 = mx ^ 79, c3 = mx ^ 80, d0 = my + 1, d1 = my + 2, d2 = my + 3, d3 = my + 4;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#define ASM(S)                                                                                            \
    asm volatile(S : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(c0), \
                 "+v"(c1), "+v"(c2), "+v"(c3), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)                       \
                 : "v"(mx), "v"(my), "s"(sel16), "s"(sel8))
            if (KIND == 0) ASM(BODY0);
            if (KIND == 1) ASM(BODY1);
            if (KIND == 2) ASM(BODY2);
            if (KIND == 3) ASM(BODY3);
            if (KIND == 4) ASM(BODY4);
            if (KIND == 5) ASM(BODY5);
            if (KIND == 6) ASM(BODY6);
            if (KIND == 7) ASM(BODY7);
            if (KIND == 8) ASM(BODY8);
#undef ASM
        }
    }
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ b0 ^ b1 ^ b2 ^ b3 ^ c0 ^ c1 ^ c2 ^ c3 ^ d0 ^ d1 ^ d2 ^ d3;
    if (r == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

struct K {
    const char* name;
    void (*fn)(uint32_t*, uint32_t);
    double ops;  // instructions per block
};

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    K ks[] = {
        {"G per column (4 G, col by col)", k_mix<0>, 48},
        {"G batched by step (4 G, op k of every col)", k_mix<1>, 48},
        {"G batched by 2 cols", k_mix<2>, 48},
        {"xor x4 | alignbit x4 (batched 1f1s)", k_mix<3>, 8},
        {"xor,alignbit alternating, independent", k_mix<4>, 8},
        {"fast only: xor x4, add x4", k_mix<5>, 8},
        {"slow only: alignbit x4, add3 x4", k_mix<6>, 8},
        {"xor x8 | alignbit x4 (2f:1s)", k_mix<7>, 12},
        {"perm rotr16/8 G batched by step", k_mix<8>, 48},
    };
    uint32_t* sink;
    for (int wps : {2, 4, 8}) {
        const int grid = p.multiProcessorCount * wps;
        (void)hipMalloc(&sink, (size_t)grid * 256 * 4);
        const uint32_t iters = 256;
        for (auto& k : ks) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            for (int w = 0; w < 20; w++) hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, sink, iters);  // clock up
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, sink, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double blocks = 5.0 * grid * 256.0 * iters * REP;
            printf("waves/SIMD %d  %-46s %6.2f T lane-ops/s\n", wps, k.name, blocks * k.ops / (ms * 1e-3) / 1e12);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
        (void)hipFree(sink);
    }
    return 0;
}
