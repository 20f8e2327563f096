// VALU issue probe, part 2: instruction MIXES and candidate BLAKE3 G-function encodings
// on gfx950.  Each kernel runs CH independent chains per lane of one inline-asm block;
// reported as blocks/s and as "G-equivalent lane-ops/s" (12 x G blocks per second).
// Build: hipcc --offload-arch=gfx950 -O3 -w -o /tmp/valu_probe2 scripts/valu_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CH 4
#define REP 8

// block bodies; a,b,c,d,t are per-chain registers, mx,my shared
#define B_FAST2 "v_xor_b32 %0, %0, %5\n v_add_u32 %0, %0, %6\n"
#define B_F1S1 "v_xor_b32 %0, %0, %5\n v_alignbit_b32 %0, %0, %0, 7\n"
#define B_F3S1 "v_xor_b32 %0, %0, %5\n v_add_u32 %0, %0, %6\n v_xor_b32 %0, %0, %6\n v_alignbit_b32 %0, %0, %0, 7\n"
#define B_SHR "v_lshrrev_b32 %0, 7, %0\n v_xor_b32 %0, %0, %5\n"
#define B_SDWA16                                                                              \
    "v_xor_b32_sdwa %4, %0, %5 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n" \
    "v_xor_b32_sdwa %4, %0, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" \
    "v_xor_b32_sdwa %0, %4, %6 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n" \
    "v_xor_b32_sdwa %0, %4, %6 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define B_MOVB "v_mov_b32_sdwa %0, %5 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n v_xor_b32 %0, %0, %6\n"

// G as the compiler emits it: add3 / xor / alignbit
#define G_REF(D)                                                     \
    "v_add3_u32 %0, %0, %1, %5\n v_xor_b32 " D ", " D ", %0\n v_alignbit_b32 " D ", " D ", " D ", 16\n" \
    "v_add_u32 %2, %2, " D "\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 12\n"            \
    "v_add3_u32 %0, %0, %1, %6\n v_xor_b32 " D ", " D ", %0\n v_alignbit_b32 " D ", " D ", " D ", 8\n" \
    "v_add_u32 %2, %2, " D "\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n"
// G with the two add3 split into plain adds
#define G_ADD2                                                                                   \
    "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %5\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 16\n" \
    "v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 12\n"                       \
    "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %6\n v_xor_b32 %3, %3, %0\n v_alignbit_b32 %3, %3, %3, 8\n"  \
    "v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n"
// G with the xor+rotr16 fused into two SDWA word-xors (d -> t, then the next G uses t)
#define G_SDWA(D, T)                                                                                        \
    "v_add3_u32 %0, %0, %1, %5\n"                                                                          \
    "v_xor_b32_sdwa " T ", " D ", %0 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n"  \
    "v_xor_b32_sdwa " T ", " D ", %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" \
    "v_add_u32 %2, %2, " T "\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 12\n"                       \
    "v_add3_u32 %0, %0, %1, %6\n v_xor_b32 " T ", " T ", %0\n v_alignbit_b32 " T ", " T ", " T ", 8\n"         \
    "v_add_u32 %2, %2, " T "\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n"
// G_SDWA plus rotr8 as xor, lshr 8, byte-3 insert (three 2-source ops)
#define G_SDWA8(D, T)                                                                                       \
    "v_add3_u32 %0, %0, %1, %5\n"                                                                          \
    "v_xor_b32_sdwa " T ", " D ", %0 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n"  \
    "v_xor_b32_sdwa " T ", " D ", %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" \
    "v_add_u32 %2, %2, " T "\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 12\n"                       \
    "v_add3_u32 %0, %0, %1, %6\n v_xor_b32 " D ", " T ", %0\n v_lshrrev_b32 " T ", 8, " D "\n"                  \
    "v_mov_b32_sdwa " T ", " D " dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n"                 \
    "v_add_u32 %2, %2, " T "\n v_xor_b32 %1, %1, %2\n v_alignbit_b32 %1, %1, %1, 7\n"

template <int KIND>
__global__ __launch_bounds__(256) void k_mix(uint32_t* sink, uint32_t iters) {
    uint32_t a[CH], b[CH], c[CH], d[CH], t[CH];
    const uint32_t mx = threadIdx.x * 0x9E3779B9u + blockIdx.x, my = mx ^ 0x5bd1e995u;
#pragma unroll
    for (int i = 0; i < CH; i++) {
        a[i] = mx + i;
        b[i] = my * (i + 3);
        c[i] = mx ^ (i * 77);
        d[i] = my + i * 0x1234567u;
        t[i] = 0;
    }
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#pragma unroll
            for (int i = 0; i < CH; i++) {
#define ASM(S) asm volatile(S : "+v"(a[i]), "+v"(b[i]), "+v"(c[i]), "+v"(d[i]), "+v"(t[i]) : "v"(mx), "v"(my))
                if (KIND == 0) ASM(B_FAST2);
                if (KIND == 1) ASM(B_F1S1);
                if (KIND == 2) ASM(B_F3S1);
                if (KIND == 3) ASM(B_SHR);
                if (KIND == 4) ASM(B_SDWA16);
                if (KIND == 5) ASM(B_MOVB);
                if (KIND == 6) ASM(G_REF("%3"));
                if (KIND == 7) ASM(G_ADD2);
                if (KIND == 8) ASM(G_SDWA("%3", "%4") G_SDWA("%4", "%3"));
                if (KIND == 9) ASM(G_SDWA8("%3", "%4") G_SDWA8("%4", "%3"));
#undef ASM
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) r ^= a[i] ^ b[i] ^ c[i] ^ d[i] ^ t[i];
    if (r == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

struct K {
    const char* name;
    void (*fn)(uint32_t*, uint32_t);
    double ops_per_block;   // instructions in one block
    double g_per_block;     // BLAKE3 G functions in one block (0 = not a G)
};

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    K ks[] = {{"xor,add (2 fast)", k_mix<0>, 2, 0},
              {"xor,alignbit (1f1s)", k_mix<1>, 2, 0},
              {"xor,add,xor,alignbit (3f1s)", k_mix<2>, 4, 0},
              {"lshrrev,xor", k_mix<3>, 2, 0},
              {"xor_sdwa x4", k_mix<4>, 4, 0},
              {"mov_sdwa byte,xor", k_mix<5>, 2, 0},
              {"G ref (add3/xor/alignbit)", k_mix<6>, 12, 1},
              {"G add3->2 add", k_mix<7>, 14, 1},
              {"G sdwa rotr16", k_mix<8>, 24, 2},
              {"G sdwa rotr16 + shr/byte rotr8", k_mix<9>, 26, 2}};
    uint32_t* sink;
    for (int wps : {1, 2, 4, 8}) {
        const int grid = p.multiProcessorCount * wps;
        (void)hipMalloc(&sink, (size_t)grid * 256 * 4);
        const uint32_t iters = 128;
        for (auto& k : ks) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, sink, iters);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, sink, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double blocks = 3.0 * grid * 256.0 * iters * REP * CH;
            const double s = ms * 1e-3;
            printf("waves/SIMD %d  %-32s instr %6.2f T lane-ops/s", wps, k.name, blocks * k.ops_per_block / s / 1e12);
            if (k.g_per_block > 0) printf("   G-equiv(12 ops/G) %6.2f T", blocks * k.g_per_block * 12 / s / 1e12);
            printf("\n");
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
        (void)hipFree(sink);
    }
    return 0;
}
