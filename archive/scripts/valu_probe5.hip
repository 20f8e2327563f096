// VALU issue probe, part 5: is the slow rate of gfx950's 3-source ops an operand-read
// (VGPR bank) cost or an encoding/issue cost?  Each kernel issues 8 independent ops of one
// kind per asm block on hard-named VGPRs (banks = register index mod 4), so the bank
// pattern of the sources is fixed: one bank vs distinct banks, same register twice, an
// SGPR source, the 2-source op in VOP3 encoding, and SDWA/VOP3P forms.
// Build: hipcc --offload-arch=gfx950 -O3 -w -o scripts/valu_probe5 scripts/valu_probe5.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP 16
#define BODY0 "v_xor_b32 v32, v40, v48\nv_xor_b32 v33, v41, v49\nv_xor_b32 v34, v42, v50\nv_xor_b32 v35, v43, v51\nv_xor_b32 v36, v44, v52\nv_xor_b32 v37, v45, v53\nv_xor_b32 v38, v46, v54\nv_xor_b32 v39, v47, v55\n"
#define BODY1 "v_xor_b32_e64 v32, v40, v48\nv_xor_b32_e64 v33, v41, v49\nv_xor_b32_e64 v34, v42, v50\nv_xor_b32_e64 v35, v43, v51\nv_xor_b32_e64 v36, v44, v52\nv_xor_b32_e64 v37, v45, v53\nv_xor_b32_e64 v38, v46, v54\nv_xor_b32_e64 v39, v47, v55\n"
#define BODY2 "v_or3_b32 v32, v40, v41, v42\nv_or3_b32 v33, v44, v45, v46\nv_or3_b32 v34, v48, v49, v50\nv_or3_b32 v35, v52, v53, v54\nv_or3_b32 v36, v40, v41, v42\nv_or3_b32 v37, v44, v45, v46\nv_or3_b32 v38, v48, v49, v50\nv_or3_b32 v39, v52, v53, v54\n"
#define BODY3 "v_or3_b32 v32, v40, v48, v56\nv_or3_b32 v33, v41, v49, v57\nv_or3_b32 v34, v42, v50, v58\nv_or3_b32 v35, v43, v51, v59\nv_or3_b32 v36, v44, v52, v60\nv_or3_b32 v37, v45, v53, v61\nv_or3_b32 v38, v46, v54, v62\nv_or3_b32 v39, v47, v55, v63\n"
#define BODY4 "v_alignbit_b32 v32, v40, v40, 7\nv_alignbit_b32 v33, v41, v41, 7\nv_alignbit_b32 v34, v42, v42, 7\nv_alignbit_b32 v35, v43, v43, 7\nv_alignbit_b32 v36, v44, v44, 7\nv_alignbit_b32 v37, v45, v45, 7\nv_alignbit_b32 v38, v46, v46, 7\nv_alignbit_b32 v39, v47, v47, 7\n"
#define BODY5 "v_alignbit_b32 v32, v40, v41, 7\nv_alignbit_b32 v33, v44, v45, 7\nv_alignbit_b32 v34, v48, v49, 7\nv_alignbit_b32 v35, v52, v53, 7\nv_alignbit_b32 v36, v40, v41, 7\nv_alignbit_b32 v37, v44, v45, 7\nv_alignbit_b32 v38, v48, v49, 7\nv_alignbit_b32 v39, v52, v53, 7\n"
#define BODY6 "v_alignbit_b32 v32, v40, v48, 7\nv_alignbit_b32 v33, v41, v49, 7\nv_alignbit_b32 v34, v42, v50, 7\nv_alignbit_b32 v35, v43, v51, 7\nv_alignbit_b32 v36, v44, v52, 7\nv_alignbit_b32 v37, v45, v53, 7\nv_alignbit_b32 v38, v46, v54, 7\nv_alignbit_b32 v39, v47, v55, 7\n"
#define BODY7 "v_add3_u32 v32, v40, v41, v42\nv_add3_u32 v33, v44, v45, v46\nv_add3_u32 v34, v48, v49, v50\nv_add3_u32 v35, v52, v53, v54\nv_add3_u32 v36, v40, v41, v42\nv_add3_u32 v37, v44, v45, v46\nv_add3_u32 v38, v48, v49, v50\nv_add3_u32 v39, v52, v53, v54\n"
#define BODY8 "v_add3_u32 v32, v40, v48, v56\nv_add3_u32 v33, v41, v49, v57\nv_add3_u32 v34, v42, v50, v58\nv_add3_u32 v35, v43, v51, v59\nv_add3_u32 v36, v44, v52, v60\nv_add3_u32 v37, v45, v53, v61\nv_add3_u32 v38, v46, v54, v62\nv_add3_u32 v39, v47, v55, v63\n"
#define BODY9 "v_add3_u32 v32, v40, v41, s4\nv_add3_u32 v33, v44, v45, s4\nv_add3_u32 v34, v48, v49, s4\nv_add3_u32 v35, v52, v53, s4\nv_add3_u32 v36, v40, v41, s4\nv_add3_u32 v37, v44, v45, s4\nv_add3_u32 v38, v48, v49, s4\nv_add3_u32 v39, v52, v53, s4\n"
#define BODY10 "v_lshl_or_b32 v32, v40, 7, v41\nv_lshl_or_b32 v33, v44, 7, v45\nv_lshl_or_b32 v34, v48, 7, v49\nv_lshl_or_b32 v35, v52, 7, v53\nv_lshl_or_b32 v36, v40, 7, v41\nv_lshl_or_b32 v37, v44, 7, v45\nv_lshl_or_b32 v38, v48, 7, v49\nv_lshl_or_b32 v39, v52, 7, v53\n"
#define BODY11 "v_perm_b32 v32, v40, v40, s5\nv_perm_b32 v33, v41, v41, s5\nv_perm_b32 v34, v42, v42, s5\nv_perm_b32 v35, v43, v43, s5\nv_perm_b32 v36, v44, v44, s5\nv_perm_b32 v37, v45, v45, s5\nv_perm_b32 v38, v46, v46, s5\nv_perm_b32 v39, v47, v47, s5\n"
#define BODY12 "v_xor_b32_sdwa v32, v40, v48 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v33, v41, v49 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v34, v42, v50 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v35, v43, v51 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v36, v44, v52 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v37, v45, v53 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v38, v46, v54 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa v39, v47, v55 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define BODY13 "v_xor_b32_sdwa v32, v40, v48 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v33, v41, v49 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v34, v42, v50 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v35, v43, v51 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v36, v44, v52 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v37, v45, v53 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v38, v46, v54 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa v39, v47, v55 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n"
#define BODY14 "v_pk_add_u16 v32, v40, v48\nv_pk_add_u16 v33, v41, v49\nv_pk_add_u16 v34, v42, v50\nv_pk_add_u16 v35, v43, v51\nv_pk_add_u16 v36, v44, v52\nv_pk_add_u16 v37, v45, v53\nv_pk_add_u16 v38, v46, v54\nv_pk_add_u16 v39, v47, v55\n"
#define BODY15 "v_add_u32 v32, v40, v48\nv_alignbit_b32 v33, v44, v45, 7\nv_add_u32 v34, v42, v50\nv_alignbit_b32 v35, v52, v53, 7\nv_add_u32 v36, v44, v52\nv_alignbit_b32 v37, v44, v45, 7\nv_add_u32 v38, v46, v54\nv_alignbit_b32 v39, v52, v53, 7\n"
#define NKINDS 16
static const char* kNames[] = {
    "v_xor_b32 (VOP2)",
    "v_xor_b32_e64 (VOP3 encoding, 2 src)",
    "v_or3_b32 distinct banks",
    "v_or3_b32 one bank",
    "v_alignbit x,x,x (same reg twice)",
    "v_alignbit x,y,7 distinct banks",
    "v_alignbit x,y,7 one bank",
    "v_add3_u32 distinct banks",
    "v_add3_u32 one bank",
    "v_add3_u32 2 vgpr + sgpr",
    "v_lshl_or_b32 distinct banks",
    "v_perm_b32 (rotr16 sel in sgpr)",
    "v_xor_b32_sdwa WORD_1 PRESERVE",
    "v_xor_b32_sdwa WORD_0 PAD",
    "v_pk_add_u16",
    "v_add_u32 + v_alignbit distinct (1f1s)"};

#define CLOB "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "s4", "s5"
template <int KIND>
__global__ __launch_bounds__(256) void k_op(uint32_t* sink, uint32_t iters) {
    asm volatile("s_mov_b32 s4, 0x12345\ns_mov_b32 s5, 0x01000302" ::: "s4", "s5");
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#define B(K) if (KIND == K) asm volatile(BODY##K ::: CLOB);
            B(0) B(1) B(2) B(3) B(4) B(5) B(6) B(7) B(8) B(9) B(10) B(11) B(12) B(13) B(14) B(15)
#undef B
        }
    }
    uint32_t r;
    asm volatile("v_mov_b32 %0, v32" : "=v"(r));
    if (r == 0x12345678u && iters == 7) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    static_assert(NKINDS == 16, "kinds");
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    void (*fns[])(uint32_t*, uint32_t) = {k_op<0>, k_op<1>, k_op<2>,  k_op<3>,  k_op<4>,  k_op<5>,  k_op<6>,  k_op<7>,
                                          k_op<8>, k_op<9>, k_op<10>, k_op<11>, k_op<12>, k_op<13>, k_op<14>, k_op<15>};
    uint32_t* sink;
    for (int wps : {4, 8}) {
        const int grid = p.multiProcessorCount * wps;
        (void)hipMalloc(&sink, (size_t)grid * 256 * 4);
        const uint32_t iters = 256;
        for (int k = 0; k < NKINDS; k++) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            for (int w = 0; w < 20; w++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, sink, iters);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, sink, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double ops = 5.0 * grid * 256.0 * iters * REP * 8;
            printf("waves/SIMD %d  %-42s %6.2f T lane-ops/s\n", wps, kNames[k], ops / (ms * 1e-3) / 1e12);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
        (void)hipFree(sink);
    }
    return 0;
}
