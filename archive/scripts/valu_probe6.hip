// VALU issue probe, part 6: the controls VERDICT r2 asked for.  Is the half rate of
// gfx950's 3-source integer ops specific to them, or does the harness cap every op near
// 38 T?  Same harness as valu_probe5 (8 independent ops of one kind per asm block on
// hard-named VGPRs, 16 blocks per iteration, 256-thread workgroups, every CU holding
// `wps` waves per SIMD), plus two clock-independent readings per kind:
//   * each workgroup's own duration in shader cycles (s_memtime, MI355X_MICROARCH.md
//     "tick = shader cycle"), so  cycles per wave-instruction per SIMD
//       = cycles / (wps x instructions per wave)            (2 = full rate on SIMD-32)
//   * the same span in s_memrealtime ticks (100 MHz), giving the clock the waves ran at.
// Build: hipcc --offload-arch=gfx950 -O3 -w -o scripts/valu_probe6 scripts/valu_probe6.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define REP 16
#define X8(op, a, b, c) \
    op " v32, v" a "0, v" b "0" c "\n" op " v33, v" a "1, v" b "1" c "\n" op " v34, v" a "2, v" b "2" c "\n" \
    op " v35, v" a "3, v" b "3" c "\n" op " v36, v" a "4, v" b "4" c "\n" op " v37, v" a "5, v" b "5" c "\n" \
    op " v38, v" a "6, v" b "6" c "\n" op " v39, v" a "7, v" b "7" c "\n"
// 2-source VOP2 forms: dst = src0 op src1 (sources v40..v47 and v50..v57)
#define BODY0 X8("v_xor_b32", "4", "5", "")
#define BODY1 X8("v_add_u32", "4", "5", "")
#define BODY2 X8("v_add_f32", "4", "5", "")
#define BODY3 X8("v_mul_f32", "4", "5", "")
#define BODY4 X8("v_mul_u32_u24", "4", "5", "")
// VOP2 with a third operand read implicitly: the accumulator (fmac) or VCC (addc)
#define BODY5 X8("v_fmac_f32", "4", "5", "")
#define ADDC(d, a, b) "v_addc_co_u32 v" d ", vcc, v" a ", v" b ", vcc\n"
#define BODY6 ADDC("32", "40", "50") ADDC("33", "41", "51") ADDC("34", "42", "52") ADDC("35", "43", "53") \
    ADDC("36", "44", "54") ADDC("37", "45", "55") ADDC("38", "46", "56") ADDC("39", "47", "57")
// 3-source VOP3 forms: dst = f(src0, src1, src2) with src2 from v60..v67
#define BODY7 X8("v_fma_f32", "4", "5", ", v6" "0")
#define BODY8 X8("v_mad_u32_u24", "4", "5", ", v6" "0")
#define BODY9 X8("v_xad_u32", "4", "5", ", v6" "0")
#define BODY10 X8("v_add3_u32", "4", "5", ", v6" "0")
#define BODY11 X8("v_alignbit_b32", "4", "5", ", 7")
#define BODY12 X8("v_bitop3_b32", "4", "5", ", v60 bitop3:0x96")
// packed f32 (VOP3P): one instruction = two f32 FMAs per lane
#define PK4(op, c2)                                                                                  \
    op " v[32:33], v[40:41], v[50:51]" c2 "[60:61]\n" op " v[34:35], v[42:43], v[52:53]" c2 "[62:63]\n"     \
    op " v[36:37], v[44:45], v[54:55]" c2 "[64:65]\n" op " v[38:39], v[46:47], v[56:57]" c2 "[66:67]\n"
#define BODY13 PK4("v_pk_fma_f32", ", v") PK4("v_pk_fma_f32", ", v")
#define BODY14 PK4("v_pk_add_f32", " ;") PK4("v_pk_add_f32", " ;")
#define NKINDS 15
static const char* kNames[NKINDS] = {"v_xor_b32        VOP2 2-src int", "v_add_u32        VOP2 2-src int",
                                     "v_add_f32        VOP2 2-src f32", "v_mul_f32        VOP2 2-src f32",
                                     "v_mul_u32_u24    VOP2 2-src int", "v_fmac_f32       VOP2 +acc f32",
                                     "v_addc_co_u32    VOP2 +vcc int",  "v_fma_f32        VOP3 3-src f32",
                                     "v_mad_u32_u24    VOP3 3-src int", "v_xad_u32        VOP3 3-src int",
                                     "v_add3_u32       VOP3 3-src int", "v_alignbit_b32   VOP3 3-src int",
                                     "v_bitop3_b32     VOP3 3-src int", "v_pk_fma_f32     VOP3P 2xf32",
                                     "v_pk_add_f32     VOP3P 2xf32"};

#define CLOB                                                                                                \
    "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", \
        "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60",     \
        "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "vcc"

template <int KIND>
__global__ __launch_bounds__(256) void k_op(uint64_t* cyc, uint32_t iters) {
    asm volatile(
        "v_mov_b32 v40, 1\nv_mov_b32 v41, 2\nv_mov_b32 v42, 3\nv_mov_b32 v43, 4\nv_mov_b32 v44, 5\n"
        "v_mov_b32 v45, 6\nv_mov_b32 v46, 7\nv_mov_b32 v47, 8\nv_mov_b32 v48, 9\nv_mov_b32 v49, 10\n"
        "v_mov_b32 v50, 11\nv_mov_b32 v51, 12\nv_mov_b32 v52, 13\nv_mov_b32 v53, 14\nv_mov_b32 v54, 15\n"
        "v_mov_b32 v55, 16\nv_mov_b32 v56, 17\nv_mov_b32 v57, 18\nv_mov_b32 v58, 19\nv_mov_b32 v59, 20\n"
        "v_mov_b32 v60, 21\nv_mov_b32 v61, 22\nv_mov_b32 v62, 23\nv_mov_b32 v63, 24\nv_mov_b32 v64, 25\n"
        "v_mov_b32 v65, 26\nv_mov_b32 v66, 27\nv_mov_b32 v67, 28\nv_mov_b32 v68, 29\n"
        "v_mov_b32 v32, 0\nv_mov_b32 v33, 0\nv_mov_b32 v34, 0\nv_mov_b32 v35, 0\nv_mov_b32 v36, 0\n"
        "v_mov_b32 v37, 0\nv_mov_b32 v38, 0\nv_mov_b32 v39, 0\ns_mov_b64 vcc, 0" ::: CLOB);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#define B(K) \
    if (KIND == K) asm volatile(BODY##K ::: CLOB);
            B(0) B(1) B(2) B(3) B(4) B(5) B(6) B(7) B(8) B(9) B(10) B(11) B(12) B(13) B(14)
#undef B
        }
    }
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t v;
    asm volatile("v_mov_b32 %0, v32" : "=v"(v));
    if (threadIdx.x == 0) {  // per-lane (vector) stores of the block's span
        cyc[2 * blockIdx.x] = t1 - t0;
        cyc[2 * blockIdx.x + 1] = (r1 - r0) + (v == 0x12345678u ? 1 : 0);
    }
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    void (*fns[NKINDS])(uint64_t*, uint32_t) = {k_op<0>, k_op<1>, k_op<2>,  k_op<3>,  k_op<4>,
                                                k_op<5>, k_op<6>, k_op<7>,  k_op<8>,  k_op<9>,
                                                k_op<10>, k_op<11>, k_op<12>, k_op<13>, k_op<14>};
    const int cus = p.multiProcessorCount;
    printf("# %s, %d CUs; 8 independent ops x %d per iteration; lane-op = one instruction on one lane\n", p.gcnArchName,
           cus, REP);
    printf("# %-3s %-34s %9s %11s %13s %9s\n", "wps", "kind", "T lane/s", "lane/clk/CU", "cyc/instr/SIMD", "MHz");
    for (int wps : {1, 2, 4, 8}) {
        const int grid = cus * wps;  // 256-thread workgroups: one wave per SIMD each
        uint64_t* cyc;
        (void)hipMalloc(&cyc, (size_t)grid * 16);
        const uint32_t iters = 256;
        for (int k = 0; k < NKINDS; k++) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            for (int w = 0; w < 20; w++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, cyc, iters);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, cyc, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            std::vector<uint64_t> h((size_t)grid * 2);
            (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
            std::vector<double> c(grid), mhz(grid);
            for (int b = 0; b < grid; b++) {
                c[b] = (double)h[2 * b];
                mhz[b] = (double)h[2 * b] / ((double)h[2 * b + 1] / 100.0);  // memrealtime = 100 MHz
            }
            std::sort(c.begin(), c.end());
            std::sort(mhz.begin(), mhz.end());
            const double cmed = c[grid / 2];
            const double per_wave = (double)iters * REP * 8;  // instructions per wave
            const double ops = 5.0 * grid * 256.0 * per_wave;
            printf("  %-3d %-34s %9.2f %11.1f %13.2f %9.0f\n", wps, kNames[k], ops / (ms * 1e-3) / 1e12,
                   per_wave * 64.0 * 4 * wps / cmed, cmed / (wps * per_wave), mhz[grid / 2]);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
        (void)hipFree(cyc);
    }
    return 0;
}
