// VALU issue-rate probe for the integer ops BLAKE3 uses on gfx950: each kernel runs
// 8 independent chains per lane of one instruction kind (inline asm, so the compiler
// cannot fold or re-select them), 8 waves per SIMD.  Prints lane-ops/s per kind.
// Build: hipcc --offload-arch=gfx950 -O3 -o oracle/_probe/valu_probe scripts/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
#define REP 16

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(uint32_t* sink, uint32_t iters) {
    uint32_t x[CHAINS];
    const uint32_t y = threadIdx.x * 0x9E3779B9u + blockIdx.x, z = y ^ 0x5bd1e995u;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) x[i] = y + i * 0x1234567u;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#pragma unroll
            for (int i = 0; i < CHAINS; i++) {
                if (KIND == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (KIND == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (KIND == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x[i]));
                if (KIND == 3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));
                if (KIND == 4) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(y), "v"(z));
                if (KIND == 5) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (KIND == 6) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (KIND == 7) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x[i]) : "v"(y));
                if (KIND == 8) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[i]) : "v"(y), "v"(z));
                if (KIND == 9) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x[i]) : "v"(y));
                if (KIND == 10) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) r ^= x[i];
    if (r == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// 64-bit packed f32 add (two lanes' worth per lane-op) on register pairs
__global__ __launch_bounds__(256) void k_probe_pk(uint32_t* sink, uint32_t iters) {
    float2 x[CHAINS];
    const float2 y = make_float2(threadIdx.x * 1e-9f, blockIdx.x * 1e-9f);
#pragma unroll
    for (int i = 0; i < CHAINS; i++) x[i] = make_float2(i, i + 1);
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
#pragma unroll
            for (int i = 0; i < CHAINS; i++) {
                double d;
                __builtin_memcpy(&d, &x[i], 8);
                double e;
                __builtin_memcpy(&e, &y, 8);
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d) : "v"(e));
                __builtin_memcpy(&x[i], &d, 8);
            }
        }
    }
    float r = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) r += x[i].x + x[i].y;
    if (r == 1234.5f) sink[blockIdx.x * blockDim.x + threadIdx.x] = 1;
}

template <typename F>
static double run(F launch, int grid, uint32_t iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipEventRecord(a);
    for (int r = 0; r < 3; r++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double ops = 3.0 * grid * 256.0 * iters * REP * CHAINS;
    return ops / (ms * 1e-3) / 1e12;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const char* names[] = {"v_xor_b32(vop2)", "v_add_u32(vop2)", "v_alignbit_b32", "v_add3_u32", "v_xad_u32",
                           "v_pk_add_u16", "v_perm_b32", "v_xor_b32_e64", "v_bitop3_b32", "v_lshl_add_u32",
                           "v_add_f32"};
    uint32_t* sink;
    for (int wps : {4, 8}) {
        const int grid = p.multiProcessorCount * wps;  // 256-thread workgroups: wps waves per SIMD
        hipMalloc(&sink, (size_t)grid * 256 * 4);
        const uint32_t iters = 256;
        double t[11];
        t[0] = run([&] { hipLaunchKernelGGL(k_probe<0>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[1] = run([&] { hipLaunchKernelGGL(k_probe<1>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[2] = run([&] { hipLaunchKernelGGL(k_probe<2>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[3] = run([&] { hipLaunchKernelGGL(k_probe<3>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[4] = run([&] { hipLaunchKernelGGL(k_probe<4>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[5] = run([&] { hipLaunchKernelGGL(k_probe<5>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[6] = run([&] { hipLaunchKernelGGL(k_probe<6>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[7] = run([&] { hipLaunchKernelGGL(k_probe<7>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[8] = run([&] { hipLaunchKernelGGL(k_probe<8>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[9] = run([&] { hipLaunchKernelGGL(k_probe<9>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        t[10] = run([&] { hipLaunchKernelGGL(k_probe<10>, dim3(grid), dim3(256), 0, 0, sink, iters); }, grid, iters);
        for (int k = 0; k < 11; k++) printf("waves/SIMD %d  %-18s %6.2f T lane-ops/s\n", wps, names[k], t[k]);
        const double pk = run([&] { hipLaunchKernelGGL(k_probe_pk, dim3(grid), dim3(256), 0, 0, sink, iters); },
                              grid, iters);
        printf("waves/SIMD %d  %-18s %6.2f T instr-lanes/s (x2 f32 each)\n", wps, "v_pk_add_f32", pk);
        hipFree(sink);
    }
    return 0;
}
