// f64_b3_probe.hip -- BLAKE3 compression with its 32-bit adds done as f64 adds of
// denormal register pairs (scripts/gen_valu_probe8.py explains the trick), checked
// bit-exact against the library's integer compression (blake3_device.h) on random
// inputs, then timed from registers beside it.
//
// A 64-bit pattern p < 2^53 read as a double is p * 2^-1074 (denormal below 2^52, and
// the normal doubles of exponent field 1 continue the same integer grid up to 2^53), so
// v_add_f64 of two such patterns is exact integer addition: the low word is the 32-bit
// modular sum, the carry goes to the high word.  State words a (row 0) and c (row 2) are
// the only add destinations, so their high words collect carries (a few dozen per
// compression) and b, d and the message keep zero high words.
//
// Variants: V=0 the library's integer compress; V=1 a+=b and c+=d as f64 adds, the
// message add on the integer side; V=2 every add as f64 (message words in zero-high pairs).
// Build: hipcc --offload-arch=gfx950 -O3 -I spacedrive_amd/csrc -o scripts/f64_b3_probe scripts/f64_b3_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "blake3_device.h"

namespace {

__device__ __forceinline__ uint64_t fadd(uint64_t x, uint64_t y) {
    return __builtin_bit_cast(uint64_t, __builtin_bit_cast(double, x) + __builtin_bit_cast(double, y));
}
__device__ __forceinline__ uint32_t lo(uint64_t x) { return (uint32_t)x; }
__device__ __forceinline__ uint64_t setlo(uint64_t x, uint32_t v) { return (x & 0xFFFFFFFF00000000ull) | v; }

template <int V>
struct F {
    // G on pairs; x, y: message pairs (V=2) or words in the low half (V=1)
    static __device__ __forceinline__ void g(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t x,
                                             uint64_t y) {
        if (V == 2) a = fadd(fadd(a, x), b);
        else a = fadd(setlo(a, lo(a) + lo(x)), b);
        d = setlo(d, sdb3::xor_rotr16(lo(d), lo(a)));
        c = fadd(c, d);
        b = setlo(b, sdb3::rotr(lo(b) ^ lo(c), 12));
        if (V == 2) a = fadd(fadd(a, y), b);
        else a = fadd(setlo(a, lo(a) + lo(y)), b);
        d = setlo(d, sdb3::rotr(lo(d) ^ lo(a), 8));
        c = fadd(c, d);
        b = setlo(b, sdb3::rotr(lo(b) ^ lo(c), 7));
    }
    template <int R>
    static __device__ __forceinline__ void round(uint64_t (&s)[16], const uint64_t (&m)[16]) {
        using sdb3::sigma;
        g(s[0], s[4], s[8], s[12], m[sigma(R, 0)], m[sigma(R, 1)]);
        g(s[1], s[5], s[9], s[13], m[sigma(R, 2)], m[sigma(R, 3)]);
        g(s[2], s[6], s[10], s[14], m[sigma(R, 4)], m[sigma(R, 5)]);
        g(s[3], s[7], s[11], s[15], m[sigma(R, 6)], m[sigma(R, 7)]);
        g(s[0], s[5], s[10], s[15], m[sigma(R, 8)], m[sigma(R, 9)]);
        g(s[1], s[6], s[11], s[12], m[sigma(R, 10)], m[sigma(R, 11)]);
        g(s[2], s[7], s[8], s[13], m[sigma(R, 12)], m[sigma(R, 13)]);
        g(s[3], s[4], s[9], s[14], m[sigma(R, 14)], m[sigma(R, 15)]);
    }
    static __device__ __forceinline__ void compress(uint32_t (&cv)[8], const uint32_t (&mw)[16], uint32_t ctr_lo,
                                                    uint32_t ctr_hi, uint32_t block_len, uint32_t flags) {
        uint64_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = mw[i];
        uint64_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4],  cv[5],  cv[6],     cv[7],
                          SD_IV0, SD_IV1, SD_IV2, SD_IV3, ctr_lo, ctr_hi, block_len, flags};
        round<0>(s, m); round<1>(s, m); round<2>(s, m); round<3>(s, m);
        round<4>(s, m); round<5>(s, m); round<6>(s, m);
#pragma unroll
        for (int i = 0; i < 8; i++) cv[i] = lo(s[i]) ^ lo(s[i + 8]);
    }
};

template <int V>
__device__ __forceinline__ void compress_v(uint32_t (&cv)[8], const uint32_t (&m)[16], uint32_t cl, uint32_t ch,
                                           uint32_t bl, uint32_t fl) {
    if (V == 0) sdb3::compress(cv, m, cl, ch, bl, fl);
    else F<V>::compress(cv, m, cl, ch, bl, fl);
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

// chain of `reps` compressions per lane from pseudo-random inputs; out = final CV
template <int V>
__global__ __launch_bounds__(256) void k_chain(uint32_t* out, uint32_t reps, uint64_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cv[8], m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) cv[i] = mix32(seed ^ (t * 64 + i));
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = mix32(~seed ^ (t * 64 + 16 + i));
    for (uint32_t r = 0; r < reps; r++) {
        compress_v<V>(cv, m, r, (uint32_t)t, 64u, (r & 3u) | 1u);
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] ^= cv[i & 7];  // next message depends on this CV
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[t * 8 + i] = cv[i];
}

}  // namespace

template <int V>
static float run(uint32_t* d, int grid, uint32_t reps, uint64_t seed, int launches) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_chain<V>, dim3(grid), dim3(256), 0, 0, d, reps, seed);
    (void)hipEventRecord(e0);
    for (int i = 0; i < launches; i++) hipLaunchKernelGGL(k_chain<V>, dim3(grid), dim3(256), 0, 0, d, reps, seed);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / launches;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    hipFuncAttributes fa[3];
    (void)hipFuncGetAttributes(&fa[0], (const void*)k_chain<0>);
    (void)hipFuncGetAttributes(&fa[1], (const void*)k_chain<1>);
    (void)hipFuncGetAttributes(&fa[2], (const void*)k_chain<2>);
    printf("# %s, %d CUs; VGPRs: V0 %d, V1 %d, V2 %d\n", p.gcnArchName, cus, fa[0].numRegs, fa[1].numRegs,
           fa[2].numRegs);
    // exactness: 1 M lanes x 64 chained compressions, every word compared
    const int grid_chk = 4096;
    const size_t words = (size_t)grid_chk * 256 * 8;
    uint32_t *d0, *d1;
    (void)hipMalloc(&d0, words * 4);
    (void)hipMalloc(&d1, words * 4);
    std::vector<uint32_t> h0(words), h1(words);
    int bad_total = 0;
    for (uint64_t seed : {0x5D5DCA51Dull, 0x123456789ull, 0xFFFFFFFFFFFFull}) {
        hipLaunchKernelGGL(k_chain<0>, dim3(grid_chk), dim3(256), 0, 0, d0, 64u, seed);
        for (int v = 1; v <= 2; v++) {
            if (v == 1) hipLaunchKernelGGL(k_chain<1>, dim3(grid_chk), dim3(256), 0, 0, d1, 64u, seed);
            else hipLaunchKernelGGL(k_chain<2>, dim3(grid_chk), dim3(256), 0, 0, d1, 64u, seed);
            (void)hipMemcpy(h0.data(), d0, words * 4, hipMemcpyDeviceToHost);
            (void)hipMemcpy(h1.data(), d1, words * 4, hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (size_t i = 0; i < words; i++) bad += h0[i] != h1[i];
            printf("exactness V%d seed %llx: %zu of %zu words differ (%d M compressions)\n", v,
                   (unsigned long long)seed, bad, words, grid_chk * 256 * 64 / 1000000);
            bad_total += bad != 0;
        }
    }
    // speed: grid of cus * wps workgroups, 2048 chained compressions per lane
    for (int wps : {4, 8}) {
        const int grid = cus * wps;
        for (int v = 0; v <= 2; v++) {
            const uint32_t reps = 2048;
            float ms = v == 0 ? run<0>(d0, grid, reps, 1, 5) : v == 1 ? run<1>(d0, grid, reps, 1, 5)
                                                                      : run<2>(d0, grid, reps, 1, 5);
            const double comps = (double)grid * 256 * reps;
            printf("wps %d V%d: %.3f ms, %.2f G compressions/s, %.2f T lane-ops/s (672 per compression)\n", wps, v,
                   ms, comps / (ms * 1e-3) / 1e9, comps * 672 / (ms * 1e-3) / 1e12);
        }
    }
    return bad_total ? 1 : 0;
}
