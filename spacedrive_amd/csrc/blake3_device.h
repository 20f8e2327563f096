// blake3_device.h -- BLAKE3 compression for gfx950, one independent compression per lane.
//
// Replaces the arithmetic of the third-party `blake3` crate 1.4.1 that
// /root/reference/core/src/object/cas.rs:24-61 and
// /root/reference/core/src/object/validation/hash.rs:12-21 call (Cargo.lock:625-628).
//
// Design (MI355X): BLAKE3 is 32-bit add/xor/rotate (ARX) work -- no contraction, so no
// MFMA.  Each lane owns one compression stream with the 16-word state, the 16 message
// words and the 8-word chaining value all in VGPRs; the 7 rounds are fully unrolled so
// the message permutation is pure register renaming.  One G function lowers to
// 2x v_add3_u32 + 2x v_add_u32 + 4x v_xor_b32 + 4x v_alignbit_b32 = 12 VALU ops,
// i.e. 672 VALU lane-ops per compression (+16 for the output fold).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdb3 {

enum : uint32_t { CHUNK_START = 1u, CHUNK_END = 2u, PARENT = 4u, ROOT = 8u };
constexpr uint32_t BLOCK_LEN = 64;
constexpr uint32_t CHUNK_LEN = 1024;

#define SD_IV0 0x6A09E667u
#define SD_IV1 0xBB67AE85u
#define SD_IV2 0x3C6EF372u
#define SD_IV3 0xA54FF53Au
#define SD_IV4 0x510E527Fu
#define SD_IV5 0x9B05688Cu
#define SD_IV6 0x1F83D9ABu
#define SD_IV7 0x5BE0CD19u

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}

// message word schedule: SIGMA(r, i) = PERM applied r times to i
constexpr int PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
constexpr int sigma(int r, int i) { return r == 0 ? i : sigma(r - 1, PERM[i]); }

// rotr(d ^ a, 16) as two VOP2-SDWA xors that write the two 16-bit halves crosswise:
// both are 2-source ops, where xor + v_alignbit pays one 3-source op (half issue rate on
// gfx950).  scripts/valu_probe7.hip at 8 waves/SIMD: 39.51 vs 38.49 T lane-ops/s for the G
// mix (profiles/r3/r3c_valu_probe7.txt; first seen with archive/scripts/valu_probe4.hip,
// profiles/r2/r2z4_valu_probe4.txt).  Not volatile: the compiler
// still schedules it; the early-clobber output keeps d and a readable by the second xor.
#ifndef SD_ROTR16_SDWA
#define SD_ROTR16_SDWA 1
#endif
__device__ __forceinline__ uint32_t xor_rotr16(uint32_t d, uint32_t a) {
#if SD_ROTR16_SDWA
    uint32_t t;
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n\t"
        "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
        : "=&v"(t)
        : "v"(d), "v"(a));
    return t;
#else
    return rotr(d ^ a, 16);
#endif
}

// a + b + m: one v_add3_u32 (3 sources, half issue rate).  Two 2-source adds issue faster
// in registers (scripts/valu_probe7.hip) but measured 8-9 % slower in the kernels (more
// VGPRs, fewer waves; DESIGN.md section 3, profiles/r5/r5b_add3_ab/, variant in 9bfbbfb).
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t m) { return a + b + m; }

// rotr(d ^ a, 8) with v_alignbit (a v_perm_b32 byte permute measured the same, r5x; c6256dd)
__device__ __forceinline__ uint32_t xor_rotr8(uint32_t d, uint32_t a) { return rotr(d ^ a, 8); }

#define SD_G(a, b, c, d, x, y)              \
    a = add3(a, b, (x)); d = xor_rotr16(d, a); \
    c = c + d;           b = rotr(b ^ c, 12); \
    a = add3(a, b, (y)); d = xor_rotr8(d, a); \
    c = c + d;           b = rotr(b ^ c, 7);

template <int R>
__device__ __forceinline__ void round_r(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                        uint32_t& s4, uint32_t& s5, uint32_t& s6, uint32_t& s7,
                                        uint32_t& s8, uint32_t& s9, uint32_t& s10, uint32_t& s11,
                                        uint32_t& s12, uint32_t& s13, uint32_t& s14, uint32_t& s15,
                                        const uint32_t (&m)[16]) {
    SD_G(s0, s4, s8, s12, m[sigma(R, 0)], m[sigma(R, 1)]);
    SD_G(s1, s5, s9, s13, m[sigma(R, 2)], m[sigma(R, 3)]);
    SD_G(s2, s6, s10, s14, m[sigma(R, 4)], m[sigma(R, 5)]);
    SD_G(s3, s7, s11, s15, m[sigma(R, 6)], m[sigma(R, 7)]);
    SD_G(s0, s5, s10, s15, m[sigma(R, 8)], m[sigma(R, 9)]);
    SD_G(s1, s6, s11, s12, m[sigma(R, 10)], m[sigma(R, 11)]);
    SD_G(s2, s7, s8, s13, m[sigma(R, 12)], m[sigma(R, 13)]);
    SD_G(s3, s4, s9, s14, m[sigma(R, 14)], m[sigma(R, 15)]);
}

// cv <- first 8 words of compress(cv, m, counter, block_len, flags)
__device__ __forceinline__ void compress(uint32_t (&cv)[8], const uint32_t (&m)[16],
                                         uint32_t ctr_lo, uint32_t ctr_hi, uint32_t block_len,
                                         uint32_t flags) {
    uint32_t s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3];
    uint32_t s4 = cv[4], s5 = cv[5], s6 = cv[6], s7 = cv[7];
    uint32_t s8 = SD_IV0, s9 = SD_IV1, s10 = SD_IV2, s11 = SD_IV3;
    uint32_t s12 = ctr_lo, s13 = ctr_hi, s14 = block_len, s15 = flags;
#define SD_ROUND(R) round_r<R>(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15, m)
    SD_ROUND(0); SD_ROUND(1); SD_ROUND(2); SD_ROUND(3); SD_ROUND(4); SD_ROUND(5); SD_ROUND(6);
#undef SD_ROUND
    cv[0] = s0 ^ s8;  cv[1] = s1 ^ s9;  cv[2] = s2 ^ s10; cv[3] = s3 ^ s11;
    cv[4] = s4 ^ s12; cv[5] = s5 ^ s13; cv[6] = s6 ^ s14; cv[7] = s7 ^ s15;
}

__device__ __forceinline__ void set_iv(uint32_t (&cv)[8]) {
    cv[0] = SD_IV0; cv[1] = SD_IV1; cv[2] = SD_IV2; cv[3] = SD_IV3;
    cv[4] = SD_IV4; cv[5] = SD_IV5; cv[6] = SD_IV6; cv[7] = SD_IV7;
}

// parent node: out <- compress(IV, left || right, 0, 64, PARENT | extra)
__device__ __forceinline__ void parent(uint32_t (&out)[8], const uint32_t (&l)[8],
                                       const uint32_t (&r)[8], uint32_t extra_flags) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { m[i] = l[i]; m[8 + i] = r[i]; }
    set_iv(out);
    compress(out, m, 0u, 0u, BLOCK_LEN, PARENT | extra_flags);
}

// 64 message bytes -> 16 little-endian words (4x 16-byte loads; ptr 16-B aligned)
// (plain loads: non-temporal ones measured 50 % slower, r5u; de4d437)
__device__ __forceinline__ void load_block(uint32_t (&m)[16], const uint8_t* __restrict__ p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = q[k];
        m[4 * k + 0] = v.x; m[4 * k + 1] = v.y; m[4 * k + 2] = v.z; m[4 * k + 3] = v.w;
    }
}

// Partial final block: len in [0, 64). Bytes past len are zero (BLAKE3 padding).  Reads
// only whole 16-byte pieces that start inside the message -- the stager pads every
// message to a 64-byte multiple, so those reads stay inside the staged buffer.
__device__ __forceinline__ void load_block_partial(uint32_t (&m)[16], const uint8_t* __restrict__ p,
                                                   uint32_t len) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (16u * k < len) v = q[k];
        m[4 * k + 0] = v.x; m[4 * k + 1] = v.y; m[4 * k + 2] = v.z; m[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int w = 0; w < 16; w++) {
        uint32_t lo = 4u * w;
        uint32_t keep = len <= lo ? 0u : (len >= lo + 4 ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (lo + 4 - len))));
        m[w] &= keep;
    }
}

// Chaining value of one chunk of `len` bytes (1..1024; 0 only for an empty message),
// chunk index `counter`.  If is_root, the last block carries ROOT and cv is the hash.
__device__ __forceinline__ void chunk_cv(uint32_t (&cv)[8], const uint8_t* __restrict__ p,
                                         uint32_t len, uint64_t counter, bool is_root) {
    set_iv(cv);
    const uint32_t clo = (uint32_t)counter, chi = (uint32_t)(counter >> 32);
    const uint32_t nblocks = len == 0 ? 1u : (len + 63u) >> 6;
    uint32_t m[16];
    for (uint32_t b = 0; b + 1 < nblocks; b++) {
        load_block(m, p + 64u * b);
        compress(cv, m, clo, chi, BLOCK_LEN, b == 0 ? CHUNK_START : 0u);
    }
    const uint32_t last = nblocks - 1;
    const uint32_t tail = len - 64u * last;
    if (tail == 64u) load_block(m, p + 64u * last);
    else load_block_partial(m, p + 64u * last, tail);
    compress(cv, m, clo, chi, tail, (last == 0 ? CHUNK_START : 0u) | CHUNK_END | (is_root ? ROOT : 0u));
}

// Full 1 KiB non-root chunk with line-pair loads (see full_chunks_cv)
__device__ __forceinline__ void full_chunk_cv_lp(uint32_t (&cv)[8], const uint8_t* __restrict__ p,
                                                 uint64_t counter) {
    set_iv(cv);
    const uint32_t clo = (uint32_t)counter, chi = (uint32_t)(counter >> 32);
    uint32_t ma[16], mb[16];
#pragma unroll 1
    for (uint32_t b = 0; b < 16; b += 2) {
        load_block(ma, p + 64u * b);
        load_block(mb, p + 64u * (b + 1));
        compress(cv, ma, clo, chi, BLOCK_LEN, b == 0 ? CHUNK_START : 0u);
        compress(cv, mb, clo, chi, BLOCK_LEN, b == 14 ? CHUNK_END : 0u);
    }
}

// Merge of U consecutive, full, non-root chunks c0..c0+U-1 (an aligned group, U = 1, 2, 4):
// the chunk CVs merged level-wise in-lane -> `out`.  Line-pair loads: blocks 2k and 2k+1 --
// one 128-byte cache line -- are loaded back to back into two register buffers, then both
// compressed, so a line is consumed whole instead of across a compression (with ~7 MB of
// lines in flight per XCD against a 4 MB L2, half-consumed lines were evicted and fetched
// again: 1.10x the algorithmic HBM bytes before, 1.00x after).
template <int U>
__device__ __forceinline__ void full_chunks_cv(uint32_t (&out)[8], const uint8_t* __restrict__ p, uint64_t c0) {
    static_assert(U == 1 || U == 2 || U == 4, "U");
    uint32_t held[2][8];  // level-wise merge stack: at most two pending nodes for U <= 4
    uint32_t ma[16], mb[16];
#pragma unroll
    for (int u = 0; u < U; u++) {
        uint32_t cv[8];
        set_iv(cv);
        const uint64_t ctr = c0 + u;
        const uint32_t clo = (uint32_t)ctr, chi = (uint32_t)(ctr >> 32);
        const uint8_t* q = p + (size_t)u * CHUNK_LEN;
#pragma unroll 1
        for (uint32_t b = 0; b < 16; b += 2) {
            load_block(ma, q + 64u * b);
            load_block(mb, q + 64u * (b + 1));
            compress(cv, ma, clo, chi, BLOCK_LEN, b == 0 ? CHUNK_START : 0u);
            compress(cv, mb, clo, chi, BLOCK_LEN, b + 1 == 15 ? CHUNK_END : 0u);
        }
        if (U == 1) {
#pragma unroll
            for (int i = 0; i < 8; i++) out[i] = cv[i];
        } else if (u == 0 || u == 2) {
#pragma unroll
            for (int i = 0; i < 8; i++) held[u >> 1][i] = cv[i];
        } else if (u == 1) {
            parent(out, held[0], cv, 0u);
            if (U == 4) {
#pragma unroll
                for (int i = 0; i < 8; i++) held[0][i] = out[i];
            }
        } else {  // u == 3
            uint32_t p23[8];
            parent(p23, held[1], cv, 0u);
            parent(out, held[0], p23, 0u);
        }
    }
}

}  // namespace sdb3
