/*
 * sd_oracle_simd.c -- SIMD multi-chunk BLAKE3 for the CPU baseline.  TEST INFRASTRUCTURE
 * ONLY (see sd_oracle.c for the rules: checker and timed CPU baseline, never shipped).
 *
 * The reference's hashing runs in the `blake3` crate 1.4.1 (Cargo.lock:625-628), whose
 * Hasher::update hashes whole chunks of a multi-chunk update many-at-a-time with SIMD
 * (`hash_many`: 16 chunks per AVX-512 pass, 8 per AVX2 pass; C/asm behind `cc`,
 * Cargo.lock:629-636), then merges parents the same way.  Timing a scalar restatement
 * against the GPU would understate the reference CPU path several-fold, so this file
 * restates that published strategy: message words transposed so each vector lane holds
 * one chunk, 7 rounds on 16 (or 8) lanes, chaining values transposed back.  It is
 * checked against the scalar oracle and the Python spec in tests/test_oracle.py.
 *
 * One-shot hashing of a complete message: full chunks 0..C-2 via hash_many, the last
 * chunk scalar, then level-wise parents via hash_many on CV pairs (level-wise merge is
 * the BLAKE3 tree; tests/test_oracle.py::test_tree_shapes_equal).
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { FS_CHUNK_START = 1, FS_CHUNK_END = 2, FS_PARENT = 4, FS_ROOT = 8 };
static const uint32_t IV_[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t SIG[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1}, {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4}, {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};

/* scalar compression from sd_oracle.c (same translation unit family, exported there) */
void sdo_compress_words(const uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len,
                        uint32_t flags, uint32_t out16[16]);

/* ------------------------------------------------------------------ AVX-512: 16 lanes */
#define A5 __attribute__((target("avx512f")))

A5 static inline __m512i a5_add(__m512i a, __m512i b) { return _mm512_add_epi32(a, b); }
A5 static inline __m512i a5_xor(__m512i a, __m512i b) { return _mm512_xor_si512(a, b); }

#define G5(a, b, c, d, x, y)                                                    \
    a = a5_add(a5_add(a, b), x); d = _mm512_ror_epi32(a5_xor(d, a), 16);       \
    c = a5_add(c, d);            b = _mm512_ror_epi32(a5_xor(b, c), 12);       \
    a = a5_add(a5_add(a, b), y); d = _mm512_ror_epi32(a5_xor(d, a), 8);        \
    c = a5_add(c, d);            b = _mm512_ror_epi32(a5_xor(b, c), 7);

A5 static void a5_transpose(__m512i r[16]) {
    __m512i t[16];
    for (int i = 0; i < 16; i += 2) {
        t[i] = _mm512_unpacklo_epi32(r[i], r[i + 1]);
        t[i + 1] = _mm512_unpackhi_epi32(r[i], r[i + 1]);
    }
    for (int i = 0; i < 16; i += 4) {
        r[i] = _mm512_unpacklo_epi64(t[i], t[i + 2]);
        r[i + 1] = _mm512_unpackhi_epi64(t[i], t[i + 2]);
        r[i + 2] = _mm512_unpacklo_epi64(t[i + 1], t[i + 3]);
        r[i + 3] = _mm512_unpackhi_epi64(t[i + 1], t[i + 3]);
    }
    for (int i = 0; i < 4; i++) {
        t[i] = _mm512_shuffle_i32x4(r[i], r[i + 4], 0x88);
        t[i + 4] = _mm512_shuffle_i32x4(r[i], r[i + 4], 0xDD);
        t[i + 8] = _mm512_shuffle_i32x4(r[i + 8], r[i + 12], 0x88);
        t[i + 12] = _mm512_shuffle_i32x4(r[i + 8], r[i + 12], 0xDD);
    }
    for (int i = 0; i < 4; i++) {
        r[i] = _mm512_shuffle_i32x4(t[i], t[i + 8], 0x88);
        r[i + 8] = _mm512_shuffle_i32x4(t[i], t[i + 8], 0xDD);
        r[i + 4] = _mm512_shuffle_i32x4(t[i + 4], t[i + 12], 0x88);
        r[i + 12] = _mm512_shuffle_i32x4(t[i + 4], t[i + 12], 0xDD);
    }
}

static int a5_col[16];  /* a5_transpose output vector j holds column a5_col[j] */
static int a5_ready;

A5 static void a5_init(void) {
    __m512i r[16];
    uint32_t buf[16];
    for (int i = 0; i < 16; i++) {
        for (int j = 0; j < 16; j++) buf[j] = (uint32_t)(i * 16 + j);
        r[i] = _mm512_loadu_si512(buf);
    }
    a5_transpose(r);
    for (int j = 0; j < 16; j++) {
        _mm512_storeu_si512(buf, r[j]);
        a5_col[j] = (int)(buf[0] % 16); /* element 0 comes from row 0: value = column */
        for (int k = 0; k < 16; k++)
            if (buf[k] != (uint32_t)(k * 16 + a5_col[j])) abort(); /* not a transpose */
    }
    a5_ready = 1;
}

/* CVs of n (<= 16) inputs of `blocks` 64-byte blocks each; counters ctr0 + i if inc */
A5 static void a5_hash_many(const uint8_t* const* in, int n, int blocks, uint64_t ctr0, int inc, uint32_t flags,
                            uint32_t fstart, uint32_t fend, uint8_t* out /* n x 32 */) {
    uint32_t lo[16], hi[16];
    for (int i = 0; i < 16; i++) {
        uint64_t c = ctr0 + (inc ? (uint64_t)i : 0);
        lo[i] = (uint32_t)c;
        hi[i] = (uint32_t)(c >> 32);
    }
    const __m512i clo = _mm512_loadu_si512(lo), chi = _mm512_loadu_si512(hi);
    __m512i h[8];
    for (int i = 0; i < 8; i++) h[i] = _mm512_set1_epi32((int)IV_[i]);
    for (int b = 0; b < blocks; b++) {
        __m512i r[16], m[16];
        for (int i = 0; i < 16; i++) r[i] = _mm512_loadu_si512(in[i < n ? i : 0] + 64 * b);
        a5_transpose(r);
        for (int j = 0; j < 16; j++) m[a5_col[j]] = r[j];
        uint32_t fl = flags | (b == 0 ? fstart : 0) | (b == blocks - 1 ? fend : 0);
        __m512i v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
        __m512i v8 = _mm512_set1_epi32((int)IV_[0]), v9 = _mm512_set1_epi32((int)IV_[1]);
        __m512i v10 = _mm512_set1_epi32((int)IV_[2]), v11 = _mm512_set1_epi32((int)IV_[3]);
        __m512i v12 = clo, v13 = chi, v14 = _mm512_set1_epi32(64), v15 = _mm512_set1_epi32((int)fl);
        for (int r_ = 0; r_ < 7; r_++) {
            const uint8_t* s = SIG[r_];
            G5(v0, v4, v8, v12, m[s[0]], m[s[1]]);
            G5(v1, v5, v9, v13, m[s[2]], m[s[3]]);
            G5(v2, v6, v10, v14, m[s[4]], m[s[5]]);
            G5(v3, v7, v11, v15, m[s[6]], m[s[7]]);
            G5(v0, v5, v10, v15, m[s[8]], m[s[9]]);
            G5(v1, v6, v11, v12, m[s[10]], m[s[11]]);
            G5(v2, v7, v8, v13, m[s[12]], m[s[13]]);
            G5(v3, v4, v9, v14, m[s[14]], m[s[15]]);
        }
        h[0] = a5_xor(v0, v8); h[1] = a5_xor(v1, v9); h[2] = a5_xor(v2, v10); h[3] = a5_xor(v3, v11);
        h[4] = a5_xor(v4, v12); h[5] = a5_xor(v5, v13); h[6] = a5_xor(v6, v14); h[7] = a5_xor(v7, v15);
    }
    uint32_t w[8][16];
    for (int i = 0; i < 8; i++) _mm512_storeu_si512(w[i], h[i]);
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 8; k++) memcpy(out + 32 * i + 4 * k, &w[k][i], 4);
}

/* ------------------------------------------------------------------ AVX2: 8 lanes */
#define A2 __attribute__((target("avx2")))

A2 static inline __m256i a2_rot16(__m256i x) {
    const __m256i k = _mm256_setr_epi8(2, 3, 0, 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13, 2, 3, 0, 1, 6, 7, 4, 5,
                                       10, 11, 8, 9, 14, 15, 12, 13);
    return _mm256_shuffle_epi8(x, k);
}
A2 static inline __m256i a2_rot8(__m256i x) {
    const __m256i k = _mm256_setr_epi8(1, 2, 3, 0, 5, 6, 7, 4, 9, 10, 11, 8, 13, 14, 15, 12, 1, 2, 3, 0, 5, 6, 7, 4,
                                       9, 10, 11, 8, 13, 14, 15, 12);
    return _mm256_shuffle_epi8(x, k);
}
#define A2ROT(x, n) _mm256_or_si256(_mm256_srli_epi32(x, n), _mm256_slli_epi32(x, 32 - (n)))
#define G2(a, b, c, d, x, y)                                                                        \
    a = _mm256_add_epi32(_mm256_add_epi32(a, b), x); d = a2_rot16(_mm256_xor_si256(d, a));          \
    c = _mm256_add_epi32(c, d);                      b = A2ROT(_mm256_xor_si256(b, c), 12);         \
    a = _mm256_add_epi32(_mm256_add_epi32(a, b), y); d = a2_rot8(_mm256_xor_si256(d, a));           \
    c = _mm256_add_epi32(c, d);                      b = A2ROT(_mm256_xor_si256(b, c), 7);

A2 static void a2_transpose(__m256i r[8]) {
    __m256i t[8];
    for (int i = 0; i < 8; i += 2) {
        t[i] = _mm256_unpacklo_epi32(r[i], r[i + 1]);
        t[i + 1] = _mm256_unpackhi_epi32(r[i], r[i + 1]);
    }
    for (int i = 0; i < 8; i += 4) {
        r[i] = _mm256_unpacklo_epi64(t[i], t[i + 2]);
        r[i + 1] = _mm256_unpackhi_epi64(t[i], t[i + 2]);
        r[i + 2] = _mm256_unpacklo_epi64(t[i + 1], t[i + 3]);
        r[i + 3] = _mm256_unpackhi_epi64(t[i + 1], t[i + 3]);
    }
    for (int i = 0; i < 4; i++) {
        t[i] = _mm256_permute2x128_si256(r[i], r[i + 4], 0x20);
        t[i + 4] = _mm256_permute2x128_si256(r[i], r[i + 4], 0x31);
    }
    for (int i = 0; i < 8; i++) r[i] = t[i];
}

static int a2_col[8];
static int a2_ready;

A2 static void a2_init(void) {
    __m256i r[8];
    uint32_t buf[8];
    for (int i = 0; i < 8; i++) {
        for (int j = 0; j < 8; j++) buf[j] = (uint32_t)(i * 8 + j);
        r[i] = _mm256_loadu_si256((const __m256i*)buf);
    }
    a2_transpose(r);
    for (int j = 0; j < 8; j++) {
        _mm256_storeu_si256((__m256i*)buf, r[j]);
        a2_col[j] = (int)(buf[0] % 8);
        for (int k = 0; k < 8; k++)
            if (buf[k] != (uint32_t)(k * 8 + a2_col[j])) abort();
    }
    a2_ready = 1;
}

A2 static void a2_hash_many(const uint8_t* const* in, int n, int blocks, uint64_t ctr0, int inc, uint32_t flags,
                            uint32_t fstart, uint32_t fend, uint8_t* out) {
    uint32_t lo[8], hi[8];
    for (int i = 0; i < 8; i++) {
        uint64_t c = ctr0 + (inc ? (uint64_t)i : 0);
        lo[i] = (uint32_t)c;
        hi[i] = (uint32_t)(c >> 32);
    }
    const __m256i clo = _mm256_loadu_si256((const __m256i*)lo), chi = _mm256_loadu_si256((const __m256i*)hi);
    __m256i h[8];
    for (int i = 0; i < 8; i++) h[i] = _mm256_set1_epi32((int)IV_[i]);
    for (int b = 0; b < blocks; b++) {
        __m256i ra[8], rb[8], m[16];
        for (int i = 0; i < 8; i++) {
            const uint8_t* p = in[i < n ? i : 0] + 64 * b;
            ra[i] = _mm256_loadu_si256((const __m256i*)p);
            rb[i] = _mm256_loadu_si256((const __m256i*)(p + 32));
        }
        a2_transpose(ra);
        a2_transpose(rb);
        for (int j = 0; j < 8; j++) {
            m[a2_col[j]] = ra[j];
            m[8 + a2_col[j]] = rb[j];
        }
        uint32_t fl = flags | (b == 0 ? fstart : 0) | (b == blocks - 1 ? fend : 0);
        __m256i v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
        __m256i v8 = _mm256_set1_epi32((int)IV_[0]), v9 = _mm256_set1_epi32((int)IV_[1]);
        __m256i v10 = _mm256_set1_epi32((int)IV_[2]), v11 = _mm256_set1_epi32((int)IV_[3]);
        __m256i v12 = clo, v13 = chi, v14 = _mm256_set1_epi32(64), v15 = _mm256_set1_epi32((int)fl);
        for (int r_ = 0; r_ < 7; r_++) {
            const uint8_t* s = SIG[r_];
            G2(v0, v4, v8, v12, m[s[0]], m[s[1]]);
            G2(v1, v5, v9, v13, m[s[2]], m[s[3]]);
            G2(v2, v6, v10, v14, m[s[4]], m[s[5]]);
            G2(v3, v7, v11, v15, m[s[6]], m[s[7]]);
            G2(v0, v5, v10, v15, m[s[8]], m[s[9]]);
            G2(v1, v6, v11, v12, m[s[10]], m[s[11]]);
            G2(v2, v7, v8, v13, m[s[12]], m[s[13]]);
            G2(v3, v4, v9, v14, m[s[14]], m[s[15]]);
        }
        h[0] = _mm256_xor_si256(v0, v8); h[1] = _mm256_xor_si256(v1, v9);
        h[2] = _mm256_xor_si256(v2, v10); h[3] = _mm256_xor_si256(v3, v11);
        h[4] = _mm256_xor_si256(v4, v12); h[5] = _mm256_xor_si256(v5, v13);
        h[6] = _mm256_xor_si256(v6, v14); h[7] = _mm256_xor_si256(v7, v15);
    }
    uint32_t w[8][8];
    for (int i = 0; i < 8; i++) _mm256_storeu_si256((__m256i*)w[i], h[i]);
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 8; k++) memcpy(out + 32 * i + 4 * k, &w[k][i], 4);
}

/* ------------------------------------------------------------------ dispatch + hashing */
int sdo_simd_level(int requested) {
    /* 2 = AVX-512, 1 = AVX2, 0 = none; requested < 0 = best available */
    int have = __builtin_cpu_supports("avx512f") ? 2 : (__builtin_cpu_supports("avx2") ? 1 : 0);
    int lvl = requested < 0 || requested > have ? have : requested;
    if (lvl == 2 && !a5_ready) a5_init();
    if (lvl == 1 && !a2_ready) a2_init();
    return lvl;
}

static void hash_many(int lvl, const uint8_t* const* in, int n, int blocks, uint64_t ctr0, int inc, uint32_t flags,
                      uint32_t fstart, uint32_t fend, uint8_t* out) {
    const int W = lvl == 2 ? 16 : 8;
    for (int off = 0; off < n; off += W) {
        int k = n - off < W ? n - off : W;
        if (lvl == 2)
            a5_hash_many(in + off, k, blocks, ctr0 + (inc ? (uint64_t)off : 0), inc, flags, fstart, fend, out + 32 * off);
        else
            a2_hash_many(in + off, k, blocks, ctr0 + (inc ? (uint64_t)off : 0), inc, flags, fstart, fend, out + 32 * off);
    }
}

static void scalar_chunk(const uint8_t* p, uint32_t len, uint64_t counter, int root, uint32_t cv[8]) {
    uint32_t m[16], o[16];
    memcpy(cv, IV_, 32);
    uint32_t nb = len == 0 ? 1 : (len + 63) / 64;
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t bl = b + 1 < nb ? 64 : len - 64 * b;
        uint8_t blk[64] = {0};
        memcpy(blk, p + 64 * b, bl);
        memcpy(m, blk, 64);
        uint32_t fl = (b == 0 ? FS_CHUNK_START : 0) | (b + 1 == nb ? FS_CHUNK_END : 0) | (root && b + 1 == nb ? FS_ROOT : 0);
        sdo_compress_words(cv, m, counter, bl, fl, o);
        memcpy(cv, o, 32);
    }
}

/* One-shot BLAKE3 of data[0, len) with SIMD multi-chunk hashing at level lvl (1 or 2).
 * scratch must hold 32 * ceil(len / 1024) bytes (the CV array). */
void sdo_blake3_simd(const uint8_t* data, uint64_t len, uint8_t out[32], int lvl, uint8_t* scratch) {
    const uint64_t C = len == 0 ? 1 : (len + 1023) / 1024;
    if (C == 1) {
        uint32_t cv[8];
        scalar_chunk(data, (uint32_t)len, 0, 1, cv);
        memcpy(out, cv, 32);
        return;
    }
    const uint8_t* ptrs[64];
    /* full chunks 0..C-2 */
    for (uint64_t c0 = 0; c0 < C - 1; c0 += 64) {
        int k = (int)((C - 1 - c0) < 64 ? (C - 1 - c0) : 64);
        for (int i = 0; i < k; i++) ptrs[i] = data + 1024 * (c0 + i);
        hash_many(lvl, ptrs, k, 16, c0, 1, 0, FS_CHUNK_START, FS_CHUNK_END, scratch + 32 * c0);
    }
    uint32_t cv[8];
    scalar_chunk(data + 1024 * (C - 1), (uint32_t)(len - 1024 * (C - 1)), C - 1, 0, cv);
    memcpy(scratch + 32 * (C - 1), cv, 32);
    /* level-wise parents, in place (parent p reads nodes 2p, 2p+1 = 64 contiguous bytes) */
    uint64_t nodes = C;
    while (nodes > 2) {
        uint64_t P = nodes / 2;
        for (uint64_t p0 = 0; p0 < P; p0 += 64) {
            int k = (int)((P - p0) < 64 ? (P - p0) : 64);
            uint8_t tmp[64 * 32];
            for (int i = 0; i < k; i++) ptrs[i] = scratch + 64 * (p0 + i);
            hash_many(lvl, ptrs, k, 1, 0, 0, FS_PARENT, 0, 0, tmp);
            memcpy(scratch + 32 * p0, tmp, 32 * (size_t)k);
        }
        if (nodes & 1) memmove(scratch + 32 * P, scratch + 32 * (nodes - 1), 32);
        nodes = P + (nodes & 1);
    }
    uint32_t m[16], o[16];
    memcpy(m, scratch, 64);
    sdo_compress_words(IV_, m, 0, 64, FS_PARENT | FS_ROOT, o);
    memcpy(out, o, 32);
}

/* CV of the subtree over data[0, len) whose first chunk has index chunk0 -- an aligned
 * power-of-two group of chunks, or the final group of a message -- merged level-wise
 * (the odd node carried up), non-root; or, with root (chunk0 = 0), the whole message's
 * hash.  lvl 0 = scalar compressions, 1/2 = hash_many.  scratch: 32 * ceil(len/1024). */
void sdo_subtree_simd(const uint8_t* data, uint64_t len, uint64_t chunk0, int root, uint8_t out[32], int lvl,
                      uint8_t* scratch) {
    const uint64_t C = len == 0 ? 1 : (len + 1023) / 1024;
    uint32_t cv[8], m[16], o[16];
    if (C == 1) {
        scalar_chunk(data, (uint32_t)len, chunk0, root, cv);
        memcpy(out, cv, 32);
        return;
    }
    const uint8_t* ptrs[64];
    for (uint64_t c0 = 0; c0 < C - 1; c0 += 64) {
        int k = (int)((C - 1 - c0) < 64 ? (C - 1 - c0) : 64);
        if (lvl) {
            for (int i = 0; i < k; i++) ptrs[i] = data + 1024 * (c0 + i);
            hash_many(lvl, ptrs, k, 16, chunk0 + c0, 1, 0, FS_CHUNK_START, FS_CHUNK_END, scratch + 32 * c0);
        } else {
            for (int i = 0; i < k; i++) {
                scalar_chunk(data + 1024 * (c0 + i), 1024, chunk0 + c0 + i, 0, cv);
                memcpy(scratch + 32 * (c0 + i), cv, 32);
            }
        }
    }
    scalar_chunk(data + 1024 * (C - 1), (uint32_t)(len - 1024 * (C - 1)), chunk0 + C - 1, 0, cv);
    memcpy(scratch + 32 * (C - 1), cv, 32);
    uint64_t nodes = C;
    while (nodes > 2) {
        uint64_t P = nodes / 2;
        for (uint64_t p = 0; p < P; p++) {
            memcpy(m, scratch + 64 * p, 64);
            sdo_compress_words(IV_, m, 0, 64, FS_PARENT, o);
            memcpy(scratch + 32 * p, o, 32);
        }
        if (nodes & 1) memmove(scratch + 32 * P, scratch + 32 * (nodes - 1), 32);
        nodes = P + (nodes & 1);
    }
    memcpy(m, scratch, 64);
    sdo_compress_words(IV_, m, 0, 64, FS_PARENT | (root ? FS_ROOT : 0), o);
    memcpy(out, o, 32);
}

/* ----------------------------------------------- multi-threaded checksum of one file */
/* Full BLAKE3 (hash.rs:10-24) of one synthetic file of `size` bytes (content cid/twin of
 * sdo_synth_fill) on nthreads threads: the threads generate 1 MiB windows and hash their
 * chunks with hash_many into one CV array, then the CVs merge level-wise as in
 * sdo_blake3_simd.  Test infrastructure for files of several GiB, where the streaming
 * scalar restatement (sdo_checksums_synth) takes minutes. */
#include <pthread.h>
#include <stdatomic.h>
void sdo_synth_fill(uint64_t cid, uint32_t twin, uint64_t offset, uint64_t length, uint8_t* out);

typedef struct {
    const uint8_t* data; /* the message in memory, or NULL: generate (cid, twin) per block */
    uint64_t size, C, cid;
    uint32_t twin;
    int lvl;
    uint8_t* cvs;
    atomic_ullong next;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    uint8_t* buf = (uint8_t*)malloc(1u << 20);
    const uint8_t* ptrs[64];
    for (;;) {
        uint64_t w = atomic_fetch_add(&j->next, 1);
        uint64_t c_begin = w * 1024;
        if (c_begin >= j->C) break;
        uint64_t off = c_begin * 1024;
        uint64_t n = j->size - off < (1u << 20) ? j->size - off : (1u << 20);
        const uint8_t* src = buf;
        if (j->data) src = j->data + off;
        else sdo_synth_fill(j->cid, j->twin, off, n, buf);
        uint64_t c_end = c_begin + 1024 < j->C ? c_begin + 1024 : j->C;
        uint64_t full_end = c_end == j->C ? j->C - 1 : c_end; /* the file's last chunk: scalar */
        for (uint64_t c0 = c_begin; c0 < full_end; c0 += 64) {
            int k = (int)((full_end - c0) < 64 ? (full_end - c0) : 64);
            for (int i = 0; i < k; i++) ptrs[i] = src + 1024 * (c0 + i - c_begin);
            hash_many(j->lvl, ptrs, k, 16, c0, 1, 0, FS_CHUNK_START, FS_CHUNK_END, j->cvs + 32 * c0);
        }
        if (c_end == j->C) {
            uint32_t cv[8];
            scalar_chunk(src + 1024 * (j->C - 1 - c_begin), (uint32_t)(j->size - 1024 * (j->C - 1)), j->C - 1, 0, cv);
            memcpy(j->cvs + 32 * (j->C - 1), cv, 32);
        }
    }
    free(buf);
    return NULL;
}

static int checksum_mt(const uint8_t* data, uint64_t size, uint64_t cid, uint32_t twin, int nthreads, int simd,
                       uint8_t out[32]) {
    int lvl = sdo_simd_level(simd < 0 ? -1 : simd);
    if (lvl == 0 || size <= 1024) { /* scalar path or a single chunk */
        void sdo_blake3(const uint8_t*, size_t, uint8_t*);
        if (data) {
            sdo_blake3(data, size, out);
            return lvl;
        }
        uint8_t* b = (uint8_t*)malloc(size ? size : 1);
        sdo_synth_fill(cid, twin, 0, size, b);
        sdo_blake3(b, size, out);
        free(b);
        return lvl;
    }
    mt_job j;
    j.data = data;
    j.size = size; j.C = (size + 1023) / 1024; j.cid = cid; j.twin = twin; j.lvl = lvl;
    j.cvs = (uint8_t*)malloc(32 * j.C);
    atomic_store(&j.next, 0);
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, mt_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    const uint8_t* ptrs[64];
    uint64_t nodes = j.C;
    while (nodes > 2) {
        uint64_t P = nodes / 2;
        for (uint64_t p0 = 0; p0 < P; p0 += 64) {
            int k = (int)((P - p0) < 64 ? (P - p0) : 64);
            uint8_t tmp[64 * 32];
            for (int i = 0; i < k; i++) ptrs[i] = j.cvs + 64 * (p0 + i);
            hash_many(lvl, ptrs, k, 1, 0, 0, FS_PARENT, 0, 0, tmp);
            memcpy(j.cvs + 32 * p0, tmp, 32 * (size_t)k);
        }
        if (nodes & 1) memmove(j.cvs + 32 * P, j.cvs + 32 * (nodes - 1), 32);
        nodes = P + (nodes & 1);
    }
    uint32_t m[16], o[16];
    memcpy(m, j.cvs, 64);
    sdo_compress_words(IV_, m, 0, 64, FS_PARENT | FS_ROOT, o);
    memcpy(out, o, 32);
    free(j.cvs);
    return lvl;
}

int sdo_checksum_synth_mt(uint64_t size, uint64_t cid, uint32_t twin, int nthreads, int simd, uint8_t out[32]) {
    return checksum_mt(NULL, size, cid, twin, nthreads, simd, out);
}

/* the same, chunk-parallel, over a message in memory (a multi-GiB file's bytes) */
int sdo_checksum_mt(const uint8_t* data, uint64_t size, int nthreads, int simd, uint8_t out[32]) {
    return checksum_mt(data, size, 0, 0, nthreads, simd, out);
}
