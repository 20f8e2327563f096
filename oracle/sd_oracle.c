/*
 * sd_oracle.c -- CPU restatement of Spacedrive's content-addressing path.
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/build/libsd_oracle.so.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, as the checker
 * and as the timed CPU baseline ("kind": "port").  The product library
 * (spacedrive_amd/libsdcas.so) never links or calls it; the library's own CPU path
 * (spacedrive_amd/csrc/cpu_blake3.cpp, the sd_cpu_* entry points and the batch policies
 * that route to them) is a separate implementation, checked against this one by tests/.
 *
 * Restates:
 *   generate_cas_id  /root/reference/core/src/object/cas.rs:23-62 (consts :10-15)
 *   file_checksum    /root/reference/core/src/object/validation/hash.rs:10-24
 *   blake3 1.4.1     /root/reference/Cargo.lock:625-628 (crate not vendored; restated
 *                    from the BLAKE3 spec -- incremental CV-stack hasher, the same
 *                    structure as the crate's portable Hasher)
 * Pinned by tests/test_oracle.py against the tests/golden JSON fixtures, which the pure-Python
 * spec (oracle/blake3_spec.py, itself pinned to the in-repo KAT DERIVE_B3_EXPECTED,
 * crates/crypto/src/keys/hashing.rs:210-213, and the official BLAKE3 vectors) wrote.
 *
 * The batch entry points run on `nthreads` POSIX threads pulling files from an atomic
 * cursor: nthreads = 1 is the faithful reference schedule (one hashing task per
 * identifier step, core/src/object/file_identifier/mod.rs:107-134, no rayon), and
 * nthreads = nproc is the all-cores variant of the CPU baseline.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define B3_BLOCK 64u
#define B3_CHUNK 1024u
enum { F_CHUNK_START = 1, F_CHUNK_END = 2, F_PARENT = 4, F_ROOT = 8 };

static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define G(a, b, c, d, x, y)                                  \
    do {                                                     \
        s[a] = s[a] + s[b] + (x); s[d] = rotr32(s[d] ^ s[a], 16); \
        s[c] = s[c] + s[d];       s[b] = rotr32(s[b] ^ s[c], 12); \
        s[a] = s[a] + s[b] + (y); s[d] = rotr32(s[d] ^ s[a], 8);  \
        s[c] = s[c] + s[d];       s[b] = rotr32(s[b] ^ s[c], 7);  \
    } while (0)

/* out16 may alias nothing; returns the 16-word extended output */
static void b3_compress(const uint32_t cv[8], const uint8_t block[64], uint64_t counter,
                        uint32_t block_len, uint32_t flags, uint32_t out16[16]) {
    uint32_t m[16], t[16], s[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) |
               ((uint32_t)block[4 * i + 2] << 16) | ((uint32_t)block[4 * i + 3] << 24);
    for (int i = 0; i < 8; i++) s[i] = cv[i];
    s[8] = B3_IV[0]; s[9] = B3_IV[1]; s[10] = B3_IV[2]; s[11] = B3_IV[3];
    s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32);
    s[14] = block_len; s[15] = flags;
    for (int r = 0; r < 7; r++) {
        G(0, 4, 8, 12, m[0], m[1]);   G(1, 5, 9, 13, m[2], m[3]);
        G(2, 6, 10, 14, m[4], m[5]);  G(3, 7, 11, 15, m[6], m[7]);
        G(0, 5, 10, 15, m[8], m[9]);  G(1, 6, 11, 12, m[10], m[11]);
        G(2, 7, 8, 13, m[12], m[13]); G(3, 4, 9, 14, m[14], m[15]);
        for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) { out16[i] = s[i] ^ s[i + 8]; out16[i + 8] = s[i + 8] ^ cv[i]; }
}

/* word-level compression (little-endian message words), used by sd_oracle_simd.c */
void sdo_compress_words(const uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len,
                        uint32_t flags, uint32_t out16[16]) {
    uint8_t blk[64];
    for (int i = 0; i < 16; i++) {
        blk[4 * i] = (uint8_t)m[i]; blk[4 * i + 1] = (uint8_t)(m[i] >> 8);
        blk[4 * i + 2] = (uint8_t)(m[i] >> 16); blk[4 * i + 3] = (uint8_t)(m[i] >> 24);
    }
    b3_compress(cv, blk, counter, block_len, flags, out16);
}

/* ------------------------------------------------------------- incremental hasher */
typedef struct {
    uint32_t cv[8];
    uint64_t chunk_counter;
    uint8_t buf[64];
    uint32_t buf_len;
    uint32_t blocks_compressed;
    uint32_t stack[54][8];
    uint32_t stack_len;
} b3_hasher;

static void b3_init(b3_hasher* h) {
    memcpy(h->cv, B3_IV, 32);
    h->chunk_counter = 0; h->buf_len = 0; h->blocks_compressed = 0; h->stack_len = 0;
}

static uint32_t chunk_start_flag(const b3_hasher* h) { return h->blocks_compressed ? 0 : F_CHUNK_START; }

static void parent_cv(const uint32_t l[8], const uint32_t r[8], uint32_t flags, uint32_t out[8]) {
    uint8_t blk[64];
    for (int i = 0; i < 8; i++) { memcpy(blk + 4 * i, &l[i], 4); memcpy(blk + 32 + 4 * i, &r[i], 4); }
    uint32_t o[16];
    b3_compress(B3_IV, blk, 0, 64, F_PARENT | flags, o);
    memcpy(out, o, 32);
}

static void push_chunk_cv(b3_hasher* h, uint32_t cv[8], uint64_t total) {
    uint32_t cur[8];
    memcpy(cur, cv, 32);
    while ((total & 1) == 0) {
        h->stack_len--;
        parent_cv(h->stack[h->stack_len], cur, 0, cur);
        total >>= 1;
    }
    memcpy(h->stack[h->stack_len++], cur, 32);
}

static void b3_update(b3_hasher* h, const uint8_t* p, size_t n) {
    /* little-endian host assumed (x86-64); the block bytes are parsed portably anyway */
    while (n) {
        uint32_t chunk_len = h->blocks_compressed * B3_BLOCK + h->buf_len;
        if (chunk_len == B3_CHUNK) {
            uint32_t o[16];
            b3_compress(h->cv, h->buf, h->chunk_counter, 64,
                        chunk_start_flag(h) | F_CHUNK_END, o);
            uint64_t total = h->chunk_counter + 1;
            push_chunk_cv(h, o, total);
            memcpy(h->cv, B3_IV, 32);
            h->chunk_counter = total; h->buf_len = 0; h->blocks_compressed = 0;
        }
        if (h->buf_len == B3_BLOCK) {
            uint32_t o[16];
            b3_compress(h->cv, h->buf, h->chunk_counter, 64, chunk_start_flag(h), o);
            memcpy(h->cv, o, 32);
            h->blocks_compressed++; h->buf_len = 0;
        }
        uint32_t room_chunk = B3_CHUNK - (h->blocks_compressed * B3_BLOCK + h->buf_len);
        uint32_t take = B3_BLOCK - h->buf_len;
        if (take > room_chunk) take = room_chunk;
        if (take > n) take = (uint32_t)n;
        memcpy(h->buf + h->buf_len, p, take);
        h->buf_len += take; p += take; n -= take;
    }
}

static void b3_finalize(const b3_hasher* h, uint8_t out[32]) {
    uint8_t blk[64];
    memset(blk, 0, 64);
    memcpy(blk, h->buf, h->buf_len);
    uint32_t flags = chunk_start_flag(h) | F_CHUNK_END;
    uint32_t o[16];
    if (h->stack_len == 0) {
        b3_compress(h->cv, blk, h->chunk_counter, h->buf_len, flags | F_ROOT, o);
    } else {
        uint32_t cur[8];
        b3_compress(h->cv, blk, h->chunk_counter, h->buf_len, flags, o);
        memcpy(cur, o, 32);
        for (int i = (int)h->stack_len - 1; i >= 1; i--) parent_cv(h->stack[i], cur, 0, cur);
        uint8_t pb[64];
        for (int i = 0; i < 8; i++) { memcpy(pb + 4 * i, &h->stack[0][i], 4); memcpy(pb + 32 + 4 * i, &cur[i], 4); }
        b3_compress(B3_IV, pb, 0, 64, F_PARENT | F_ROOT, o);
    }
    for (int i = 0; i < 8; i++) memcpy(out + 4 * i, &o[i], 4);
}

void sdo_blake3(const uint8_t* data, size_t len, uint8_t out[32]) {
    b3_hasher h;
    b3_init(&h);
    b3_update(&h, data, len);
    b3_finalize(&h, out);
}

/* ---------------------------------------------------------------- cas.rs restated */
#define SAMPLE_COUNT 4u
#define SAMPLE_SIZE (1024u * 10u)
#define HEADER_OR_FOOTER_SIZE (1024u * 8u)
#define MINIMUM_FILE_SIZE (1024u * 100u)
#define SAMPLED_MSG_LEN (8u + 2u * HEADER_OR_FOOTER_SIZE + SAMPLE_COUNT * SAMPLE_SIZE)

uint64_t sdo_cas_message_len(uint64_t size) {
    return size <= MINIMUM_FILE_SIZE ? 8 + size : SAMPLED_MSG_LEN;
}

/* sample window offsets, cas.rs:35-58 traced literally (see oracle/cas_spec.py), for a
 * file whose length is `size`: the footer window is at (file length - 8192), cas.rs:54
 * seeks SeekFrom::End(-8192).  read_cas_message takes the footer from the real end of
 * the file instead (the two agree when the file length equals `size`). */
static int cas_windows(uint64_t size, uint64_t off[6], uint64_t len[6]) {
    int k = 0;
    off[k] = 0; len[k++] = HEADER_OR_FOOTER_SIZE;
    uint64_t current_pos = HEADER_OR_FOOTER_SIZE;
    uint64_t seek_jump = (size - 2ull * HEADER_OR_FOOTER_SIZE) / SAMPLE_COUNT;
    for (;;) {
        off[k] = current_pos; len[k++] = SAMPLE_SIZE;
        if (current_pos >= HEADER_OR_FOOTER_SIZE + seek_jump * (SAMPLE_COUNT - 1)) break;
        current_pos += seek_jump;
    }
    off[k] = size - HEADER_OR_FOOTER_SIZE; len[k++] = HEADER_OR_FOOTER_SIZE;
    return k;
}

/* ------------------------------------------------------------- synthetic content */
#define SYNTH_SEED 0x5D5DCA51Dull
#define GOLDEN 0x9E3779B97F4A7C15ull
#define TWIN_OFFSET (HEADER_OR_FOOTER_SIZE + SAMPLE_SIZE)

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void sdo_synth_fill(uint64_t cid, uint32_t twin, uint64_t offset, uint64_t length, uint8_t* out) {
    uint64_t key = SYNTH_SEED ^ (cid * GOLDEN);
    for (uint64_t i = 0; i < length;) {
        uint64_t o = offset + i;
        uint64_t w = splitmix64(key ^ (o >> 3));
        uint32_t b = (uint32_t)(o & 7);
        while (b < 8 && i < length) { out[i++] = (uint8_t)(w >> (8 * b)); b++; }
    }
    if (twin && offset <= TWIN_OFFSET && TWIN_OFFSET < offset + length)
        out[TWIN_OFFSET - offset] ^= (uint8_t)((twin & 0xFF) | 1);
}

/* writes the exact generate_cas_id hashed stream of a synthetic file into out */
uint64_t sdo_synth_cas_message(uint64_t cid, uint32_t twin, uint64_t size, uint8_t* out) {
    for (int i = 0; i < 8; i++) out[i] = (uint8_t)(size >> (8 * i)); /* cas.rs:25 le64 */
    if (size <= MINIMUM_FILE_SIZE) {                                  /* cas.rs:27-29 */
        sdo_synth_fill(cid, twin, 0, size, out + 8);
        return 8 + size;
    }
    uint64_t off[6], len[6], pos = 8;
    int k = cas_windows(size, off, len);
    for (int i = 0; i < k; i++) { sdo_synth_fill(cid, twin, off[i], len[i], out + pos); pos += len[i]; }
    return pos;
}

/* ------------------------------------------------------------ threaded batch runs */
typedef struct {
    uint64_t size, msg_offset;
    uint32_t msg_len, kind;
} sdo_extent; /* same layout as sd_extent in include/sd_cas.h */

void sdo_blake3_simd(const uint8_t* data, uint64_t len, uint8_t out[32], int lvl, uint8_t* scratch);
int sdo_simd_level(int requested);

typedef struct {
    int mode;
    int simd; /* 0 = scalar incremental hasher; 1 = AVX2, 2 = AVX-512 multi-chunk */
    uint64_t n;
    const uint8_t* staged;
    const sdo_extent* ext;
    const uint64_t *sizes, *cids;
    const uint32_t* twins;
    const uint8_t* data;
    const uint64_t *offsets, *lens;
    const char* const* paths;
    int32_t* status;
    uint8_t* out;
    uint32_t out_stride;
    atomic_ullong cursor;
} job_t;

enum { MODE_CAS_STAGED = 0, MODE_CAS_SYNTH = 1, MODE_CHECKSUM = 2, MODE_CHECKSUM_SYNTH = 3, MODE_CAS_FILES = 4,
       MODE_FILE_CHECKSUM = 5 };

/* read exactly n bytes at the current position (read_exact); 0 ok, -1 EOF, else errno */
static int read_exact_fd(int fd, uint8_t* p, uint64_t n) {
    while (n) {
        ssize_t r = read(fd, p, n);
        if (r < 0) { if (errno == EINTR) continue; return errno; }
        if (r == 0) return -1;
        p += r; n -= (uint64_t)r;
    }
    return 0;
}

/* generate_cas_id (cas.rs:23-62) with the reference's own read schedule:
 *   size <= 102400 (:27-29): fs::read -- the file's actual bytes, read until read()
 *     returns 0, whatever their count (the file may be shorter or longer than `size`,
 *     which is only hashed as the le64 header, :25);
 *   else (:31-58): open, read_exact(head) at 0, then per sample read_exact at current_pos
 *     and seek(Start(current_pos + seek_jump)), then seek(End(-8192)) -- relative to the
 *     file's real end, failing with EINVAL when the file is shorter than 8192 bytes --
 *     and read_exact(tail).
 * The message is assembled in *msg (realloc'd to *cap as needed; the le64 header first,
 * :25); returns its length, or -1 with *st = 2 | errno << 16 (I/O error) or 3
 * (read_exact's UnexpectedEof), as sd_file_status. */
static int64_t read_cas_message(const char* path, uint64_t size, uint8_t** msg, uint64_t* cap, int32_t* st) {
    if (*cap < 8 + SAMPLED_MSG_LEN + 64) {
        *cap = 8 + MINIMUM_FILE_SIZE + 64;
        *msg = (uint8_t*)realloc(*msg, *cap);
    }
    for (int i = 0; i < 8; i++) (*msg)[i] = (uint8_t)(size >> (8 * i));
    int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) { *st = 2 | (errno << 16); return -1; }
    uint64_t len = 8;
    int rc = 0;
    if (size <= MINIMUM_FILE_SIZE) { /* fs::read: read_to_end */
        for (;;) {
            if (*cap - len < 4096) { *cap *= 2; *msg = (uint8_t*)realloc(*msg, *cap); }
            ssize_t r = read(fd, *msg + len, *cap - len);
            if (r < 0) { if (errno == EINTR) continue; rc = errno; break; }
            if (r == 0) break;
            len += (uint64_t)r;
        }
    } else {
        uint64_t off[6], wl[6];
        int k = cas_windows(size, off, wl);
        for (int i = 0; i < k && !rc; i++) {
            off_t at;
            if (i == k - 1) at = lseek(fd, -(off_t)HEADER_OR_FOOTER_SIZE, SEEK_END); /* :54 */
            else at = lseek(fd, (off_t)off[i], SEEK_SET);
            if (at < 0) { rc = errno; break; }
            rc = read_exact_fd(fd, *msg + len, wl[i]);
            len += wl[i];
        }
    }
    close(fd);
    if (rc == -1) { *st = 3; return -1; }
    if (rc) { *st = 2 | (rc << 16); return -1; }
    *st = 0;
    return (int64_t)len;
}

/* subtree CV / whole-message hash with the SIMD hasher (sd_oracle_simd.c) */
void sdo_subtree_simd(const uint8_t* data, uint64_t len, uint64_t chunk0, int root, uint8_t out[32], int lvl,
                      uint8_t* scratch);

/* file_checksum (hash.rs:10-24) with the reference's read schedule: one read() of up to
 * BLOCK_LEN = 1 MiB per iteration (:15, tokio's File::read is one read call), every
 * returned byte hashed (:16), stop at the first read that returns fewer than 1 MiB
 * (:17-19).  The hasher is the crate's structure at 1 MiB granularity: each full 1 MiB
 * piece is a complete 1024-chunk subtree (hashed with hash_many when simd > 0), pushed
 * on a CV stack only once more input is known to follow (the crate's lazy merge), and
 * the final piece is merged down the stack with ROOT on the last parent.  Returns 0, or
 * an sd_file_status (2 | errno << 16). */
static int32_t file_checksum_fd(int fd, uint8_t out[32], int simd, uint8_t* buf, uint8_t* scratch) {
    const uint64_t BL = 1u << 20;
    uint32_t stack[64][8];
    int sp = 0;
    uint64_t blocks = 0, have = 0; /* `have`: bytes of the pending (last read) piece */
    int pending = 0;
    for (;;) {
        ssize_t r;
        for (;;) {
            r = read(fd, buf + (pending ? BL : 0), BL);
            if (r < 0 && errno == EINTR) continue;
            break;
        }
        if (r < 0) return 2 | (errno << 16);
        if (pending && r > 0) { /* the pending full piece is not the last: push its CV */
            uint8_t cv[32];
            sdo_subtree_simd(buf, BL, blocks * 1024, 0, cv, simd, scratch);
            blocks++;
            memcpy(stack[sp++], cv, 32);
            for (uint64_t t = blocks; (t & 1) == 0; t >>= 1) {
                sp--;
                parent_cv(stack[sp - 1], stack[sp], 0, stack[sp - 1]);
            }
            memmove(buf, buf + BL, (size_t)r);
        }
        if (!pending || r > 0) have = (uint64_t)r;
        pending = 1;
        if ((uint64_t)r != BL) break; /* :17-19 */
    }
    /* the last piece: buf[0, have) at chunk blocks * 1024 */
    if (sp == 0) {
        if (simd && have > 1024) sdo_subtree_simd(buf, have, 0, 1, out, simd, scratch);
        else sdo_blake3(buf, have, out);
        return 0;
    }
    uint32_t cur[8];
    sdo_subtree_simd(buf, have, blocks * 1024, 0, (uint8_t*)cur, simd, scratch);
    for (int i = sp - 1; i >= 1; i--) parent_cv(stack[i], cur, 0, cur);
    parent_cv(stack[0], cur, F_ROOT, cur);
    memcpy(out, cur, 32);
    return 0;
}


static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    uint8_t* scratch = NULL;
    uint64_t scratch_cap = 0;
    if (j->mode == MODE_CAS_SYNTH) scratch = (uint8_t*)malloc(8 + MINIMUM_FILE_SIZE);
    if (j->mode == MODE_CHECKSUM_SYNTH) scratch = (uint8_t*)malloc(1u << 20);
    if (j->mode == MODE_FILE_CHECKSUM) scratch = (uint8_t*)malloc((2u << 20) + 64);
    uint8_t* cvs = NULL;
    uint64_t cvs_cap = 0;
    for (;;) {
        uint64_t i = atomic_fetch_add(&j->cursor, 1);
        if (i >= j->n) break;
        uint8_t h[32];
        if (j->mode == MODE_FILE_CHECKSUM) {
            if (!cvs) { cvs_cap = 32 * 1025; cvs = (uint8_t*)malloc(cvs_cap); }
            memset(h, 0, 32);
            int fd = open(j->paths[i], O_RDONLY | O_CLOEXEC);
            if (fd < 0) j->status[i] = 2 | (errno << 16);
            else {
                j->status[i] = file_checksum_fd(fd, h, j->simd, scratch, cvs);
                close(fd);
            }
        } else if (j->mode == MODE_CAS_FILES) {
            int32_t st = 0;
            int64_t m = read_cas_message(j->paths[i], j->sizes[i], &scratch, &scratch_cap, &st);
            j->status[i] = st;
            if (m < 0) { memset(h, 0, 32); }
            else if (j->simd) {
                uint64_t need = 32 * (((uint64_t)m + 1023) / 1024 + 1);
                if (need > cvs_cap) { free(cvs); cvs_cap = need * 2; cvs = (uint8_t*)malloc(cvs_cap); }
                sdo_blake3_simd(scratch, (uint64_t)m, h, j->simd, cvs);
            } else {
                sdo_blake3(scratch, (uint64_t)m, h);
            }
        } else if (j->mode == MODE_CAS_STAGED && j->simd) {
            uint64_t need = 32 * ((j->ext[i].msg_len + 1023) / 1024 + 1);
            if (need > cvs_cap) { free(cvs); cvs_cap = need * 2; cvs = (uint8_t*)malloc(cvs_cap); }
            sdo_blake3_simd(j->staged + j->ext[i].msg_offset, j->ext[i].msg_len, h, j->simd, cvs);
        } else if (j->mode == MODE_CHECKSUM && j->simd) {
            uint64_t need = 32 * ((j->lens[i] + 1023) / 1024 + 1);
            if (need > cvs_cap) { free(cvs); cvs_cap = need * 2; cvs = (uint8_t*)malloc(cvs_cap); }
            sdo_blake3_simd(j->data + j->offsets[i], j->lens[i], h, j->simd, cvs);
        } else if (j->mode == MODE_CAS_STAGED) {
            sdo_blake3(j->staged + j->ext[i].msg_offset, j->ext[i].msg_len, h);
        } else if (j->mode == MODE_CAS_SYNTH) {
            uint64_t m = sdo_synth_cas_message(j->cids[i], j->twins ? j->twins[i] : 0, j->sizes[i], scratch);
            if (j->simd) {
                uint64_t need = 32 * ((m + 1023) / 1024 + 1);
                if (need > cvs_cap) { free(cvs); cvs_cap = need * 2; cvs = (uint8_t*)malloc(cvs_cap); }
                sdo_blake3_simd(scratch, m, h, j->simd, cvs);
            } else {
                sdo_blake3(scratch, m, h);
            }
        } else if (j->mode == MODE_CHECKSUM) {
            sdo_blake3(j->data + j->offsets[i], j->lens[i], h);
        } else { /* hash.rs:14-20: 1 MiB reads streamed through one hasher */
            b3_hasher hs;
            b3_init(&hs);
            uint64_t size = j->sizes[i];
            for (uint64_t pos = 0; pos < size; pos += (1u << 20)) {
                uint64_t n = size - pos < (1u << 20) ? size - pos : (1u << 20);
                sdo_synth_fill(j->cids[i], j->twins ? j->twins[i] : 0, pos, n, scratch);
                b3_update(&hs, scratch, n);
            }
            b3_finalize(&hs, h);
        }
        memcpy(j->out + (size_t)i * j->out_stride, h, j->out_stride);
    }
    free(scratch);
    free(cvs);
    return NULL;
}

static void run_job(job_t* j, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    atomic_store(&j->cursor, 0);
    if (nthreads == 1) { worker(j); return; }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
}

/* cas ids (first 8 hash bytes) of staged messages; simd: -1 best available, 0 scalar,
 * 1 AVX2, 2 AVX-512 (capped at what the CPU has).  Returns the level used. */
int sdo_cas_ids_staged_simd(const uint8_t* staged, const sdo_extent* ext, uint64_t n, uint8_t* out8, int nthreads,
                            int simd) {
    job_t j = {0};
    j.mode = MODE_CAS_STAGED; j.n = n; j.staged = staged; j.ext = ext; j.out = out8; j.out_stride = 8;
    j.simd = simd == 0 ? 0 : sdo_simd_level(simd);
    run_job(&j, nthreads);
    return j.simd;
}

void sdo_cas_ids_staged(const uint8_t* staged, const sdo_extent* ext, uint64_t n, uint8_t* out8, int nthreads) {
    sdo_cas_ids_staged_simd(staged, ext, n, out8, nthreads, 0);
}

/* full 32-byte hashes of byte ranges with the SIMD multi-chunk hasher */
int sdo_checksums_simd(const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                       uint8_t* out32, int nthreads, int simd) {
    job_t j = {0};
    j.mode = MODE_CHECKSUM; j.n = n; j.data = data; j.offsets = offsets; j.lens = lens;
    j.out = out32; j.out_stride = 32;
    j.simd = simd == 0 ? 0 : sdo_simd_level(simd);
    run_job(&j, nthreads);
    return j.simd;
}

/* cas ids of synthetic files: builds each message from the generator, then hashes */
void sdo_cas_ids_synth(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins, uint64_t n,
                       uint8_t* out8, int nthreads) {
    job_t j = {0};
    j.mode = MODE_CAS_SYNTH; j.n = n; j.sizes = sizes; j.cids = cids; j.twins = twins;
    j.out = out8; j.out_stride = 8;
    run_job(&j, nthreads);
}

/* the same with the SIMD multi-chunk hasher (library-scale parity runs: 10 M files);
 * simd as in sdo_cas_ids_staged_simd.  Returns the level used. */
int sdo_cas_ids_synth_simd(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins, uint64_t n,
                           uint8_t* out8, int nthreads, int simd) {
    job_t j = {0};
    j.mode = MODE_CAS_SYNTH; j.n = n; j.sizes = sizes; j.cids = cids; j.twins = twins;
    j.out = out8; j.out_stride = 8;
    j.simd = simd == 0 ? 0 : sdo_simd_level(simd);
    run_job(&j, nthreads);
    return j.simd;
}

/* full 32-byte BLAKE3 of n byte ranges of one buffer */
void sdo_checksums(const uint8_t* data, const uint64_t* offsets, const uint64_t* lens, uint64_t n,
                   uint8_t* out32, int nthreads) {
    job_t j = {0};
    j.mode = MODE_CHECKSUM; j.n = n; j.data = data; j.offsets = offsets; j.lens = lens;
    j.out = out32; j.out_stride = 32;
    run_job(&j, nthreads);
}

/* full checksums of synthetic files streamed 1 MiB at a time (hash.rs:14-20) */
void sdo_checksums_synth(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins, uint64_t n,
                         uint8_t* out32, int nthreads) {
    job_t j = {0};
    j.mode = MODE_CHECKSUM_SYNTH; j.n = n; j.sizes = sizes; j.cids = cids; j.twins = twins;
    j.out = out32; j.out_stride = 32;
    run_job(&j, nthreads);
}

/* stage the exact cas messages of synthetic files at the given offsets (host buffer) */
void sdo_stage_synth(const uint64_t* sizes, const uint64_t* cids, const uint32_t* twins,
                     const uint64_t* offsets, uint64_t n, uint8_t* buf) {
    for (uint64_t i = 0; i < n; i++)
        sdo_synth_cas_message(cids[i], twins ? twins[i] : 0, sizes[i], buf + offsets[i]);
}

/* cas ids of files on disk through the reference's read schedule (read_cas_message);
 * status[n] as sd_file_status.  simd as sdo_cas_ids_staged_simd.  Returns the level. */
int sdo_cas_ids_files(const char* const* paths, const uint64_t* sizes, uint64_t n, uint8_t* out8, int32_t* status,
                      int nthreads, int simd) {
    job_t j = {0};
    j.mode = MODE_CAS_FILES; j.n = n; j.paths = paths; j.sizes = sizes; j.status = status;
    j.out = out8; j.out_stride = 8;
    j.simd = simd == 0 ? 0 : sdo_simd_level(simd);
    run_job(&j, nthreads);
    return j.simd;
}

/* full checksums of files on disk through the reference's read schedule
 * (file_checksum_fd, hash.rs:10-24); status[n] as sd_file_status.  Returns the level. */
int sdo_file_checksums(const char* const* paths, uint64_t n, uint8_t* out32, int32_t* status, int nthreads, int simd) {
    job_t j = {0};
    j.mode = MODE_FILE_CHECKSUM; j.n = n; j.paths = paths; j.status = status;
    j.out = out32; j.out_stride = 32;
    j.simd = simd == 0 ? 0 : sdo_simd_level(simd);
    run_job(&j, nthreads);
    return j.simd;
}
