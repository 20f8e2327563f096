// uring_probe.c -- can io_uring cut the per-file host cost of the cas stager?
//
// The GPU route of sd_cas_ids_files is bound by its readers: ~10 host CPU-us per file from
// the page cache, for an open, 1-5 reads and a close -- up to 7 syscalls --
// plus the copies.  io_uring can issue a whole file as one linked chain -- OPENAT into a
// direct (registered) descriptor slot, the READs on that slot, CLOSE of the slot -- and a
// batch of files per io_uring_enter, so a thread pays one kernel entry per batch and never
// touches the process's fd table.  This probe reads the stager's exact windows (cas.rs:
// 25-58: a whole file's bytes + 1 probe byte; a sampled file's head + sample 0 in one read,
// samples 1-3, and the footer read of 8192 + 1 bytes at size - 8192) for a library-mixture
// file set on tmpfs, two ways on T threads:
//   pread : open / pread x k / close per file, each thread on a private fd table (as the stager)
//   uring : one ring per thread, batches of B files as linked chains on direct descriptors
// and prints files/s and host CPU-us per file (getrusage of the process) per mode.
// Every result byte is compared between the modes.
//
// Build: gcc -O2 -o scripts/uring_probe scripts/uring_probe.c -lpthread
// Run:   scripts/uring_probe [nfiles=200000] [threads=16] [batch=32] [rd]
//        (rd, round 5: the reads only through io_uring, opens and closes plain syscalls)
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#define MINWHOLE 102400ull
#define SLOT (128u << 10)  // per-file destination: <= 102401 (whole + probe) or 57352 + 1

static int NF = 200000, T = 16, B = 32;
static const char* DIR = "/dev/shm/sd_uring_probe";
static uint64_t* sizes;
static uint64_t *dig_a, *dig_b;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}
static double cpu_s(void) {
    struct rusage r;
    getrusage(RUSAGE_SELF, &r);
    return r.ru_utime.tv_sec + r.ru_utime.tv_usec * 1e-6 + r.ru_stime.tv_sec + r.ru_stime.tv_usec * 1e-6;
}
static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}
static uint64_t digest(const uint8_t* p, uint64_t n, int64_t status) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)status;
    for (uint64_t i = 0; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = mix64(h ^ w);
    }
    for (uint64_t i = n & ~7ull; i < n; i++) h = mix64(h ^ p[i]);
    return h ^ n;
}
static void path_of(int i, char* buf) { snprintf(buf, 256, "%s/f%07d", DIR, i); }

// the stager's reads of file i: (offset, length) pairs; returns their count
static int plan(int i, uint64_t off[5], uint64_t len[5]) {
    const uint64_t s = sizes[i];
    if (s <= MINWHOLE) {  // cas.rs:29 fs::read: the planned room + 1 probe byte
        off[0] = 0;
        len[0] = s + 1;
        return 1;
    }
    const uint64_t j = (s - 16384) / 4;  // cas.rs:41
    off[0] = 0;
    len[0] = 8192 + 10240;  // head + sample 0 (contiguous)
    for (int k = 1; k < 4; k++) {
        off[k] = 8192 + k * j;
        len[k] = 10240;
    }
    off[4] = s - 8192;  // the footer + 1 byte: exactly 8192 back means the end is at size
    len[4] = 8193;
    return 5;
}

static void make_files(void) {
    mkdir(DIR, 0700);
    sizes = malloc(sizeof(uint64_t) * NF);
    uint64_t x = 12345;
    static uint8_t buf[128 << 10];
    for (size_t k = 0; k < sizeof buf; k++) buf[k] = (uint8_t)(k * 131 + 7);
    for (int i = 0; i < NF; i++) {
        x = mix64(x + i);
        const double u = (double)(x >> 11) / 9007199254740992.0;
        uint64_t s;
        if (i % 5 < 3)  // 60 %: log-uniform in [1, 102400], hashed whole
            s = (uint64_t)exp(u * log(102400.0));
        else  // 40 %: log-uniform in [102401, 4 GiB], sampled (written sparse)
            s = 102401 + (uint64_t)exp(u * log(4294967296.0 - 102401));
        if (s < 1) s = 1;
        sizes[i] = s;
        char p[256];
        path_of(i, p);
        const int fd = open(p, O_CREAT | O_TRUNC | O_WRONLY, 0600);
        if (fd < 0) exit(3);
        uint64_t off[5], len[5];
        const int n = plan(i, off, len);
        if (s <= MINWHOLE) {
            if (write(fd, buf, s) != (ssize_t)s) exit(4);
        } else {
            for (int k = 0; k < n; k++) {
                const uint64_t l = k == 4 ? 8192 : len[k];
                buf[0] = (uint8_t)i;
                if (pwrite(fd, buf, l, off[k]) != (ssize_t)l) exit(4);
            }
            if (ftruncate(fd, s) != 0) exit(4);
        }
        close(fd);
    }
}

// ---------------------------------------------------------------- pread mode
static volatile int cursor_a;
static void* worker_pread(void* arg) {
    (void)arg;
    unshare(CLONE_FILES);  // a private fd table (stage_pool.h)
    uint8_t* dst = aligned_alloc(4096, SLOT);
    for (;;) {
        const int i0 = __atomic_fetch_add(&cursor_a, 64, __ATOMIC_RELAXED);
        if (i0 >= NF) break;
        for (int i = i0; i < i0 + 64 && i < NF; i++) {
            char p[256];
            path_of(i, p);
            uint64_t off[5], len[5];
            const int n = plan(i, off, len);
            const int fd = open(p, O_RDONLY | O_CLOEXEC);
            uint64_t pos = 0, got = 0;
            int64_t st = fd < 0 ? -errno : 0;
            for (int k = 0; k < n && fd >= 0; k++) {
                const ssize_t r = pread(fd, dst + pos, len[k], (off_t)off[k]);
                if (r < 0) {
                    st = -errno;
                    break;
                }
                st = st * 131 + r;
                pos += len[k];
                got += (uint64_t)r;
            }
            if (fd >= 0) close(fd);
            dig_a[i] = digest(dst, got, st);
        }
    }
    free(dst);
    return NULL;
}

// ---------------------------------------------------------------- io_uring mode
struct ring {
    int fd;
    unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
    struct io_uring_sqe* sqes;
    struct io_uring_cqe* cqes;
};
static int ring_init(struct ring* r, unsigned entries) {
    struct io_uring_params p;
    memset(&p, 0, sizeof p);
    r->fd = (int)syscall(__NR_io_uring_setup, entries, &p);
    if (r->fd < 0) return -errno;
    size_t sq_sz = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    size_t cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(struct io_uring_cqe);
    uint8_t* sq = mmap(0, sq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_SQ_RING);
    uint8_t* cq = mmap(0, cq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_CQ_RING);
    r->sqes = mmap(0, p.sq_entries * sizeof(struct io_uring_sqe), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE,
                   r->fd, IORING_OFF_SQES);
    if (sq == MAP_FAILED || cq == MAP_FAILED || r->sqes == MAP_FAILED) return -ENOMEM;
    r->sq_head = (unsigned*)(sq + p.sq_off.head);
    r->sq_tail = (unsigned*)(sq + p.sq_off.tail);
    r->sq_mask = (unsigned*)(sq + p.sq_off.ring_mask);
    r->sq_array = (unsigned*)(sq + p.sq_off.array);
    r->cq_head = (unsigned*)(cq + p.cq_off.head);
    r->cq_tail = (unsigned*)(cq + p.cq_off.tail);
    r->cq_mask = (unsigned*)(cq + p.cq_off.ring_mask);
    r->cqes = (struct io_uring_cqe*)(cq + p.cq_off.cqes);
    // a sparse table of direct descriptors, one slot per file of a batch
    int fds[1024];
    for (int k = 0; k < 1024; k++) fds[k] = -1;
    if (syscall(__NR_io_uring_register, r->fd, IORING_REGISTER_FILES, fds, 1024) < 0) return -errno;
    return 0;
}
static struct io_uring_sqe* sqe_get(struct ring* r) {
    const unsigned tail = *r->sq_tail;
    const unsigned idx = tail & *r->sq_mask;
    struct io_uring_sqe* s = &r->sqes[idx];
    memset(s, 0, sizeof *s);
    r->sq_array[idx] = idx;
    __atomic_store_n(r->sq_tail, tail + 1, __ATOMIC_RELEASE);
    return s;
}

static volatile int cursor_b;
static int uring_failed;
static void* worker_uring(void* arg) {
    (void)arg;
    struct ring r;
    const int rc = ring_init(&r, 1024);
    if (rc < 0) {
        fprintf(stderr, "io_uring setup: %s\n", strerror(-rc));
        uring_failed = 1;
        return NULL;
    }
    uint8_t* dst = aligned_alloc(4096, (size_t)SLOT * B);
    char(*paths)[256] = malloc(256 * (size_t)B);
    int64_t res[64][8];
    for (;;) {
        const int i0 = __atomic_fetch_add(&cursor_b, B, __ATOMIC_RELAXED);
        if (i0 >= NF) break;
        const int nb = i0 + B <= NF ? B : NF - i0;
        int nsqe = 0;
        for (int q = 0; q < nb; q++) {
            const int i = i0 + q;
            path_of(i, paths[q]);
            uint64_t off[5], len[5];
            const int n = plan(i, off, len);
            struct io_uring_sqe* s = sqe_get(&r);  // OPENAT into direct slot q
            s->opcode = IORING_OP_OPENAT;
            s->fd = AT_FDCWD;
            s->addr = (uint64_t)(uintptr_t)paths[q];
            s->open_flags = O_RDONLY;  // (O_CLOEXEC is refused for direct descriptors)
            s->file_index = (uint32_t)q + 1;
            s->flags = IOSQE_IO_HARDLINK;  // hard: a short read (EOF) must not cancel the rest
            s->user_data = ((uint64_t)q << 8) | 0;
            uint64_t pos = 0;
            for (int k = 0; k < n; k++) {
                s = sqe_get(&r);
                s->opcode = IORING_OP_READ;
                s->fd = q;  // the direct descriptor
                s->flags = IOSQE_FIXED_FILE | IOSQE_IO_HARDLINK;
                s->addr = (uint64_t)(uintptr_t)(dst + (size_t)q * SLOT + pos);
                s->len = (uint32_t)len[k];
                s->off = off[k];
                s->user_data = ((uint64_t)q << 8) | (uint64_t)(k + 1);
                pos += len[k];
            }
            s = sqe_get(&r);  // CLOSE the slot: the end of the chain, after the reads
            s->opcode = IORING_OP_CLOSE;
            s->file_index = (uint32_t)q + 1;
            s->user_data = ((uint64_t)q << 8) | 7;
            nsqe += n + 2;
            for (int k = 0; k < 8; k++) res[q][k] = INT64_MIN;
        }
        int done = 0;
        while (done < nsqe) {
            const int want = nsqe - done;
            const int sub = done == 0 ? nsqe : 0;
            if (syscall(__NR_io_uring_enter, r.fd, sub, want, IORING_ENTER_GETEVENTS, NULL, 0) < 0 && errno != EINTR) {
                fprintf(stderr, "io_uring_enter: %s\n", strerror(errno));
                uring_failed = 1;
                return NULL;
            }
            unsigned head = *r.cq_head;
            const unsigned tail = __atomic_load_n(r.cq_tail, __ATOMIC_ACQUIRE);
            for (; head != tail; head++) {
                const struct io_uring_cqe* c = &r.cqes[head & *r.cq_mask];
                res[c->user_data >> 8][c->user_data & 0xFF] = c->res;
                done++;
            }
            __atomic_store_n(r.cq_head, head, __ATOMIC_RELEASE);
        }
        for (int q = 0; q < nb; q++) {
            const int i = i0 + q;
            uint64_t off[5], len[5];
            const int n = plan(i, off, len);
            int64_t st = res[q][0] < 0 ? res[q][0] : 0;
            uint64_t got = 0;
            for (int k = 0; k < n && res[q][0] >= 0; k++) {
                if (res[q][k + 1] < 0) {
                    st = res[q][k + 1];
                    break;
                }
                st = st * 131 + res[q][k + 1];
                got += (uint64_t)res[q][k + 1];
            }
            // (the pread mode's digest covers the same bytes: each read lands after the last)
            dig_b[i] = digest(dst + (size_t)q * SLOT, got, st);
            if (res[q][7] < 0 || res[q][0] < 0) {  // the OPENAT or the CLOSE failed
                if (!uring_failed)
                    fprintf(stderr, "file %d: openat %lld, reads %lld %lld, close %lld\n", i, (long long)res[q][0],
                            (long long)res[q][1], (long long)res[q][2], (long long)res[q][7]);
                uring_failed = 2;
            }
        }
    }
    free(dst);
    free(paths);
    close(r.fd);
    return NULL;
}

// ---------------------------------------------------------------- io_uring for the reads only
// (round 5) the opens and closes stay plain syscalls on the thread's private fd table (round
// 4's OPENAT went to io-wq workers); a batch of B files' reads is one io_uring_enter, each
// read on a plain descriptor, completed inline when the pages are cached
static volatile int cursor_c;
static int urd_failed;
static uint64_t* dig_c;
static void* worker_uring_rd(void* arg) {
    (void)arg;
    unshare(CLONE_FILES);
    struct ring r;
    const int rc = ring_init(&r, 1024);
    if (rc < 0) {
        fprintf(stderr, "io_uring setup: %s\n", strerror(-rc));
        urd_failed = 1;
        return NULL;
    }
    uint8_t* dst = aligned_alloc(4096, (size_t)SLOT * B);
    int64_t res[64][6];
    int fds[64];
    for (;;) {
        const int i0 = __atomic_fetch_add(&cursor_c, B, __ATOMIC_RELAXED);
        if (i0 >= NF) break;
        const int nb = i0 + B <= NF ? B : NF - i0;
        int nsqe = 0;
        for (int q = 0; q < nb; q++) {
            const int i = i0 + q;
            char p[256];
            path_of(i, p);
            fds[q] = open(p, O_RDONLY | O_CLOEXEC);
            for (int k = 0; k < 6; k++) res[q][k] = INT64_MIN;
            res[q][0] = fds[q] < 0 ? -errno : 0;
            if (fds[q] < 0) continue;
            uint64_t off[5], len[5];
            const int n = plan(i, off, len);
            uint64_t pos = 0;
            for (int k = 0; k < n; k++) {
                struct io_uring_sqe* sq = sqe_get(&r);
                sq->opcode = IORING_OP_READ;
                sq->fd = fds[q];
                sq->addr = (uint64_t)(uintptr_t)(dst + (size_t)q * SLOT + pos);
                sq->len = (uint32_t)len[k];
                sq->off = off[k];
                sq->user_data = ((uint64_t)q << 8) | (uint64_t)(k + 1);
                pos += len[k];
            }
            nsqe += n;
        }
        int done = 0;
        while (done < nsqe) {
            const int sub = done == 0 ? nsqe : 0;
            if (syscall(__NR_io_uring_enter, r.fd, sub, nsqe - done, IORING_ENTER_GETEVENTS, NULL, 0) < 0 &&
                errno != EINTR) {
                fprintf(stderr, "io_uring_enter: %s\n", strerror(errno));
                urd_failed = 1;
                return NULL;
            }
            unsigned head = *r.cq_head;
            const unsigned tail = __atomic_load_n(r.cq_tail, __ATOMIC_ACQUIRE);
            for (; head != tail; head++) {
                const struct io_uring_cqe* c = &r.cqes[head & *r.cq_mask];
                res[c->user_data >> 8][c->user_data & 0xFF] = c->res;
                done++;
            }
            __atomic_store_n(r.cq_head, head, __ATOMIC_RELEASE);
        }
        for (int q = 0; q < nb; q++) {
            const int i = i0 + q;
            if (fds[q] >= 0) close(fds[q]);
            uint64_t off[5], len[5];
            const int n = plan(i, off, len);
            int64_t st = res[q][0];
            uint64_t got = 0, pos = 0;
            // the pread mode reads each window right after the last, stopping at an error;
            // its digest covers the bytes up to the first error, in order
            for (int k = 0; k < n && res[q][0] >= 0; k++) {
                if (res[q][k + 1] < 0) {
                    st = res[q][k + 1];
                    break;
                }
                st = st * 131 + res[q][k + 1];
                if (pos != got) memmove(dst + (size_t)q * SLOT + got, dst + (size_t)q * SLOT + pos, (size_t)res[q][k + 1]);
                got += (uint64_t)res[q][k + 1];
                pos += len[k];
            }
            dig_c[i] = digest(dst + (size_t)q * SLOT, got, st);
        }
    }
    free(dst);
    close(r.fd);
    return NULL;
}

static double run(void* (*fn)(void*), double* us_per_file) {
    pthread_t th[256];
    const double c0 = cpu_s(), t0 = now();
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, fn, NULL);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    const double dt = now() - t0;
    *us_per_file = (cpu_s() - c0) / NF * 1e6;
    return NF / dt;
}

int main(int argc, char** argv) {
    if (argc > 1) NF = atoi(argv[1]);
    if (argc > 2) T = atoi(argv[2]);
    if (argc > 3) B = atoi(argv[3]);
    if (B > 64) B = 64;
    make_files();
    dig_a = calloc(NF, 8);
    dig_b = calloc(NF, 8);
    dig_c = calloc(NF, 8);
    double us;
    if (argc > 4 && strcmp(argv[4], "rd") == 0) {  // pread vs io_uring for the reads only
        for (int rnd = 0; rnd < 3; rnd++) {
            cursor_a = 0;
            const double ra = run(worker_pread, &us);
            printf("{\"mode\": \"pread\", \"round\": %d, \"threads\": %d, \"files_per_s\": %.0f, "
                   "\"cpu_us_per_file\": %.2f}\n", rnd, T, ra, us);
            cursor_c = 0;
            const double rc = run(worker_uring_rd, &us);
            int same = 1;
            for (int i = 0; i < NF; i++) same &= dig_a[i] == dig_c[i];
            printf("{\"mode\": \"uring_reads\", \"round\": %d, \"threads\": %d, \"batch\": %d, \"files_per_s\": %.0f, "
                   "\"cpu_us_per_file\": %.2f, \"same_bytes\": %s, \"failed\": %d}\n",
                   rnd, T, B, rc, us, same ? "true" : "false", urd_failed);
            fflush(stdout);
            if (urd_failed) break;
        }
        char p[256];
        for (int i = 0; i < NF; i++) {
            path_of(i, p);
            unlink(p);
        }
        rmdir(DIR);
        return 0;
    }
    for (int rnd = 0; rnd < 3; rnd++) {
        cursor_a = 0;
        const double ra = run(worker_pread, &us);
        printf("{\"mode\": \"pread\", \"round\": %d, \"threads\": %d, \"files_per_s\": %.0f, \"cpu_us_per_file\": %.2f}\n",
               rnd, T, ra, us);
        cursor_b = 0;
        const double rb = run(worker_uring, &us);
        int same = 1;
        for (int i = 0; i < NF; i++) same &= dig_a[i] == dig_b[i];
        printf("{\"mode\": \"uring\", \"round\": %d, \"threads\": %d, \"batch\": %d, \"files_per_s\": %.0f, "
               "\"cpu_us_per_file\": %.2f, \"same_bytes\": %s, \"failed\": %d}\n",
               rnd, T, B, rb, us, same ? "true" : "false", uring_failed);
        fflush(stdout);
        if (uring_failed) break;
    }
    char p[256];
    for (int i = 0; i < NF; i++) {
        path_of(i, p);
        unlink(p);
    }
    rmdir(DIR);
    return 0;
}
