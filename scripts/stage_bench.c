// stage_bench.c -- host staging microbenchmark: pread threads (mode 0) vs io_uring batches
// (mode 1) reading the generate_cas_id windows (cas.rs:27-58) of a file list; mode 2 = the
// preads of mode 0 into a per-thread 128 KiB buffer (cache-hot, as the CPU path reads)
// instead of each file's slot of one large buffer; mode 3 = mode 2, then the message copied
// to its slot of the large buffer with non-temporal (streaming) stores; mode 4 = the same
// with memcpy; mode 5 = mode 0 with each thread on a private file-descriptor table
// (unshare(CLONE_FILES)), so open/close do not share the process's fd-table lock.  Not part
// of the product; used to choose the stager design.
#define _GNU_SOURCE
#include <sched.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <immintrin.h>

static int n; static char** paths; static uint64_t* sizes; static uint8_t* buf; static uint64_t* offs;
static atomic_int cursor; static int mode, B = 64;
static double now() { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
static int wins(uint64_t size, uint64_t off[6], uint64_t len[6]) {
    if (size <= 102400) { off[0] = 0; len[0] = size; return 1; }
    uint64_t j = (size - 16384) / 4; int k = 0;
    off[k] = 0; len[k++] = 8192;
    for (int s = 0; s < 4; s++) { off[k] = 8192 + s * j; len[k++] = 10240; }
    off[k] = size - 8192; len[k++] = 8192; return k;
}
static void nt_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {  /* 64-B aligned dst, n % 64 == 0 */
    for (uint64_t i = 0; i < n; i += 64) {
        __m128i a = _mm_load_si128((const __m128i*)(src + i)), b = _mm_load_si128((const __m128i*)(src + i + 16));
        __m128i c = _mm_load_si128((const __m128i*)(src + i + 32)), d = _mm_load_si128((const __m128i*)(src + i + 48));
        _mm_stream_si128((__m128i*)(dst + i), a); _mm_stream_si128((__m128i*)(dst + i + 16), b);
        _mm_stream_si128((__m128i*)(dst + i + 32), c); _mm_stream_si128((__m128i*)(dst + i + 48), d);
    }
    _mm_sfence();
}
static void* w_pread(void* a) {
    if (mode == 5 && unshare(CLONE_FILES) != 0) { perror("unshare"); exit(1); }
    uint8_t* hot = (mode >= 2 && mode <= 4) ? aligned_alloc(4096, 128 << 10) : 0;
    if (hot) memset(hot, 0, 128 << 10);
    for (;;) {
        int i = atomic_fetch_add(&cursor, 1); if (i >= n) break;
        int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
        uint64_t o[6], l[6]; int k = wins(sizes[i], o, l); uint8_t* d = hot ? hot + 8 : buf + offs[i] + 8;
        for (int q = 0; q < k; q++) { pread(fd, d, l[q], o[q]); d += l[q]; }
        close(fd);
        uint64_t m = ((sizes[i] <= 102400 ? 8 + sizes[i] : 57352) + 63) / 64 * 64;
        if (mode == 3) nt_copy(buf + offs[i], hot, m);
        if (mode == 4) memcpy(buf + offs[i], hot, m);
    }
    free(hot);
    return 0;
}
struct ring { int fd; unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask; struct io_uring_sqe* sqes; struct io_uring_cqe* cqes; };
static int ring_init(struct ring* r, unsigned entries) {
    struct io_uring_params p; memset(&p, 0, sizeof p);
    r->fd = syscall(__NR_io_uring_setup, entries, &p); if (r->fd < 0) return -1;
    size_t sqsz = p.sq_off.array + p.sq_entries * 4, cqsz = p.cq_off.cqes + p.cq_entries * sizeof(struct io_uring_cqe);
    uint8_t* sq = mmap(0, sqsz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_SQ_RING);
    uint8_t* cq = mmap(0, cqsz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_CQ_RING);
    r->sqes = mmap(0, p.sq_entries * sizeof(struct io_uring_sqe), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_SQES);
    r->sq_head = (unsigned*)(sq + p.sq_off.head); r->sq_tail = (unsigned*)(sq + p.sq_off.tail); r->sq_mask = (unsigned*)(sq + p.sq_off.ring_mask); r->sq_array = (unsigned*)(sq + p.sq_off.array);
    r->cq_head = (unsigned*)(cq + p.cq_off.head); r->cq_tail = (unsigned*)(cq + p.cq_off.tail); r->cq_mask = (unsigned*)(cq + p.cq_off.ring_mask); r->cqes = (struct io_uring_cqe*)(cq + p.cq_off.cqes);
    return 0;
}
static void* w_uring(void* a) {
    struct ring r; if (ring_init(&r, 512)) { perror("uring"); exit(1); }
    int fds[64];
    for (;;) {
        int i0 = atomic_fetch_add(&cursor, B); if (i0 >= n) break;
        int i1 = i0 + B < n ? i0 + B : n;
        unsigned tail = *r.sq_tail, cnt = 0;
        for (int i = i0; i < i1; i++) {
            fds[i - i0] = open(paths[i], O_RDONLY | O_CLOEXEC);
            uint64_t o[6], l[6]; int k = wins(sizes[i], o, l); uint8_t* d = buf + offs[i] + 8;
            for (int q = 0; q < k; q++) {
                unsigned idx = tail & *r.sq_mask; struct io_uring_sqe* s = &r.sqes[idx]; memset(s, 0, sizeof *s);
                s->opcode = IORING_OP_READ; s->fd = fds[i - i0]; s->addr = (uint64_t)d; s->len = l[q]; s->off = o[q];
                r.sq_array[idx] = idx; tail++; cnt++; d += l[q];
            }
        }
        __atomic_store_n(r.sq_tail, tail, __ATOMIC_RELEASE);
        int got = syscall(__NR_io_uring_enter, r.fd, cnt, cnt, IORING_ENTER_GETEVENTS, 0, 0);
        if (got < 0) { perror("enter"); exit(1); }
        unsigned done = 0;
        while (done < cnt) {
            unsigned h = *r.cq_head, t = __atomic_load_n(r.cq_tail, __ATOMIC_ACQUIRE);
            while (h != t) { if (r.cqes[h & *r.cq_mask].res < 0) { fprintf(stderr, "read err\n"); } h++; done++; }
            __atomic_store_n(r.cq_head, h, __ATOMIC_RELEASE);
            if (done < cnt) syscall(__NR_io_uring_enter, r.fd, 0, cnt - done, IORING_ENTER_GETEVENTS, 0, 0);
        }
        for (int i = i0; i < i1; i++) close(fds[i - i0]);
    }
    return 0;
}
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "r"); int T = atoi(argv[2]); mode = atoi(argv[3]); if (argc > 4) B = atoi(argv[4]);
    fscanf(f, "%d", &n); paths = malloc(n * sizeof(char*)); sizes = malloc(n * 8); offs = malloc(n * 8);
    uint64_t tot = 0;
    for (int i = 0; i < n; i++) { char p[512]; unsigned long long s; fscanf(f, "%s %llu", p, &s); paths[i] = strdup(p); sizes[i] = s; offs[i] = tot; tot += ((s <= 102400 ? 8 + s : 57352) + 63) / 64 * 64; }
    buf = aligned_alloc(4096, (tot + 4095) / 4096 * 4096); memset(buf, 0, tot);
    for (int rep = 0; rep < 3; rep++) {
        struct rusage ru0, ru1; getrusage(RUSAGE_SELF, &ru0);
        atomic_store(&cursor, 0); pthread_t th[64]; double t0 = now();
        for (int t = 0; t < T; t++) pthread_create(&th[t], 0, mode == 1 ? w_uring : w_pread, 0);
        for (int t = 0; t < T; t++) pthread_join(th[t], 0);
        double dt = now() - t0; getrusage(RUSAGE_SELF, &ru1);
        double cpu = (ru1.ru_utime.tv_sec - ru0.ru_utime.tv_sec) + (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) +
                     1e-6 * ((ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec) + (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec));
        printf("mode %d T %d: %.1f ms, %.0f files/s, %.2f GB/s, %.2f cpu-us/file\n", mode, T, dt * 1e3, n / dt,
               tot / dt / 1e9, cpu / n * 1e6);
    }
    return 0;
}
