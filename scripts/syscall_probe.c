// syscall_probe.c -- cost of the system calls the file stager makes per file, on this host
// (one thread): getppid, open+close of a tmpfs file, 1-byte and 10 KiB preads, lseek(END).
// Build/run: gcc -O2 -o /tmp/syscall_probe scripts/syscall_probe.c && /tmp/syscall_probe
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
static double now() { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
int main() {
    char path[] = "/dev/shm/sysprobe_XXXXXX";
    int fd = mkstemp(path);
    static char buf[1 << 20];
    memset(buf, 7, sizeof buf);
    if (write(fd, buf, sizeof buf) != sizeof buf) return 1;
    const int N = 200000;
    double t0 = now();
    for (int i = 0; i < N; i++) getppid();
    double t_ppid = (now() - t0) / N;
    t0 = now();
    for (int i = 0; i < N; i++) { int f = open(path, O_RDONLY | O_CLOEXEC); close(f); }
    double t_oc = (now() - t0) / N;
    t0 = now();
    for (int i = 0; i < N; i++) if (pread(fd, buf, 1, (i * 4099) % (1 << 20)) != 1) return 2;
    double t_p1 = (now() - t0) / N;
    t0 = now();
    for (int i = 0; i < N; i++) if (pread(fd, buf, 10240, (i * 4096) % ((1 << 20) - 10240)) != 10240) return 3;
    double t_p10k = (now() - t0) / N;
    t0 = now();
    for (int i = 0; i < N; i++) lseek(fd, -8192, SEEK_END);
    double t_ls = (now() - t0) / N;
    printf("{\"getppid_us\": %.3f, \"open_close_us\": %.3f, \"pread_1B_us\": %.3f, \"pread_10KiB_us\": %.3f, "
           "\"lseek_end_us\": %.3f}\n", t_ppid * 1e6, t_oc * 1e6, t_p1 * 1e6, t_p10k * 1e6, t_ls * 1e6);
    close(fd);
    unlink(path);
    return 0;
}
