// Can the GPU route read a cached file without the host copying it (round 5)?  The split
// validator's host cost is the pread copy into pinned memory (0.07-0.10 ns per byte,
// DESIGN.md §4.1).  If a file's page-cache pages could be mapped (mmap) and registered with
// HIP (hipHostRegister), the DMA engine would read them straight from the page cache with no
// host copy at all.  This probe measures, for a file on tmpfs: whether registering a
// read-only shared mapping works (HIP ignores hipHostRegisterReadOnly on AMD, so the pages may
// be requested writable), what registering costs per byte, the H2D rate from the
// registration, and that the bytes arrive intact.  A private writable mapping is tried too
// (it would copy every page on write-fault: the cost shows whether that happens).
//   hipcc --offload-arch=gfx950 -O2 scripts/mmap_register_probe.cpp -o scripts/mmap_register_probe
//   scripts/mmap_register_probe [dir=/dev/shm] [MiB=256]  -> JSON lines
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/dev/shm";
    const size_t mib = argc > 2 ? strtoull(argv[2], nullptr, 10) : 256;
    const size_t len = mib << 20;
    const std::string path = dir + "/sd_mmap_register_probe.bin";
    std::vector<uint8_t> want(len);
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < len; i += 8) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        memcpy(&want[i], &x, 8);
    }
    {
        int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        if (fd < 0 || write(fd, want.data(), len) != (ssize_t)len) { perror("write"); return 1; }
        close(fd);
    }
    uint8_t* dev = nullptr;
    if (hipMalloc(&dev, len) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); return 1; }
    std::vector<uint8_t> back(len);
    struct Mode { const char* name; int prot, flags, oflags; };
    const Mode modes[] = {{"shared_readonly", PROT_READ, MAP_SHARED, O_RDONLY},
                          {"private_writable", PROT_READ | PROT_WRITE, MAP_PRIVATE, O_RDONLY}};
    for (const size_t win : {len, (size_t)32 << 20}) {
        for (const Mode& m : modes) {
            int fd = open(path.c_str(), m.oflags);
            double t_map = 0, t_reg = 0, t_h2d = 0, t_unreg = 0;
            hipError_t rc = hipSuccess;
            for (size_t off = 0; off < len && rc == hipSuccess; off += win) {
                double t0 = now();
                void* p = mmap(nullptr, win, m.prot, m.flags, fd, (off_t)off);
                if (p == MAP_FAILED) { perror("mmap"); return 1; }
                double t1 = now();
                rc = hipHostRegister(p, win, hipHostRegisterDefault);
                double t2 = now();
                if (rc == hipSuccess) {
                    (void)hipMemcpy(dev + off, p, win, hipMemcpyHostToDevice);
                    double t3 = now();
                    (void)hipHostUnregister(p);
                    t_h2d += t3 - t2;
                    t_unreg += now() - t3;
                }
                munmap(p, win);
                t_map += t1 - t0;
                t_reg += t2 - t1;
            }
            close(fd);
            bool equal = false;
            if (rc == hipSuccess) {
                (void)hipMemcpy(back.data(), dev, len, hipMemcpyDeviceToHost);
                equal = memcmp(back.data(), want.data(), len) == 0;
            }
            (void)hipMemset(dev, 0, len);
            printf("{\"mode\": \"%s\", \"window_MiB\": %zu, \"file_MiB\": %zu, \"register\": \"%s\", "
                   "\"mmap_s\": %.6f, \"register_s\": %.6f, \"register_GBps\": %.2f, \"h2d_s\": %.6f, \"h2d_GBps\": %.2f, "
                   "\"unregister_s\": %.6f, \"bytes_equal\": %s}\n",
                   m.name, win >> 20, mib, hipGetErrorString(rc), t_map, t_reg, len / t_reg / 1e9, t_h2d,
                   t_h2d > 0 ? len / t_h2d / 1e9 : 0.0, t_unreg, equal ? "true" : "false");
            fflush(stdout);
        }
    }
    // threads registering windows at once: do registrations serialise (the process's mmap
    // lock, the driver's), or does the registration rate add up?
    const size_t W = (size_t)32 << 20, nw = len / W;
    for (const int T : {1, 2, 4, 8}) {
        std::vector<double> t_reg(T, 0.0);
        std::vector<int> bad(T, 0);
        int fd = open(path.c_str(), O_RDONLY);
        double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                hipStream_t s;
                (void)hipStreamCreate(&s);
                for (size_t w = t; w < nw; w += T) {
                    void* p = mmap(nullptr, W, PROT_READ, MAP_SHARED, fd, (off_t)(w * W));
                    if (p == MAP_FAILED) { bad[t]++; continue; }
                    double a = now();
                    if (hipHostRegister(p, W, hipHostRegisterDefault) != hipSuccess) { bad[t]++; munmap(p, W); continue; }
                    t_reg[t] += now() - a;
                    (void)hipMemcpyAsync(dev + w * W, p, W, hipMemcpyHostToDevice, s);
                    (void)hipStreamSynchronize(s);
                    (void)hipHostUnregister(p);
                    munmap(p, W);
                }
                (void)hipStreamDestroy(s);
            });
        for (auto& x : th) x.join();
        const double wall = now() - t0;
        close(fd);
        (void)hipMemcpy(back.data(), dev, nw * W, hipMemcpyDeviceToHost);
        const bool equal = memcmp(back.data(), want.data(), nw * W) == 0;
        double reg = 0;
        int nbad = 0;
        for (int t = 0; t < T; t++) { reg += t_reg[t]; nbad += bad[t]; }
        printf("{\"mode\": \"threads\", \"threads\": %d, \"window_MiB\": %zu, \"file_MiB\": %zu, \"wall_s\": %.6f, "
               "\"GBps\": %.2f, \"register_s_sum\": %.6f, \"register_GBps_per_thread\": %.2f, \"failed\": %d, "
               "\"bytes_equal\": %s}\n", T, W >> 20, mib, wall, nw * W / wall / 1e9, reg, nw * W / reg / 1e9 * T / T,
               nbad, equal ? "true" : "false");
        fflush(stdout);
        (void)hipMemset(dev, 0, len);
    }
    unlink(path.c_str());
    (void)hipFree(dev);
    return 0;
}
