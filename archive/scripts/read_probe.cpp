// Host read probe for the file-backed checksum leg: parallel 1 MiB preads from a tmpfs file
// into pageable memory and into hipHostMalloc'd (pinned) memory, by thread count.
// Build: hipcc -O2 -std=c++17 scripts/read_probe.cpp -o scripts/read_probe (in-tree, on CPU)
// Run on the GPU box: ./scripts/read_probe [MiB]   -> one JSON line
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double run(int fd, uint8_t* buf, size_t size, int nt) {
    const size_t piece = 1 << 20, pieces = size / piece;
    double best = 0;
    for (int rep = 0; rep < 3; rep++) {
        std::atomic<size_t> next{0};
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < nt; t++)
            th.emplace_back([&] {
                for (size_t k; (k = next.fetch_add(1)) < pieces;)
                    if (pread(fd, buf + k * piece, piece, (off_t)(k * piece)) != (ssize_t)piece) abort();
            });
        for (auto& x : th) x.join();
        const double gbps = size / (now() - t0) / 1e9;
        if (gbps > best) best = gbps;
    }
    return best;
}

int main(int argc, char** argv) {
    const size_t size = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
    std::string path = "/dev/shm/read_probe_" + std::to_string(getpid());
    {
        std::vector<uint8_t> tmp(size);
        for (size_t i = 0; i < size; i++) tmp[i] = (uint8_t)(i * 2654435761u >> 13);
        FILE* f = fopen(path.c_str(), "wb");
        if (!f || fwrite(tmp.data(), 1, size, f) != size) return 1;
        fclose(f);
    }
    const int fd = open(path.c_str(), O_RDONLY);
    uint8_t* pageable = (uint8_t*)aligned_alloc(4096, size);
    uint8_t* pinned = nullptr;
    if (hipHostMalloc((void**)&pinned, size, hipHostMallocDefault) != hipSuccess) pinned = nullptr;
    uint8_t* pinned_nc = nullptr;
    if (hipHostMalloc((void**)&pinned_nc, size, hipHostMallocNonCoherent) != hipSuccess) pinned_nc = nullptr;
    memset(pageable, 0, size);
    if (pinned) memset(pinned, 0, size);
    if (pinned_nc) memset(pinned_nc, 0, size);
    printf("{\"bytes\": %zu", size);
    const int nts[] = {1, 4, 8, 16, 32};
    for (int nt : nts) printf(", \"pageable_t%d\": %.2f", nt, run(fd, pageable, size, nt));
    if (pinned)
        for (int nt : nts) printf(", \"pinned_t%d\": %.2f", nt, run(fd, pinned, size, nt));
    if (pinned_nc)
        for (int nt : nts) printf(", \"pinned_noncoherent_t%d\": %.2f", nt, run(fd, pinned_nc, size, nt));
    // memcpy bandwidth pageable -> pinned, for comparison (16 threads)
    {
        double best = 0;
        for (int rep = 0; rep < 3 && pinned; rep++) {
            const double t0 = now();
            std::vector<std::thread> th;
            for (int t = 0; t < 16; t++)
                th.emplace_back([&, t] {
                    const size_t per = size / 16;
                    memcpy(pinned + t * per, pageable + t * per, per);
                });
            for (auto& x : th) x.join();
            const double g = size / (now() - t0) / 1e9;
            if (g > best) best = g;
        }
        printf(", \"memcpy_to_pinned_t16\": %.2f", best);
    }
    printf(", \"unit\": \"GB/s\"}\n");
    close(fd);
    unlink(path.c_str());
    return 0;
}
