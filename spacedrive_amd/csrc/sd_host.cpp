// sd_host.cpp -- GPU-free host logic of libsdcas (see sd_host.h): batch planners, the
// file stager with generate_cas_id's read semantics (cas.rs:23-62), and the sequential
// message reader with file_checksum's (hash.rs:10-24).
#include "sd_host.h"

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/syscall.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <emmintrin.h>

#include <algorithm>
#include <atomic>

// ------------------------------------------------------------------ errors, knobs
namespace {
thread_local std::string g_err;
// defaults: 200 us coalescing window, 4096-request batches, 32 MiB file windows, LDS-bucket
// dedup grouping, single-file calls on the CPU while fewer than 16 are in flight, 16 reader
// threads for sd_file_checksums, the one-wave-per-file sampled kernel up to 6144 files
// and one workgroup per whole-kind file up to 512 files (profiles/r2/r2z_small_batch_kernels.json:
// the crossovers lie between 4096 and 8192 sampled files, 256 and 1024 whole-kind files),
// sd_cas_ids_files calls of up to 4096 files on the CPU path (profiles/r3/r3p_batch_sizes.json,
// p50 per call from the page cache on 16 threads: GPU route / CPU path 286 / 109 us at 100
// files, 3.39 / 3.07 ms at 4000, 6.24 / 6.36 ms at 8000, 10.8 / 13.7 ms at 16000 -- a call's
// fixed GPU-route cost loses below ~8000 files), 4 pinned windows the stager may fill ahead, every
// sd_file_checksums call on the CPU path unless it is large enough to split (DESIGN.md §4:
// from the page cache the host hashes faster than PCIe carries the bytes), the stager's
// readers through their cache-resident buffers (profiles/r3/r3n_files_ab_private_fds.json:
// 1.04 vs 0.84 M files/s), large sd_file_checksums calls split between the GPU route (at most
// 6 of the 16 threads feeding it at once) and the CPU path, claimed by 1 MiB blocks, the GPU
// route's readers through pread_stream (profiles/r5/r5e_hybrid_blocks.json: 1.20-1.43x the
// CPU path alone from the page cache), the CPU path's block reads in 256 KiB pieces
// (profiles/r5/r5d_hybrid.json: 1.04-1.07x); no host thread budget override; library threads left unplaced
// ("numa_pin" 0: placing them on the GPU's node measured neutral with the page cache where
// the writer left it, profiles/r4/r4h_numa_lib_probe.json); 15 host threads hashing beside the GPU in
// large sd_cas_ids calls (profiles/r3/r3ad_cohash_probe.json: 300 000 files from pinned memory,
// GPU alone 1.89-1.94 M files/s, CPU path alone 2.24-2.36 M, both at once 3.87-4.08 M); a
// 5-minute bound on every wait of the RCCL exchange for its peers (torch's own NCCL watchdog
// waits 10)
std::atomic<int> g_tune[SD_TUNE_NKEYS] = {{200}, {4096}, {32}, {1}, {16}, {16}, {6144}, {512}, {4096}, {4}, {2147483647}, {1}, {6}, {15}, {0}, {1}, {0}, {256}, {1}, {8}, {300000}};
const char* const TUNE_NAMES[SD_TUNE_NKEYS] = {"coalesce_window_us", "coalesce_max",    "files_window_mb",
                                               "dedup_variant",      "latency_cpu_max", "read_threads",
                                               "sampled_wave_max",   "whole_wave_max",  "batch_cpu_max",
                                               "files_ring",         "checksum_cpu_max", "files_stage_hot",
                                               "checksum_hybrid_threads", "host_cohash_threads",
                                               "host_cpu_budget",    "checksum_stage_hot", "numa_pin",
                                               "cpu_read_piece_kib", "checksum_split_blocks",
                                               "checksum_split_adapt", "comm_timeout_ms"};

bool read_small(const std::string& path, char* buf, size_t cap) {
    FILE* f = fopen(path.c_str(), "re");
    if (!f) return false;
    const size_t got = fread(buf, 1, cap - 1, f);
    fclose(f);
    buf[got] = 0;
    return got > 0;
}
}  // namespace

// ------------------------------------------------------------------ host thread budget
CpuBudget cpu_budget_resolve(int affinity, int online, double quota_cpus, int local_world) {
    CpuBudget b;
    b.affinity = std::max(1, affinity);
    b.online = std::max(b.affinity, online);
    b.quota_milli = quota_cpus > 0 ? (int)std::min(1e9, quota_cpus * 1000.0 + 0.5) : 0;
    b.local_world = std::max(1, local_world);
    // The affinity mask is this process's own: a mask narrower than the machine is a per-rank
    // binding (numactl, Slurm --cpu-bind, a launcher's placement) and already this rank's
    // share; a mask of every online CPU is shared by the node's ranks and is split.
    const int aff_share = b.affinity >= b.online ? b.affinity / b.local_world : b.affinity;
    int cpus = std::max(1, aff_share);
    // the cgroup quota covers every rank in the container: always split.  A fractional quota
    // still runs that many threads' worth of time: round up (1.5 CPUs allows 2 threads)
    if (quota_cpus > 0) cpus = std::min(cpus, std::max(1, (int)(quota_cpus + 0.999) / b.local_world));
    b.budget = std::max(1, cpus);
    return b;
}

double cgroup_cpu_quota(const char* root) {
    char buf[128];
    const std::string r = root ? root : "/sys/fs/cgroup";
    if (read_small(r + "/cpu.max", buf, sizeof buf)) {  // v2: "<quota|max> <period>"
        char q[32] = {0};
        double period = 0;
        if (sscanf(buf, "%31s %lf", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
            return atof(q) / period;
        return 0;
    }
    char pb[64];  // v1: cfs quota -1 = unlimited
    if (read_small(r + "/cpu/cpu.cfs_quota_us", buf, sizeof buf) &&
        read_small(r + "/cpu/cpu.cfs_period_us", pb, sizeof pb)) {
        const double q = atof(buf), p = atof(pb);
        if (q > 0 && p > 0) return q / p;
    }
    return 0;
}

namespace {
// one directory's own limit: v2 cpu.max, or v1 cpu.cfs_quota_us / cpu.cfs_period_us
double cgroup_dir_quota(const std::string& dir, bool v1) {
    char buf[128], pb[64];
    if (!v1) {
        if (!read_small(dir + "/cpu.max", buf, sizeof buf)) return 0;
        char q[32] = {0};
        double period = 0;
        if (sscanf(buf, "%31s %lf", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) return atof(q) / period;
        return 0;
    }
    if (read_small(dir + "/cpu.cfs_quota_us", buf, sizeof buf) && read_small(dir + "/cpu.cfs_period_us", pb, sizeof pb)) {
        const double q = atof(buf), p = atof(pb);
        if (q > 0 && p > 0) return q / p;
    }
    return 0;
}
double min_quota(double a, double b) { return a <= 0 ? b : (b <= 0 ? a : std::min(a, b)); }
}  // namespace

double cgroup_cpu_quota_self(const char* root, const char* proc_cgroup) {
    const std::string mnt = root ? root : "/sys/fs/cgroup";
    // the process's own cgroup: "0::/path" (v2), or "N:...cpu...:/path" (v1)
    std::string v2path, v1path;
    bool have_v2 = false, have_v1 = false;
    if (FILE* f = fopen(proc_cgroup ? proc_cgroup : "/proc/self/cgroup", "re")) {
        char line[4096];
        while (fgets(line, sizeof line, f)) {
            line[strcspn(line, "\n")] = 0;
            char* c1 = strchr(line, ':');
            char* c2 = c1 ? strchr(c1 + 1, ':') : nullptr;
            if (!c2) continue;
            const std::string ctrl(c1 + 1, c2);
            if (strncmp(line, "0:", 2) == 0 && ctrl.empty()) {
                v2path = c2 + 1;
                have_v2 = true;
            } else {
                // v1 controller lists: "cpu", "cpu,cpuacct", "cpuacct,cpu"
                size_t s = 0;
                while (s <= ctrl.size()) {
                    size_t e = ctrl.find(',', s);
                    if (e == std::string::npos) e = ctrl.size();
                    if (ctrl.compare(s, e - s, "cpu") == 0) {
                        v1path = c2 + 1;
                        have_v1 = true;
                    }
                    s = e + 1;
                }
            }
        }
        fclose(f);
    }
    // the mount root's own limit (a private cgroup namespace shows "/" and lands here)
    double q = cgroup_cpu_quota(mnt.c_str());
    // walk from the process's cgroup up to the mount root: the tightest limit on the way
    // binds (systemd slices, cgroupns=host containers keep it in a nested directory)
    auto walk = [&](const std::string& base, std::string rel, bool v1) {
        while (!rel.empty() && rel != "/") {
            q = min_quota(q, cgroup_dir_quota(base + rel, v1));
            const size_t slash = rel.find_last_of('/');
            rel = slash == std::string::npos ? std::string() : rel.substr(0, slash);
        }
    };
    if (have_v2) walk(mnt, v2path, false);
    if (have_v1) {  // the cpu controller's hierarchy: <root>/cpu (often a link to cpu,cpuacct)
        walk(mnt + "/cpu", v1path, true);
    }
    return q;
}

int cpulist_count(const char* list) {
    int n = 0;
    const char* p = list;
    while (*p && *p != '\n') {
        char* e = nullptr;
        const long a = strtol(p, &e, 10);
        if (e == p || a < 0) return 0;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            if (e == p + 1 || b < a) return 0;
            p = e;
        }
        n += (int)(b - a + 1);
        if (*p == ',') p++;
        else if (*p && *p != '\n') return 0;
    }
    return n;
}

int cgroup_cpuset_count(const char* root, const char* proc_cgroup) {
    const std::string mnt = root ? root : "/sys/fs/cgroup";
    std::string v2path, v1path;
    bool have_v2 = false, have_v1 = false;
    if (FILE* f = fopen(proc_cgroup ? proc_cgroup : "/proc/self/cgroup", "re")) {
        char line[4096];
        while (fgets(line, sizeof line, f)) {
            line[strcspn(line, "\n")] = 0;
            char* c1 = strchr(line, ':');
            char* c2 = c1 ? strchr(c1 + 1, ':') : nullptr;
            if (!c2) continue;
            const std::string ctrl(c1 + 1, c2);
            if (strncmp(line, "0:", 2) == 0 && ctrl.empty()) {
                v2path = c2 + 1;
                have_v2 = true;
            } else if (("," + ctrl + ",").find(",cpuset,") != std::string::npos) {
                v1path = c2 + 1;
                have_v1 = true;
            }
        }
        fclose(f);
    }
    char buf[4096];
    auto count = [&](const std::string& file) { return read_small(file, buf, sizeof buf) ? cpulist_count(buf) : 0; };
    if (have_v1) {
        const std::string d = mnt + "/cpuset" + (v1path == "/" ? std::string() : v1path);
        int n = count(d + "/cpuset.effective_cpus");
        if (!n) n = count(d + "/cpuset.cpus");
        if (n) return n;
    }
    if (have_v2 && v2path != "/") {
        const int n = count(mnt + v2path + "/cpuset.cpus.effective");
        if (n) return n;
    }
    return count(mnt + "/cpuset.cpus.effective");
}

CpuBudget host_cpu_budget_detail() {
    static const CpuBudget resolved = [] {
        int affinity = 1;
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof set, &set) == 0) affinity = CPU_COUNT(&set);
        long online = sysconf(_SC_NPROCESSORS_ONLN);
        // a container's cpuset narrower than the machine is the scope the mask is compared
        // with: a mask of all of it is the node's shared set, split over the ranks
        const int cpuset = cgroup_cpuset_count(nullptr, nullptr);
        if (cpuset > 0 && (online <= 0 || cpuset < online)) online = cpuset;
        int world = 1;
        if (const char* w = getenv("LOCAL_WORLD_SIZE")) world = std::max(1, atoi(w));
        return cpu_budget_resolve(affinity, online > 0 ? (int)online : affinity, cgroup_cpu_quota_self(nullptr, nullptr),
                                  world);
    }();
    CpuBudget b = resolved;
    const int o = tuning_get(SD_TUNE_HOST_CPU_BUDGET);
    if (o > 0) {
        b.budget = o;
        b.overridden = 1;
    }
    return b;
}

int host_cpu_budget() { return host_cpu_budget_detail().budget; }

// ------------------------------------------------------------------ NUMA placement
namespace {
std::mutex g_numa_mu;
cpu_set_t g_numa_set;              // the preferred CPUs
int g_numa_count = 0;             // CPUs in g_numa_set (0 = no preference)
int g_numa_node = -1;             // the node they belong to
std::atomic<int> g_numa_gen{0};   // bumped when the preference changes
thread_local int t_numa_gen = 0;  // the generation this thread applied
thread_local bool t_placed = false;  // this thread runs on a mask library_thread_place set
thread_local cpu_set_t t_orig_mask;  // its own mask from before that
}  // namespace

int numa_prefer_cpus(const char* list) {
    cpu_set_t allowed, want;
    CPU_ZERO(&allowed);
    CPU_ZERO(&want);
    if (!list || sched_getaffinity(0, sizeof allowed, &allowed) != 0) return 0;
    for (const char* p = list; *p;) {  // "a-b,c,d-e"
        char* end;
        const long a = strtol(p, &end, 10);
        if (end == p) break;
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            p = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
        while (*p == ',' || *p == '\n' || *p == ' ') p++;
    }
    const int n = CPU_COUNT(&want);
    // nothing of the node is ours, or all of our CPUs are on it: nothing to prefer
    if (n == 0 || n == CPU_COUNT(&allowed)) return 0;
    std::lock_guard<std::mutex> g(g_numa_mu);
    if (g_numa_count) return g_numa_count;  // the first context's node stays
    g_numa_set = want;
    g_numa_count = n;
    g_numa_gen.fetch_add(1);
    return n;
}

void numa_note_node(int node) {
    std::lock_guard<std::mutex> g(g_numa_mu);
    if (g_numa_node < 0) g_numa_node = node;
}

int pci_numa_node(const char* bdf) {
    char buf[32];
    if (!bdf || !read_small(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node", buf, sizeof buf)) return -1;
    return atoi(buf);
}

std::string numa_node_cpulist(int node) {
    char buf[1024];
    if (node < 0 || !read_small("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", buf, sizeof buf))
        return "";
    return buf;
}

int numa_placement(int* ncpus, int* node) {
    std::lock_guard<std::mutex> g(g_numa_mu);
    if (ncpus) *ncpus = g_numa_count;
    if (node) *node = g_numa_node;
    return g_numa_count > 0 && tuning_get(SD_TUNE_NUMA_PIN) != 0;
}

void library_thread_place() {
    const int gen = g_numa_gen.load(std::memory_order_acquire);
    if (gen == t_numa_gen) return;
    t_numa_gen = gen;
    cpu_set_t s;
    bool place;
    {
        std::lock_guard<std::mutex> g(g_numa_mu);
        place = g_numa_count > 0 && tuning_get(SD_TUNE_NUMA_PIN) != 0;
        s = g_numa_set;
    }
    if (!place) {
        // "numa_pin" 0 (the default): a thread this library never placed keeps whatever mask
        // its creator gave it; one placed earlier goes back to its own mask from before
        if (t_placed) {
            (void)sched_setaffinity(0, sizeof t_orig_mask, &t_orig_mask);
            t_placed = false;
        }
        return;
    }
    if (!t_placed) {  // remember this thread's own mask, to narrow it and to restore it
        CPU_ZERO(&t_orig_mask);
        if (sched_getaffinity(0, sizeof t_orig_mask, &t_orig_mask) != 0) return;
    }
    cpu_set_t both;
    CPU_AND(&both, &s, &t_orig_mask);  // never widen a thread beyond its own mask
    if (CPU_COUNT(&both) == 0) return;  // none of the node's CPUs is this thread's: leave it
    if (sched_setaffinity(0, sizeof both, &both) == 0) t_placed = true;  // best effort
}

void sd_set_err(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

namespace {
std::atomic<uint64_t> g_split_gen{1};
}  // namespace

uint64_t split_route_tuning_gen() { return g_split_gen.load(std::memory_order_relaxed); }

int split_route_choose(const SplitRoutes& s, uint32_t explore_every) {
    if (s.n[0] == 0) return 0;  // each route once
    if (s.n[1] == 0) return 1;
    const int better = s.rate[0] >= s.rate[1] ? 0 : 1;
    if (explore_every && s.calls % explore_every == explore_every - 1) return 1 - better;  // keep the loser's rate current
    return better;
}

void split_route_record(SplitRoutes& s, int route, double gbps) {
    const int r = route ? 1 : 0;
    if (s.seen[r]++ == 0) return;  // the route's first call: a warm-up, not counted
    s.rate[r] = s.n[r] ? 0.5 * s.rate[r] + 0.5 * gbps : gbps;
    s.n[r]++;
    s.calls++;
}

int tuning_get(int key) { return (key >= 0 && key < SD_TUNE_NKEYS) ? g_tune[key].load(std::memory_order_relaxed) : 0; }

SplitPlan split_plan(uint64_t total, int nranks, int rank) {
    if (nranks < 1 || nranks > 4096 || rank < 0 || rank >= nranks)
        throw sd_failure(SD_ERR_INVALID, "rank / nranks out of range");
    SplitPlan p;
    p.total = total;
    p.nranks = nranks;
    p.rank = rank;
    p.nb = total == 0 ? 1 : (total + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
    if (p.nb >= (1ull << 32)) throw sd_failure(SD_ERR_INVALID, "file too large");
    p.q = (p.nb + (uint64_t)nranks - 1) / (uint64_t)nranks;
    p.b0 = std::min<uint64_t>(p.nb, (uint64_t)rank * p.q);
    p.b1 = std::min<uint64_t>(p.nb, p.b0 + p.q);
    p.off = std::min<uint64_t>(total, p.b0 * SD_CK_BLOCK);
    p.len = std::min<uint64_t>(total, p.b1 * SD_CK_BLOCK) - p.off;
    return p;
}

ExchangePlan exchange_plan(const uint64_t* rows, int R, int me) {
    const size_t row = (size_t)R + SD_EXCHANGE_ROW_EXTRA;
    auto cnt = [&](int src, int dst) { return rows[(size_t)src * row + dst]; };
    ExchangePlan p;
    p.send_cnt.resize(R);
    p.send_off.resize(R);
    p.recv_cnt.resize(R);
    p.recv_off.resize(R);
    for (int r = 0; r < R; r++) {
        uint64_t in = 0, out = 0;
        for (int src = 0; src < R; src++) in += cnt(src, r);
        for (int dst = 0; dst < R; dst++) out += cnt(r, dst);
        if (in > rows[(size_t)r * row + R + 2]) p.fits = false;
        if (out != rows[(size_t)r * row + R + 3]) p.consistent = false;
        if (r + 1 < R && rows[(size_t)r * row + R] + rows[(size_t)r * row + R + 1] > rows[(size_t)(r + 1) * row + R])
            p.ascending = false;
    }
    for (int q = 0; q < R; q++) {
        p.send_cnt[q] = cnt(me, q);
        p.send_off[q] = p.send_total;
        p.send_total += p.send_cnt[q];
        p.recv_cnt[q] = cnt(q, me);
        p.recv_off[q] = p.recv_total;
        p.recv_total += p.recv_cnt[q];
    }
    return p;
}

extern "C" {
const char* sd_cas_last_error(void) { return g_err.c_str(); }
int sd_cas_abi_version(void) { return SD_CAS_ABI_VERSION; }
int sd_host_numa(int out[3]) {
    SD_GUARD_BEGIN
    if (!out) throw sd_failure(SD_ERR_INVALID, "null argument");
    out[0] = numa_placement(&out[1], &out[2]);
    return SD_OK;
    SD_GUARD_END
}

int sd_host_cpu_budget(int out[5]) {
    SD_GUARD_BEGIN
    if (!out) throw sd_failure(SD_ERR_INVALID, "null argument");
    const CpuBudget b = host_cpu_budget_detail();
    out[0] = b.budget;
    out[1] = b.affinity;
    out[2] = b.quota_milli;
    out[3] = b.local_world;
    out[4] = b.overridden;
    return SD_OK;
    SD_GUARD_END
}
int sd_shard_plan(const uint64_t* sizes, size_t n, int nranks, uint64_t* bounds_out) {
    SD_GUARD_BEGIN
    if (!bounds_out || (n && !sizes)) throw sd_failure(SD_ERR_INVALID, "null argument");
    if (nranks < 1 || nranks > 4096) throw sd_failure(SD_ERR_INVALID, "nranks out of range");
    std::vector<uint64_t> prefix(n + 1, 0);  // prefix[i] = cost of files [0, i)
    for (size_t i = 0; i < n; i++) {
        const uint64_t len = sizes[i] <= SD_MINIMUM_FILE_SIZE ? 8 + sizes[i] : SD_SAMPLED_MSG_LEN;
        prefix[i + 1] = prefix[i] + msg_compressions(len);
    }
    const uint64_t total = prefix[n];
    bounds_out[0] = 0;
    for (int r = 1; r < nranks; r++) {  // first file whose cost starts at or past r/R of the total
        const unsigned __int128 target = (unsigned __int128)total * (unsigned)r / (unsigned)nranks;
        const uint64_t t = (uint64_t)target;
        const size_t i = (size_t)(std::lower_bound(prefix.begin(), prefix.end(), t) - prefix.begin());
        bounds_out[r] = std::max<uint64_t>(bounds_out[r - 1], std::min<uint64_t>(i, n));
    }
    bounds_out[nranks] = n;
    return SD_OK;
    SD_GUARD_END
}

int sd_split_range(uint64_t total_len, int nranks, int rank, uint64_t* offset, uint64_t* len, uint64_t* cv_bytes) {
    SD_GUARD_BEGIN
    if (!offset || !len || !cv_bytes) throw sd_failure(SD_ERR_INVALID, "null argument");
    const SplitPlan p = split_plan(total_len, nranks, rank);
    *offset = p.off;
    *len = p.len;
    *cv_bytes = p.cv_bytes();
    return SD_OK;
    SD_GUARD_END
}

int sd_cas_set_tuning(const char* key, int value) {
    SD_GUARD_BEGIN
    if (!key) throw sd_failure(SD_ERR_INVALID, "null key");
    for (int k = 0; k < SD_TUNE_NKEYS; k++)
        if (strcmp(key, TUNE_NAMES[k]) == 0) {
            const int was = g_tune[k].exchange(value, std::memory_order_relaxed);
            if (k == SD_TUNE_NUMA_PIN) g_numa_gen.fetch_add(1);  // threads re-place at their next run
            switch (k) {  // keys the split / CPU-path rates depend on (split_route_tuning_gen)
                case SD_TUNE_READ_THREADS: case SD_TUNE_CHECKSUM_HYBRID_THREADS: case SD_TUNE_HOST_CPU_BUDGET:
                case SD_TUNE_CHECKSUM_SPLIT_BLOCKS: case SD_TUNE_CPU_READ_PIECE_KIB:
                case SD_TUNE_CHECKSUM_STAGE_HOT: case SD_TUNE_NUMA_PIN: case SD_TUNE_HOST_COHASH_THREADS:
                    if (was != value) g_split_gen.fetch_add(1, std::memory_order_relaxed);
                    break;
                default: break;
            }
            return SD_OK;
        }
    throw sd_failure(SD_ERR_INVALID, std::string("unknown tuning key ") + key);
    SD_GUARD_END
}

int sd_cas_get_tuning(const char* key, int* value) {
    SD_GUARD_BEGIN
    if (!key || !value) throw sd_failure(SD_ERR_INVALID, "null argument");
    for (int k = 0; k < SD_TUNE_NKEYS; k++)
        if (strcmp(key, TUNE_NAMES[k]) == 0) {
            *value = g_tune[k].load(std::memory_order_relaxed);
            return SD_OK;
        }
    throw sd_failure(SD_ERR_INVALID, std::string("unknown tuning key ") + key);
    SD_GUARD_END
}
}  // extern "C"

// ------------------------------------------------------------------ planners
sd_extent plan_extent(uint64_t size, uint64_t off) {
    sd_extent e;
    e.size = size;
    const bool whole = size <= SD_MINIMUM_FILE_SIZE;  // cas.rs:27 (<=)
    e.kind = whole ? SD_KIND_WHOLE : SD_KIND_SAMPLED;
    e.msg_len = whole ? (uint32_t)(8 + size) : SD_SAMPLED_MSG_LEN;
    e.msg_offset = off;
    return e;
}

void validate_extent(const sd_extent& e, size_t i) {
    const bool whole = e.size <= SD_MINIMUM_FILE_SIZE;
    const bool len_ok = whole ? e.msg_len >= 8 : e.msg_len == SD_SAMPLED_MSG_LEN;
    if (e.kind != (whole ? SD_KIND_WHOLE : SD_KIND_SAMPLED) || !len_ok)
        throw sd_failure(SD_ERR_INVALID, "extent " + std::to_string(i) + ": kind/msg_len do not match size");
    if (e.msg_offset % 16)
        throw sd_failure(SD_ERR_INVALID, "extent " + std::to_string(i) + ": msg_offset not 16-byte aligned");
}

uint32_t msg_chunks(uint32_t msg_len) { return msg_len == 0 ? 1u : (msg_len + 1023u) / 1024u; }

uint64_t msg_compressions(uint64_t len) {
    const uint64_t C = len == 0 ? 1 : (len + 1023) / 1024;
    const uint64_t last = len - (C - 1) * 1024;
    return (C - 1) * 16 + (last == 0 ? 1 : (last + 63) / 64) + (C - 1);
}

namespace {
// compressions of aligned chunk pair (c0, c0 + 1) holding glen (1..2048) message bytes
uint32_t pair_compressions(uint32_t glen) {
    const uint32_t l0 = std::min<uint32_t>(glen, 1024), l1 = glen - l0;
    return (l0 + 63) / 64 + (l1 ? (l1 + 63) / 64 + 1 : 0);
}
bool items_message(const sd_extent& e) { return e.kind == SD_KIND_WHOLE && e.msg_len <= SD_WHOLE_ITEMS_MAX; }
}  // namespace

// Work lists for the whole-file messages (msg_len <= SD_WHOLE_ITEMS_MAX) of ext[0, n):
//  * full-pair items in file (= staged address) order, so the waves sweep the staged
//    buffer front to back as the sampled kernel does;
//  * tail items counting-sorted by compressions, descending (equal trip counts per wave);
//  * merge8 items -- pass A over aligned groups of <= 8 pair nodes (the whole tree when a
//    message has <= 8 nodes), pass B over the pass-A nodes of messages with more than 8.
// CV slots and merge items follow the multi-pair messages sorted by pair count, descending,
// so the lanes of a merge wave have nearly equal trip counts.
void plan_whole_items(WholePlan& p, const sd_extent* ext, size_t n) {
    p.full.clear();
    p.tail.clear();
    p.merge_a.clear();
    p.merge_b.clear();
    constexpr uint32_t PMAX = (SD_WHOLE_ITEMS_MAX + 2047) / 2048;  // 51 pairs
    auto pairs = [&](size_t i) { return (msg_chunks(ext[i].msg_len) + 1) / 2; };
    // multi-pair messages (>= 3 chunks) by pair count, descending: counting sort
    std::vector<uint32_t> start(PMAX + 2, 0);
    for (size_t i = 0; i < n; i++)
        if (items_message(ext[i]) && msg_chunks(ext[i].msg_len) >= 3) start[PMAX - pairs(i)]++;
    uint32_t acc = 0;
    for (auto& s : start) {
        const uint32_t t = s;
        s = acc;
        acc += t;
    }
    std::vector<uint32_t> sorted(acc);
    for (size_t i = 0; i < n; i++)
        if (items_message(ext[i]) && msg_chunks(ext[i].msg_len) >= 3) sorted[start[PMAX - pairs(i)]++] = (uint32_t)i;
    std::vector<uint32_t> slot(n, 0);  // first CV slot of each multi-pair message
    uint32_t cv = 0;
    for (uint32_t f : sorted) {
        slot[f] = cv;
        cv += pairs(f);
    }
    std::vector<uint8_t> tail_cost;
    for (size_t file = 0; file < n; file++) {
        const sd_extent& e = ext[file];
        if (!items_message(e)) continue;
        const uint32_t C = msg_chunks(e.msg_len), P = (C + 1) / 2;
        const bool multi = C >= 3;
        for (uint32_t j = 0; j < P; j++) {
            const uint64_t off = e.msg_offset + 2048ull * j;
            const uint32_t glen = std::min<uint32_t>(2048, e.msg_len - 2048 * j);
            const uint32_t lo = (uint32_t)off, hi = (uint32_t)(off >> 32);
            if (multi && glen == 2048) {
                p.full.push_back({lo, hi, slot[file] + j, 2 * j});
            } else {
                const uint32_t w = glen | ((2 * j) << 12) | (multi ? 0u : 0x80000000u);
                p.tail.push_back({lo, hi, multi ? slot[file] + j : (uint32_t)file, w});
                tail_cost.push_back((uint8_t)pair_compressions(glen));
            }
        }
    }
    {  // stable counting sort of the tail items by cost, descending (cost 1..33)
        std::vector<uint32_t> st(35, 0);
        for (uint8_t c : tail_cost) st[34 - c]++;
        uint32_t a = 0;
        for (auto& s : st) {
            const uint32_t t = s;
            s = a;
            a += t;
        }
        std::vector<sd_u32x4> out(p.tail.size());
        for (size_t i = 0; i < p.tail.size(); i++) out[st[34 - tail_cost[i]]++] = p.tail[i];
        p.tail.swap(out);
    }
    uint32_t cv2 = 0;
    for (uint32_t file : sorted) {
        const uint32_t P = pairs(file);
        if (P <= 8) {
            p.merge_a.push_back({slot[file], P | 0x80000000u, file, 0});
            continue;
        }
        const uint32_t G = (P + 7) / 8;  // <= 7 for messages of <= 102408 B
        for (uint32_t a = 0; a < G; a++)
            p.merge_a.push_back({slot[file] + 8 * a, std::min<uint32_t>(8, P - 8 * a), cv2 + a, 0});
        p.merge_b.push_back({cv2, G | 0x80000000u, file, 0});
        cv2 += G;
    }
    p.n_cv = cv;
    p.n_cv2 = cv2;
}

// Checksum batch over byte ranges: one leaf workgroup per 1 MiB block of each message;
// reduce passes of groups of 256 CVs per workgroup until every message has its root.
void plan_checksum(CkPlan& p, const uint64_t* offsets, const uint64_t* lens, size_t n) {
    if (n >= (1ull << 31)) throw sd_failure(SD_ERR_INVALID, "batch too large");
    p.files.resize(n);
    p.wg_map.clear();
    p.passes.clear();
    p.total_bytes = p.compressions = p.blocks = 0;
    std::vector<uint64_t> level_n(n), base(n, 0);
    uint64_t cv0 = 0;
    for (size_t i = 0; i < n; i++) {
        if (offsets[i] % 16)
            throw sd_failure(SD_ERR_INVALID, "checksum range " + std::to_string(i) + " not 16-byte aligned");
        const uint64_t nb = lens[i] == 0 ? 1 : (lens[i] + SD_CK_BLOCK - 1) / SD_CK_BLOCK;
        if (nb >= (1ull << 32)) throw sd_failure(SD_ERR_INVALID, "file too large");
        p.files[i] = ck_file{offsets[i], lens[i], nb > 1 ? cv0 : 0};
        for (uint64_t k = 0; k < nb; k++) p.wg_map.push_back({(uint32_t)i, (uint32_t)k});
        base[i] = p.files[i].cv_base;
        if (nb > 1) cv0 += nb;
        level_n[i] = nb;
        p.total_bytes += lens[i];
        p.compressions += msg_compressions(lens[i]);
        p.blocks += nb;
    }
    p.lvl_cap[0] = cv0;
    p.lvl_cap[1] = 0;
    int src = 0;
    for (;;) {
        std::vector<ck_reduce_wg> wgs;
        uint64_t dst_total = 0;
        std::vector<uint64_t> nbase(n, 0);
        for (size_t i = 0; i < n; i++) {
            const uint64_t cnt = level_n[i];
            if (cnt <= 1) continue;
            const uint64_t groups = (cnt + 255) / 256;
            nbase[i] = dst_total;
            for (uint64_t g = 0; g < groups; g++) {
                ck_reduce_wg w{};
                w.src_base = base[i] + g * 256;
                w.dst_index = dst_total + g;
                w.count = (uint32_t)std::min<uint64_t>(256, cnt - g * 256);
                w.file = (uint32_t)i;
                w.is_root = groups == 1;
                wgs.push_back(w);
            }
            dst_total += groups == 1 ? 0 : groups;
            level_n[i] = groups == 1 ? 1 : groups;
        }
        if (wgs.empty()) break;
        p.passes.push_back(std::move(wgs));
        p.lvl_cap[1 - src] = std::max<uint64_t>(p.lvl_cap[1 - src], dst_total);
        base = nbase;
        src = 1 - src;
    }
}

// ------------------------------------------------------------------ file reading
namespace {
// set when this thread took (or, where unshare is refused or under TSan, was meant to take)
// a private fd table: the rule is about the thread's role, so it holds in every build
thread_local bool t_private_fds = false;
}  // namespace

bool on_private_fd_table() { return t_private_fds; }

void hip_thread_check(const char* what) {
    if (t_private_fds)
        throw sd_failure(SD_ERR_INTERNAL, std::string("HIP call on a private-fd-table worker thread (its device "
                                                      "descriptors are closed): ") + what);
}

void private_fd_table() {
    t_private_fds = true;
#if defined(__SANITIZE_THREAD__)
    // ThreadSanitizer tracks descriptors by number across threads: fd 3 of two private
    // tables would read as one descriptor raced on.  The TSan build keeps the shared table.
    return;
#endif
    if (unshare(CLONE_FILES) != 0) return;  // not permitted here: keep the shared table
#ifdef SYS_close_range
    if (syscall(SYS_close_range, 3u, ~0u, 0u) == 0) return;
#endif
    const long hi = sysconf(_SC_OPEN_MAX);
    for (long fd = 3; fd < (hi > 0 ? hi : 1024); fd++) close((int)fd);
}

namespace {

// read exactly n bytes at off (read_exact after a seek); 0, SD_FILE_SHORT_READ or io_status
int32_t pread_exact(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
    while (n) {
        const ssize_t r = pread(fd, dst, n, (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return io_status(errno);
        }
        if (r == 0) return SD_FILE_SHORT_READ;
        dst += r;
        n -= (uint64_t)r;
        off += (uint64_t)r;
    }
    return SD_FILE_OK;
}

// one read() call, retried on EINTR (tokio's blocking read is uninterruptible)
ssize_t read_once(int fd, uint8_t* dst, uint64_t n) {
    for (;;) {
        const ssize_t r = read(fd, dst, n);
        if (r < 0 && errno == EINTR) continue;
        return r;
    }
}

struct Fd {
    int fd;
    ~Fd() {
        if (fd >= 0) close(fd);
    }
};

}  // namespace

int64_t pread_full(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
    uint64_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, dst + got, n - got, (off_t)(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            return -(int64_t)errno;
        }
        if (r == 0) break;
        got += (uint64_t)r;
    }
    return (int64_t)got;
}

int64_t pread_stream(int fd, uint8_t* dst, uint64_t n, uint64_t off) {
    constexpr uint64_t HOT = 256 << 10;
    thread_local std::unique_ptr<uint8_t[]> hot_buf(new uint8_t[HOT + 64]);
    uint8_t* hot = reinterpret_cast<uint8_t*>(sd_align_up(reinterpret_cast<uintptr_t>(hot_buf.get()), 64));
    if (reinterpret_cast<uintptr_t>(dst) % 16) return pread_full(fd, dst, n, off);  // (never, for windows)
    uint64_t got = 0;
    while (got < n) {
        const uint64_t want = std::min(HOT, n - got);
        const int64_t r = pread_full(fd, hot, want, off + got);
        if (r < 0) return r;
        const uint64_t body = (uint64_t)r & ~uint64_t(15);
        for (uint64_t o = 0; o < body; o += 16)
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + got + o), _mm_load_si128(reinterpret_cast<const __m128i*>(hot + o)));
        memcpy(dst + got + body, hot + body, (uint64_t)r - body);
        got += (uint64_t)r;
        if ((uint64_t)r < want) break;  // EOF
    }
    _mm_sfence();  // the streamed lines are globally visible before the caller hands dst on
    return (int64_t)got;
}

int32_t stage_one(const char* path, sd_extent& e, uint8_t* staged, std::vector<uint8_t>* capture) {
    uint8_t* dst = staged + e.msg_offset;
    const uint64_t size = e.size;
    for (int i = 0; i < 8; i++) dst[i] = (uint8_t)(size >> (8 * i));  // cas.rs:25 le64
    const uint64_t padded = sd_align_up(e.msg_len, SD_STAGE_PAD);   // the planned extent's end
    Fd f{open(path, O_RDONLY | O_CLOEXEC)};
    if (f.fd < 0) return io_status(errno);
    if (e.kind == SD_KIND_WHOLE) {  // cas.rs:29 fs::read: read_to_end
        const uint64_t room = e.msg_len - 8;
        uint64_t got = 0;
        {
            // A seekable file in one call: the planned room plus a probe byte.  Exactly the
            // room back -- the file holds what its stat said, the common case -- is
            // read_to_end's outcome without its final zero-length read; a count past the room
            // means the file holds more than planned.  A count short of the room (a file that
            // shrank, or a filesystem that returns short counts: FUSE direct_io, network
            // mounts) continues in the read loop below until a read returns 0, as read_to_end
            // does.  A pipe or character device fails with ESPIPE having consumed nothing,
            // and takes the read loop from the start.
            uint8_t probe;
            struct iovec iov[2] = {{dst + 8, (size_t)room}, {&probe, 1}};
            ssize_t r;
            do {
                r = preadv(f.fd, iov, 2, 0);
            } while (r < 0 && errno == EINTR);
            if (r >= 0) {
                if ((uint64_t)r > room) return SD_FILE_CHANGED;  // the caller re-reads it whole
                if ((uint64_t)r == room) {
                    memset(dst + e.msg_len, 0, padded - e.msg_len);
                    return SD_FILE_OK;
                }
                if (lseek(f.fd, (off_t)r, SEEK_SET) < 0) return io_status(errno);
                got = (uint64_t)r;
            } else if (errno != ESPIPE) {
                return io_status(errno);
            }
        }
        for (;;) {
            if (got == room) {  // planned room full: does the file hold more?
                uint8_t probe;
                const ssize_t r = read_once(f.fd, &probe, 1);
                if (r < 0) return io_status(errno);
                if (r > 0) {
                    struct stat st;
                    if (!capture || (fstat(f.fd, &st) == 0 && S_ISREG(st.st_mode))) return SD_FILE_CHANGED;
                    // a pipe or device: what was read is gone from it -- keep every byte
                    capture->assign(dst + 8, dst + 8 + room);
                    capture->push_back(probe);
                    uint8_t buf[1 << 16];
                    for (;;) {
                        const ssize_t k = read_once(f.fd, buf, sizeof buf);
                        if (k < 0) {
                            const int err = errno;
                            capture->clear();
                            return io_status(err);
                        }
                        if (k == 0) break;
                        capture->insert(capture->end(), buf, buf + k);
                    }
                    return SD_FILE_CHANGED;
                }
                break;
            }
            const ssize_t r = read_once(f.fd, dst + 8 + got, room - got);
            if (r < 0) return io_status(errno);
            if (r == 0) break;
            got += (uint64_t)r;
        }
        e.msg_len = (uint32_t)(8 + got);
        memset(dst + e.msg_len, 0, padded - e.msg_len);
        return SD_FILE_OK;
    }
    // cas.rs:31-58: header, 4 samples at 8192 + k * seek_jump, footer at End(-8192)
    memset(dst + e.msg_len, 0, padded - e.msg_len);
    const uint64_t H = SD_HEADER_OR_FOOTER_SIZE, S = SD_SAMPLE_SIZE;
    const uint64_t jump = (size - 2 * H) / SD_SAMPLE_COUNT;
    uint8_t* p = dst + 8;
    // :35-38 the header, and the first sample that follows it on disk (current_pos = 8192),
    // in one read: the two are contiguous, and either falling short is the same UnexpectedEof
    int32_t st = pread_exact(f.fd, p, H + S, 0);
    p += H + S;
    uint64_t current_pos = H + jump;
    for (int k = 1; k < (int)SD_SAMPLE_COUNT && st == SD_FILE_OK; k++) {  // :42-51
        st = pread_exact(f.fd, p, S, current_pos);
        p += S;
        current_pos += jump;
    }
    if (st != SD_FILE_OK) return st;
    // :54-58 the footer at SeekFrom::End(-8192).  In the common case the file is exactly
    // `size` bytes long: one pread of 8192 + 1 bytes at size - 8192 then returns exactly 8192
    // -- the footer, and proof that the end is at `size` (the extra byte lands in the
    // message's zero padding and is cleared).  Anything else (a file longer or shorter than
    // `size`, an interrupted read) seeks to the real end as the reference does.
    ssize_t r;
    do {
        r = pread(f.fd, p, H + 1, (off_t)(size - H));
    } while (r < 0 && errno == EINTR);
    if (r == (ssize_t)H) return SD_FILE_OK;
    p[H] = 0;  // the probe byte, if the file was longer
    const off_t end = lseek(f.fd, -(off_t)H, SEEK_END);  // :54-55 SeekFrom::End(-8192)
    if (end < 0) return io_status(errno);
    return pread_exact(f.fd, p, H, (uint64_t)end);  // :56-58
}

void MsgSource::set_prefix_le64(uint64_t v) {
    for (int i = 0; i < 8; i++) prefix_[i] = (uint8_t)(v >> (8 * i));
    prefix_len_ = 8;
    prefix_pos_ = 0;
}

uint64_t MsgSource::read(uint8_t* dst, uint64_t n) {
    const uint64_t got = read_impl(dst, n);
    if (has_eof_hint_ && !done && !err && got == n && file_pos_ == eof_hint_ && pend_len_ == 0) {
        uint8_t probe;
        ssize_t r;
        do r = pread(fd_, &probe, 1, (off_t)file_pos_);
        while (r < 0 && errno == EINTR);
        if (r == 0) done = true;  // the next read would return 0: the message ends here
    }
    return got;
}

uint64_t MsgSource::read_impl(uint8_t* dst, uint64_t n) {
    uint64_t got = 0;
    while (got < n && prefix_pos_ < prefix_len_) dst[got++] = prefix_[prefix_pos_++];
    if (pend_len_ && got < n) {
        const uint64_t k = std::min(pend_len_, n - got);
        memcpy(dst + got, pend_, k);
        pend_ += k;
        pend_len_ -= k;
        got += k;
    }
    if (mem_only_) {
        if (pend_len_ == 0 && prefix_pos_ == prefix_len_) done = true;
        return got;
    }
    if (done || err) return got;
    if (pool_ && mode_ == CHECKSUM_READS && got < n) return got + read_parallel(dst + got, n - got);
    if (mode_ == READ_TO_EOF) {
        const uint64_t got0 = got;  // prefix and pending bytes are not new file bytes
        while (got < n) {
            const ssize_t r = read_once(fd_, dst + got, n - got);
            if (r < 0) {
                err = errno;
                break;
            }
            if (r == 0) {
                done = true;
                break;
            }
            got += (uint64_t)r;
        }
        file_pos_ += got - got0;
        return got;
    }
    const uint64_t got0 = got;
    while (got < n) {  // hash.rs:14-20
        const uint64_t want = std::min<uint64_t>(CHECKSUM_READ, n - got);
        const ssize_t r = read_once(fd_, dst + got, want);
        if (r < 0) {
            err = errno;
            break;
        }
        got += (uint64_t)r;
        if ((uint64_t)r != CHECKSUM_READ) {  // :17-19 a short read ends the file
            done = true;
            break;
        }
    }
    file_pos_ += got - got0;
    return got;
}

uint64_t MsgSource::read_parallel(uint8_t* dst, uint64_t n) {
    const uint64_t pieces = (n + CHECKSUM_READ - 1) / CHECKSUM_READ;
    std::vector<int64_t> r(pieces, 0);
    pool_->run(
        pieces,
        [&](size_t k) {
            const uint64_t len = std::min<uint64_t>(CHECKSUM_READ, n - k * CHECKSUM_READ);
            uint8_t* d = dst + k * CHECKSUM_READ;
            const uint64_t at = file_pos_ + k * CHECKSUM_READ;
            r[k] = par_stream_ ? pread_stream(fd_, d, len, at) : pread_full(fd_, d, len, at);
        },
        par_threads_);
    uint64_t got = 0;
    for (uint64_t k = 0; k < pieces; k++) {
        if (r[k] < 0) {
            err = (int)-r[k];
            break;
        }
        got += (uint64_t)r[k];
        if ((uint64_t)r[k] != CHECKSUM_READ) {  // the first short piece is EOF
            done = true;
            break;
        }
    }
    file_pos_ += got;
    return got;
}

size_t shared_range_pick(const uint64_t* lens, size_t n, uint64_t min_len, int host_threads, double gpu_gbps,
                         double thread_gbps) {
    double all = 0;
    for (size_t q = 0; q < n; q++) all += (double)lens[q];
    const double meet = all * gpu_gbps / (gpu_gbps + thread_gbps * std::max(0, host_threads));
    size_t pick = SIZE_MAX;
    double best = 0, pos = 0;
    for (size_t q = 0; q < n; pos += (double)lens[q], q++) {
        if (lens[q] < min_len) continue;
        const double lo = pos, hi = pos + (double)lens[q];
        const double dist = meet < lo ? lo - meet : meet > hi ? meet - hi : 0;
        if (pick == SIZE_MAX || dist < best) {
            pick = q;
            best = dist;
        }
    }
    return pick;
}
