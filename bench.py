"""bench.py -- cas_id files/s (+ checksum GB/s) on 1..8 MI355X, one process per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json configs[4], weak-scaled): a 10 M-file synthetic library with the
configs[0] mixture (60 % of files <= 100 KiB hashed whole, 40 % sampled), sharded by file
index: each GPU owns ``--files-per-gpu`` (default 1 250 000 = 10 M / 8) files, so N = 8 is
the full 10 M-file library.  One step = hash every file of the shard (sampled kernel +
whole-file kernels) + the dedup step through the C ABI (sd_cas_dedup_mgpu: partition by
cas_id prefix, RCCL all-gather of the count matrix + grouped send/recv of the records,
sort + group, Object owners).  Inputs are resident in HBM before timing (generated on
device from the counter-based generator); PCIe-inclusive rates are reported beside
`value` ("with_h2d"), never as it.

After the timed steps: configs[3] (full-file checksums of 16 x 4 GiB files, then its mixed 2..8 GiB variant) on every
rank as `checksum`; on rank 0 at N = 1 the configs[1]/[2] kernel legs, the with-H2D legs
(cas_ids and checksums from pinned host memory), the file-backed legs (cas_ids and
checksums from tmpfs beside the reference's read schedule on the CPU), single-call
latency percentiles of the GPU-coalesced and CPU paths, and the CPU baseline
(oracle/sd_oracle_simd.c, the C restatement of cas.rs + blake3) on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
# The int32 VALU roof of BLAKE3.  Its G function is 2x v_add3_u32 + 2x v_add_u32 + 4x
# v_xor_b32 + 4x v_alignbit_b32 (rotr16 as two v_xor_b32_sdwa).  Measured per op and per mix
# (scripts/valu_probe7.hip, profiles/r3/r3c_valu_probe7.txt; 8 waves/SIMD): the 2-source
# ops and -- the control -- v_fma_f32 and v_bitop3_b32 issue at the SIMD-32 full rate (68-70 T
# at 2.38 GHz), while v_add3 / v_alignbit / v_perm / SDWA / v_xad / v_mad_u32_u24 / v_addc
# issue at about half of it (37.4 T), and fp32 ops overlap those slow integer ops completely
# (v_fma_f32 : v_add3 1:1 runs at the full rate) -- the slow integer ops are a separate, half-
# rate datapath, not a harness limit.  BLAKE3's G mix written in asm, registers only, issues
# at 39.5 T = 64.7 lane-ops/clk/CU (the in-library k_valu_peak is the same block: 39.3-39.5 T,
# profiles/r3/r3d_valu_peak.txt).  So the roof is 64 lane-ops/clk/CU x 256 CU x 2.4 GHz:
N_CUS = 256
VALU_PEAK_TOPS = N_CUS * 64 * 2.4e9 / 1e12
# The G mix's measured issue rate per clock (valu_probe7, 8 waves/SIMD: 39.51 T at 2386 MHz =
# 64.7 lane-ops/clk/CU): the denominator of the roofline's frac at the measured clock.
G_MIX_LANE_OPS_PER_CLK = 64.7
# The guide's full VALU rate (MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 op in 2
# cycles): 256 x 128 x 2.4 GHz = 78.6 T lane-ops/s -- reported as frac_full_rate.
VALU_FULL_RATE_TOPS = 256 * 128 * 2.4e9 / 1e12
PEAK_BASIS = ("BLAKE3 G-mix issue ceiling: 256 CU x 64 lane-ops/clk x 2.4 GHz = 39.3 T.  Measured (scripts/valu_probe7.hip, "
              "profiles/r3/r3c_valu_probe7.txt, 8 waves/SIMD): v_xor/v_add and the control v_fma_f32 issue at the full rate "
              "(68-70 T), v_add3/v_alignbit/SDWA at about half (37.4 T), fp32 ops overlap them fully; the kernels' G mix in "
              "asm from registers reaches 39.5 T (64.7 lane-ops/clk/CU) -- measured_valu_peak is that block in-library. "
              "frac_full_rate is against the SIMD-32 full rate, 256 CU x 128 lane-ops/clk x 2.4 GHz = 78.6 T")
SAMPLED_MSG = 57352
S_LANES_PER_FILE = 7  # k_cas_sampled_lanes: one 256-lane grid slot per 8-chunk group (cas_kernels.hip)
SAMPLED_KERNELS = ["k_cas_sampled_lanes", "k_cas_sampled_merge"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# True when the process group is up (world > 1, or --force-dist at any world size): every
# collective below is gated on it, not on the world size, so a one-rank rehearsal runs the
# same statements an 8-rank node does
DIST = False


def rccl_libs() -> dict:
    """Which RCCL this process uses (VERDICT r3 "two RCCL libraries"): every librccl file
    mapped into the process (/proc/self/maps), the one libsdcas's communicators are bound
    to with the version it reports (sd_comm_rccl_info), and torch's RCCL version."""
    from spacedrive_amd import _native
    mapped = set()
    try:
        for line in open("/proc/self/maps"):
            parts = line.split()
            if len(parts) >= 6 and "librccl" in os.path.basename(parts[-1]):
                mapped.add(os.path.realpath(parts[-1]))
    except OSError:
        pass
    try:
        v = torch.cuda.nccl.version()
        torch_v = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 -- a diagnostic
        torch_v = None
    info = _native.rccl_info()
    return {"mapped": sorted(mapped), "sdcas_comm": info, "torch_nccl_version": torch_v,
            "one_rccl": len(mapped) == 1 and info["path"] in mapped,
            "note": "librccl.so.1 is one soname: torch loads its own copy first (ProcessGroupNCCL), and libsdcas's "
                    "NEEDED librccl.so.1 binds to that same copy -- one RCCL serves both communicators"}


def parity(files: int, mismatches: int, what: str, **kw) -> dict:
    """A leg's oracle check (outside its timed region); a mismatch fails the run."""
    res = dict(files=int(files), mismatches=int(mismatches), oracle=what, **kw)
    assert mismatches == 0, res
    return res


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--files-per-gpu", type=int, default=1_250_000)
    p.add_argument("--checksum-gib", type=int, default=64, help="configs[3] size per GPU; 0 = skip")
    p.add_argument("--checksum-steps", type=int, default=5)
    p.add_argument("--split-gib", type=int, default=32,
                   help="one file of this many GiB (+12345 B) split over the ranks; 0 = skip")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target seconds per CPU-baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (rehearsal)")
    p.add_argument("--force-dist", action="store_true",
                   help="initialise the process group even at world size 1 and take the N > 1 code path "
                        "(every collective, the per-rank legs, no N = 1 side legs): a one-GPU rehearsal of the "
                        "8-GPU run, launched with torch.distributed.run --nproc-per-node 1")
    p.add_argument("--dedup", default=None, choices=["rccl", "torch"],
                   help="exchange transport: rccl = sd_cas_dedup_mgpu (C ABI; default with nccl), torch = "
                        "torch.distributed all_to_all (default with gloo)")
    p.add_argument("--share-gpu", action="store_true", help="map every rank onto the visible GPUs (rehearsal)")
    p.add_argument("--config-files", type=int, default=1_000_000,
                   help="N=1 only: files of the configs[1] (small) and configs[2] (sampled) kernel legs; 0 = skip")
    p.add_argument("--config-reps", type=int, default=20)
    p.add_argument("--warm-ms", type=float, default=150.0,
                   help="side legs: run a kernel this long before timing it (the clock ramps up from idle: "
                        "profiles/r2/r2b_whole_ab.json)")
    p.add_argument("--file-backed-files", type=int, default=200_000,
                   help="N=1 only: time the drop-in from files on disk (pread stager + sd_cas_ids) on this many "
                        "files of the shard, beside the reference's read schedule on the CPU; 0 = skip")
    p.add_argument("--identifier-files", type=int, default=100_000,
                   help="N=1 only: the identifier job (100-row steps) over this many of the file-backed files, "
                        "look-ahead GPU hashing vs per-step CPU path; 0 = skip")
    p.add_argument("--host-staged-files", type=int, default=300_000,
                   help="with-H2D leg, sd_cas_ids over this many files from pinned host memory on every rank "
                        "(at most 150 000 per rank at N > 1); 0 = skip")
    p.add_argument("--host-checksum-gib", type=int, default=4,
                   help="N=1 only: with-H2D checksum leg, sd_checksums over this many GiB of pinned memory; 0 = skip")
    p.add_argument("--file-checksum-mib", type=int, default=8192,
                   help="N=1 only: file-backed checksum leg on tmpfs (MiB, 256 MiB files); 0 = skip")
    p.add_argument("--latency-calls", type=int, default=400, help="N=1 only: single-call latency legs; 0 = skip")
    p.add_argument("--no-extras", action="store_true", help="skip every N=1 side leg (profiling passes)")
    p.add_argument("--no-overlap", action="store_true",
                   help="report the serial steps (hash, then dedup, one stream) as the value instead of the "
                        "pipelined ones (batch k's dedup beside batch k+1's hashing)")
    p.add_argument("--host-cpu-budget", type=int, default=0,
                   help="cap the library's host threads (and the oracle checks') at this many, as the tuning key "
                        "host_cpu_budget does: 2 rehearses one rank's share of an 8-GPU node's 16-CPU quota on a "
                        "one-GPU box; 0 = resolved from the affinity mask, quota and LOCAL_WORLD_SIZE")
    p.add_argument("--oracle-live", action="store_true",
                   help="recompute the multi-GiB oracle checks (configs[3] files, the mixed file, the split file) "
                        "on this host instead of comparing with tests/golden/bench_checksums.json (the same oracle's "
                        "output, committed)")
    p.add_argument("--full-out", default=os.path.join("gpurun_out", "bench_full.json"),
                   help="rank 0 writes the full record here (stdout carries the compact line); '' = skip")
    return p.parse_args(argv)


# ------------------------------------------------------------------ launcher (--gpus N)
def launch_mode(gpus: int, env) -> str:
    """How this process runs the requested --gpus:
    "rank"      -- started by torch.distributed.run (WORLD_SIZE set): one rank of `gpus`;
    "spawn"     -- WORLD_SIZE unset and gpus > 1: start the ranks as a child launcher;
    "inprocess" -- WORLD_SIZE unset and gpus == 1: run here, as before.
    Raises SystemExit when WORLD_SIZE disagrees with --gpus (a silent one-GPU run labelled
    as N would be worse than none)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} (the launcher's rank count) but --gpus {gpus}: "
                             f"launch with --nproc-per-node {gpus}, or pass --gpus {ws}")
        return "rank"
    return "spawn" if gpus > 1 else "inprocess"


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(gpus: int, argv: list, port: int) -> list:
    """The child launch of `bench.py --gpus N` without WORLD_SIZE: torch.distributed.run with
    N local ranks on 127.0.0.1, the same arguments (the driver's own N > 1 command line)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def spawn_ranks(gpus: int, argv: list) -> int:
    """Runs the N ranks as a child process group (subprocess, never exec: this process has
    made no HIP call and makes none), relays rank 0's JSON line to stdout and everything else
    the child prints on stdout to stderr, and returns the child's exit code (1 if it exited 0
    without a line)."""
    import signal
    import subprocess
    cmd = launcher_cmd(gpus, argv, free_port())
    log("bench.py: --gpus %d without WORLD_SIZE: launching %s" % (gpus, " ".join(cmd)))
    env = dict(os.environ, SD_BENCH_SPAWNED="1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env)

    def forward(sig, _frame):  # a timeout's SIGTERM reaches the ranks through their launcher
        try:
            proc.send_signal(sig)
        except OSError:
            pass
    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    lines = []
    try:
        for line in proc.stdout:
            if line.lstrip().startswith("{"):
                lines.append(line.strip())
            else:
                sys.stderr.write(line)
                sys.stderr.flush()
        rc = proc.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    if lines:
        print(lines[-1], flush=True)
    if rc == 0 and not lines:
        log("bench.py: the ranks exited 0 without a JSON line")
        return 1
    return rc


# ------------------------------------------------------------------ PMC traffic lookup
def pmc_traffic(kernel: str, grid: int):
    """HBM bytes per launch of `kernel` at launch shape `grid` (work-items) from the
    committed rocprofv3 PMC summary (profiles/pmc_summary.json), or None when no pass
    measured that launch shape."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
        for e in d["kernels"].get(kernel, []):
            if int(e["grid"]) == int(grid):
                return {"bytes": e["hbm_bytes_per_launch"], "tag": d.get("tag"), "grid": grid,
                        "fetch_factor": e["fetch_factor"]}
    except (OSError, KeyError, ValueError, TypeError, AttributeError):
        pass
    return None


def sampled_grids(n_sampled: int) -> list:
    """work-items of the two sampled launches: lanes (7 per file), merge (1 per file)"""
    return [(n_sampled * S_LANES_PER_FILE + 255) // 256 * 256, (n_sampled + 255) // 256 * 256]


def pmc_traffic_sum(kernels, grids):
    """pmc_traffic summed over launches that run as one unit; None unless every one is measured"""
    parts = [pmc_traffic(k, g) for k, g in zip(kernels, grids)]
    if not all(parts):
        return None
    return {"bytes": sum(p["bytes"] for p in parts), "tag": parts[0]["tag"], "grid": list(grids),
            "fetch_factor": parts[0]["fetch_factor"], "per_kernel": {k: p["bytes"] for k, p in zip(kernels, parts)}}


def pmc_issue_rate(kernel: str, grid: int):
    """VALU lane-ops per clock per CU of `kernel` at launch shape `grid` from the committed
    PMC summary: SQ_INSTS_VALU x 64 lanes / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs), against the
    G mix's measured ceiling of G_MIX_LANE_OPS_PER_CLK -- a per-clock figure, so the board's
    clock drops out.  GRBM_GUI_ACTIVE also counts busy cycles around the launch, so the rate
    is a slight underestimate.  None when no pass measured that shape."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
        for e in d["kernels"].get(kernel, []):
            c = e.get("counters", {})
            if int(e["grid"]) == int(grid) and c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
                r = c["SQ_INSTS_VALU"] * 64 / (c["GRBM_GUI_ACTIVE"] / 8 * N_CUS)
                return {"lane_ops_per_clk_cu": r, "ceiling": G_MIX_LANE_OPS_PER_CLK,
                        "frac": r / G_MIX_LANE_OPS_PER_CLK, "kernel": kernel, "grid": grid, "tag": d.get("tag"),
                        "source": "profiles/pmc_summary.json (rocprofv3 --pmc SQ_INSTS_VALU ... GRBM_GUI_ACTIVE)"}
    except (OSError, KeyError, ValueError, TypeError, AttributeError, ZeroDivisionError):
        pass
    return None


def ck_leaf_grid(blocks: int) -> int:
    """work-items of a k_ck_leaf launch over `blocks` 1 MiB blocks: two blocks of 256 lanes per
    workgroup (cas_kernels.hip CK_WG_BLOCKS)"""
    return (blocks + 1) // 2 * 512


def whole_grid(batch) -> int:
    return ((batch.full_items + 255) // 256 + (batch.tail_items + 255) // 256) * 256


class ClockSampler:
    """This device's shader clock and board power from its hwmon (sysfs; the host's other
    cards are listed too, so the device is matched by PCI address), sampled every 10 ms on a
    host thread while the timed steps run: the clock the kernels actually ran at, so the
    roofline can say how much of the gap to the nominal 2.4 GHz ceiling is the clock
    (the board's power limit) and how much is issue.  None when unreadable."""

    def __init__(self, device: int):
        import glob
        self.dir, self.rows, self.stop, self.t = None, [], None, None
        try:
            import ctypes
            buf = ctypes.create_string_buffer(64)
            if ctypes.CDLL("libamdhip64.so").hipDeviceGetPCIBusId(buf, 64, int(device)) != 0:
                return
            want = buf.value.decode().lower()
            for h in glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*"):
                pci = os.path.basename(os.path.realpath(os.path.join(h, "..", ".."))).lower()
                if pci == want and os.path.exists(os.path.join(h, "freq1_input")):
                    self.dir = h
        except Exception:  # noqa: BLE001 -- a diagnostic: absent is fine
            self.dir = None

    def _read(self, key):
        try:
            with open(os.path.join(self.dir, key)) as f:
                return int(f.read().strip())
        except (OSError, ValueError):
            return None

    def _run(self):
        while not self.stop.is_set():
            self.rows.append((self._read("freq1_input"), self._read("power1_input")))
            self.stop.wait(0.01)

    def start(self):
        import threading
        if self.dir:
            self.stop = threading.Event()
            self.t = threading.Thread(target=self._run, daemon=True)
            self.t.start()
        return self

    def result(self):
        if not self.dir or self.t is None:
            return None
        self.stop.set()
        self.t.join()
        f = [r[0] for r in self.rows if r[0]]
        p = [r[1] for r in self.rows if r[1]]
        if not f:
            return None
        return {"sclk_mhz_median": float(np.median(f)) / 1e6, "sclk_mhz_min": min(f) / 1e6, "samples": len(f),
                "board_power_w_median": float(np.median(p)) / 1e6 if p else None,
                "power_cap_w": (self._read("power1_cap") or 0) / 1e6 or None, "hwmon": self.dir,
                "note": "this device's hwmon, sampled every 10 ms over the timed steps"}


def valu_roof(compressions: int, ms: float) -> dict:
    a = compressions * 672 / (ms * 1e-3) / 1e12
    return {"achieved": a, "frac": a / VALU_PEAK_TOPS, "frac_full_rate": a / VALU_FULL_RATE_TOPS}


# ------------------------------------------------------------------ host CPU
def host_cpu() -> dict:
    import subprocess
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    quota = None
    try:  # the cgroup's CPU bandwidth limit, if any ("max" = none)
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q[0] == "max" else float(q[0]) / float(q[1])
    except (OSError, ValueError, IndexError):
        pass
    return {"model": model, "cpus_online": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


def all_cores() -> int:
    """nproc: every CPU in this process's affinity mask."""
    return len(os.sched_getaffinity(0))


def effective_cpus() -> int:
    """The CPUs this process can actually use: its affinity mask, capped by the cgroup's CPU
    quota (rounded up) where one is set -- SURVEY.md 8(d) configs[0](ii)'s "all cores" on a
    container whose nproc exceeds its quota (the GPU box: 256 online, a 16-CPU quota)."""
    q = host_cpu().get("cgroup_cpu_quota")
    n = all_cores()
    return max(1, min(n, int(np.ceil(q)))) if q else n


def cpu_baseline(sizes, cids, twins, seconds: float):
    """Oracle C restatement on the host, hash only over pre-staged messages.

    Uses the SIMD multi-chunk hasher (oracle/sd_oracle_simd.c: AVX-512 16-way / AVX2 8-way
    hash_many, the strategy of the reference's blake3 crate), so the baseline is the
    reference's arithmetic at its own CPU speed, not a scalar strawman.  Rows: 16 threads
    (the host's share per GPU of an 8-GPU node), 1 thread (the reference's one hashing task
    per step), and all cores (nproc)."""
    from oracle import native
    from spacedrive_amd.device import stage_plan
    threads = max(1, min(16, effective_cpus()))  # the box's CPU share for one GPU
    level = native.simd_level(-1)

    # the shard's messages are staged once (the plan of the first n files is the first n
    # extents of the shard's plan, at the same offsets) and each leg hashes a prefix of them
    staged = {}

    def prefix(n):
        if "buf" not in staged or staged["n"] < n:
            staged.clear()
            n_stage = len(sizes) if n > len(sizes) // 8 else n
            ext, total = stage_plan(sizes[:n_stage])
            staged.update(n=n_stage, ext=ext, buf=native.stage_synth(sizes[:n_stage], cids[:n_stage], twins[:n_stage],
                                                                     ext["msg_offset"], total, nthreads=threads))
        return staged["buf"], staged["ext"][:n]

    def rate(nthreads, n0):
        n = n0
        while True:
            buf, ext = prefix(n)
            t0 = time.perf_counter()
            native.cas_ids_staged(buf, ext, nthreads=nthreads, simd=-1)
            dt = time.perf_counter() - t0
            if dt >= seconds * 0.5 or n >= len(sizes):
                return n, dt, float(ext["msg_len"].astype(np.float64).sum())
            n = min(len(sizes), int(n * max(2.0, seconds / max(dt, 1e-3))))

    n1, dt1, b1 = rate(1, 2000)
    nT, dtT, bT = rate(threads, 20000)
    nA = effective_cpus()
    nN, dtN, bN = rate(nA, 100000)
    simd = {0: "scalar", 1: "AVX2 8-way", 2: "AVX-512 16-way"}[level]
    return {
        "value": nT / dtT, "unit": "files/s", "cores": threads, "kind": "port", "sample_files": nT,
        "sample": f"first {nT} files of this shard (same mixture), messages pre-staged in host RAM, hash only; "
                  f"C restatement of cas.rs + blake3 with {simd} multi-chunk hash_many (oracle/sd_oracle_simd.c) "
                  f"on {threads} threads; {bT / dtT / 1e9:.2f} GB/s of message bytes",
        "single_thread": {"value": n1 / dt1, "unit": "files/s", "cores": 1, "sample_files": n1,
                          "GBps": b1 / dt1 / 1e9},
        "all_cores": {"value": nN / dtN, "unit": "files/s", "cores": nA, "sample_files": nN, "GBps": bN / dtN / 1e9,
                      "nproc": all_cores(), "cgroup_cpu_quota": host_cpu().get("cgroup_cpu_quota"),
                      "note": "the same hash-only leg on every CPU this process can use: min(nproc, the cgroup's CPU "
                              "quota) threads (a thread count past the quota only shares the same CPU time)"},
        "simd": simd, "host_cpu": host_cpu(),
    }


# ------------------------------------------------------------------ parity of the timed steps
def oracle_threads() -> int:
    """host threads for the oracle checks: this rank's share of the host (the library's host
    thread budget, min(affinity, quota) / LOCAL_WORLD_SIZE), at most 16"""
    from spacedrive_amd._native import host_cpu_budget
    return max(1, min(16, host_cpu_budget()["budget"]))


def sample_idx(n: int, k: int = 4096, head: int = 32) -> np.ndarray:
    """k indices at an even stride over [0, n) plus the first `head` (the edge sizes)"""
    return np.unique(np.concatenate([np.arange(min(head, n)), np.linspace(0, n - 1, min(k, n)).astype(np.int64)]))


def oracle_hashes(sizes, cids, twins, idx) -> np.ndarray:
    """[len(idx), 32]: the full BLAKE3 of the cas messages of synthetic files idx, built by
    the C oracle from the same generator and hashed by its scalar BLAKE3 (oracle/sd_oracle.c)"""
    from oracle import native
    from spacedrive_amd.device import stage_plan
    s, c, t = sizes[idx], cids[idx], twins[idx]
    ext, total = stage_plan(s)
    buf = native.stage_synth(s, c, t, ext["msg_offset"], total)
    return native.checksums(buf, ext["msg_offset"], ext["msg_len"], nthreads=oracle_threads())


def parity_sample(sizes, cids, twins, d_hash, start: int, k: int = 4096) -> dict:
    """The timed steps' own output checked against the oracle (outside the timed region):
    a fixed sample of this rank's shard -- k files at an even stride, plus the shard's first
    32 (the edge sizes of SURVEY.md 8(d) on rank 0) -- has its cas messages built by the C
    oracle from the same generator and hashed by the oracle's BLAKE3 (oracle/sd_oracle.c);
    every sampled file's full 32-byte hash in d_hash must be equal."""
    n = len(sizes)
    idx = sample_idx(n, k)
    want = oracle_hashes(sizes, cids, twins, idx)
    got = d_hash.view(-1, 32)[torch.from_numpy(idx).to(d_hash.device)].cpu().numpy()
    bad = np.nonzero((got != want).any(axis=1))[0]
    return {"files": int(len(idx)), "mismatches": int(len(bad)),
            "first_bad_global_index": int(start + idx[bad[0]]) if len(bad) else None,
            "sampled_kind": int((sizes[idx] > 102400).sum()),
            "note": "full 32-byte hashes of the timed steps' output vs the C oracle (oracle/sd_oracle.c) on the "
                    "same generator: the shard's first 32 files + an even-stride sample"}


def _gather_rows(t: torch.Tensor, world: int, dev) -> list:
    """all_gather of a [m, w] int64 tensor whose m differs per rank (padded to the max)."""
    if not DIST:
        return [t]
    m = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    ms = [torch.zeros_like(m) for _ in range(world)]
    dist.all_gather(ms, m)
    mx = max(int(x.item()) for x in ms)
    pad = torch.zeros((mx, t.shape[1]), dtype=t.dtype, device=dev)
    pad[:t.shape[0]] = t.to(dev)
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return [o[:int(k.item())] for o, k in zip(outs, ms)]


def dedup_parity(d_hash, d_valid, n: int, start: int, recs, rep, owners, world: int, dev, transport: str) -> dict:
    """The multi-rank exchange checked end to end on a slice of the key space: every record
    whose cas_id key has bits 40..47 == 0 (1/256 of the keys, spread over every rank's
    prefix range, so every destination and every source takes part; a group is wholly in or
    out).  Input side: each rank's (key, global index) records of that slice, from its own
    hashes.  Output side: each rank's exchanged, grouped records of that slice with their
    representative and Object owner.  Rank 0 groups the input with group_host (the host
    mirror of the grouping) and applies identifier.object_owners; the output must be the
    same records, representatives and owners.  Returns the same dict on every rank."""
    from spacedrive_amd import identifier
    from spacedrive_amd.dedup import group_host
    h = d_hash.view(n, 32)[:, :8].to(torch.int64)
    key = torch.zeros(n, dtype=torch.int64, device=h.device)
    for j in range(8):  # big-endian u64 of the first 8 hash bytes (the hex cas_id's order)
        key = key | (h[:, j] << (56 - 8 * j))

    def in_slice(k):
        return ((k >> 40) & 0xFF) == 0

    sel = in_slice(key) & (d_valid.view(-1) != 0)
    gidx = torch.arange(start, start + n, dtype=torch.int64, device=h.device)
    inp = torch.stack([key[sel], gidx[sel]], dim=1)
    osel = in_slice(recs[:, 0])
    outp = torch.stack([recs[osel, 0], recs[osel, 1], rep[osel], owners[osel]], dim=1)
    cdev = dev if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu"
    ins = _gather_rows(inp, world, cdev)
    outs = _gather_rows(outp, world, cdev)
    ok = torch.zeros(1, dtype=torch.int64, device=cdev)
    res = {}
    if int(os.environ.get("RANK", "0")) == 0:
        a = torch.cat([x.cpu() for x in ins]).numpy()
        b = torch.cat([x.cpu() for x in outs]).numpy()
        r, rep_h, ng = group_host(a)
        own_h = identifier.object_owners(torch.from_numpy(r[:, 1].copy()), torch.from_numpy(rep_h.copy())).numpy()
        order = np.lexsort((b[:, 1], b[:, 0].view(np.uint64)))
        b = b[order]
        same = (len(b) == len(r) and np.array_equal(b[:, :2], r) and np.array_equal(b[:, 2], rep_h)
                and np.array_equal(b[:, 3], own_h))
        per_rank_out = [int(x.shape[0]) for x in outs]
        res = {"records": int(len(r)), "groups": int(ng), "linked": int((own_h != r[:, 1]).sum()),
               "out_records_per_rank": per_rank_out, "parity": bool(same)}
        ok[0] = 1 if same else 0
    if DIST:
        dist.broadcast(ok, 0)
    res["parity"] = bool(int(ok.item()))
    res["slice"] = "cas_id keys with bits 40..47 == 0 (1/256 of the key space, every prefix range)"
    out_side = {"rccl": "sd_cas_dedup_mgpu over libsdcas's RCCL communicator",
                "torch": "dedup.dedup_shard over torch.distributed (" + (dist.get_backend() if DIST else "no") +
                         " process group)"}[transport]
    res["transport"] = transport
    res["note"] = ("input records (each rank's own hashes) grouped on rank 0 by group_host + identifier.object_owners "
                   f"vs the exchanged, grouped output of {out_side} from every rank")
    return res


# ------------------------------------------------------------------ with-H2D legs
def ev_ms(fn, stream, reps=1):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _native_budget() -> int:
    from spacedrive_amd._native import host_cpu_budget
    return int(host_cpu_budget()["budget"])


def host_staged(ctx, ext, d_staged, k, dev, stream, world: int = 1, lib_=None):
    """with-H2D cas_ids: the first k files' staged messages in pinned host memory through
    the drop-in sd_cas_ids (host plan + H2D + kernels + D2H + hex, windows pipelined on two
    streams), beside the raw H2D copy of the same bytes and the device-resident kernels.
    Runs on every rank at once (one PCIe link per GPU): a fixed count of calls -- one warm,
    then 2 timed -- between barriers; the aggregate is all ranks' files over the slowest
    rank's time."""
    from spacedrive_amd._native import check, lib
    k = min(k, len(ext))
    nbytes = (int(ext["msg_offset"][k - 1]) + int(ext["msg_len"][k - 1]) + 63) // 64 * 64
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.copy_(d_staged[:nbytes])
    sub = np.ascontiguousarray(ext[:k])
    dbuf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    h2d_ms = min(ev_ms(lambda: dbuf.copy_(host, non_blocking=True), stream) for _ in range(3))
    b = ctx.cas_batch(sub)
    hh = torch.empty(k * 32, dtype=torch.uint8, device=dev)
    b.run(dbuf, hh, stream)
    kernel_ms = ev_ms(lambda: b.run(dbuf, hh, stream), stream, reps=3)
    want = hh.cpu().numpy().reshape(k, 32)[:, :8]
    del dbuf, b, hh
    out = ctypes.create_string_buffer(17 * k)

    def call():
        check(lib().sd_cas_ids(ctx.handle, host.data_ptr(), nbytes, sub.ctypes.data, k, out, None))

    import spacedrive_amd as sd
    keep = sd.get_tuning("host_cohash_threads")
    e2e = {}
    for mode, h in (("gpu_only", 0), ("default", keep)):  # the GPU alone, then the library default
        sd.set_tuning("host_cohash_threads", h)
        try:
            call()  # warm: the context's windows and tables
            reps = 2
            if DIST:
                dist.barrier()
            s0 = np.zeros(2, np.uint64)
            s1 = np.zeros(2, np.uint64)
            check(lib().sd_cas_ids_stats(ctx.handle, s0.ctypes.data))
            t0 = time.perf_counter()
            for _ in range(reps):
                call()
            # the threads the library runs for h: at most the host budget less one (sd_cas_ids)
            e2e[mode] = ((time.perf_counter() - t0) / reps,
                         max(0, min(h, _native_budget() - 1)))
            check(lib().sd_cas_ids_stats(ctx.handle, s1.ctypes.data))
            e2e[mode] += (float((s1 - s0)[1]) / (reps * k),)
            if DIST:
                dist.barrier()
        finally:
            sd.set_tuning("host_cohash_threads", keep)
        if mode == "gpu_only":
            raw_gpu = out.raw
    e2e_s = e2e["default"][0]
    raw = out.raw  # one copy: each .raw access copies the whole buffer
    assert raw == raw_gpu, "sd_cas_ids with host co-hashing differs from the GPU alone"
    got = np.frombuffer(bytes.fromhex("".join(raw[17 * i:17 * i + 16].decode() for i in range(k))),
                        np.uint8).reshape(k, 8)
    assert np.array_equal(got, want), "sd_cas_ids differs from the device-resident batch"
    par = None
    if lib_ is not None:  # the call's own cas_ids against the oracle, on an even-stride sample
        idx = sample_idx(k)
        w8 = oracle_hashes(*lib_, idx)[:, :8]
        par = parity(len(idx), int((got[idx] != w8).any(axis=1).sum()),
                     "cas_ids of an even-stride sample (+ the first 32) vs the C oracle on the same generator")
    cpu_row = None
    if not DIST:  # the library's CPU path over the same messages (one process: no other rank's load)
        from spacedrive_amd._native import host_cpu_budget
        nt = min(16, host_cpu_budget()["budget"])
        cout = ctypes.create_string_buffer(17 * k)
        runs = []
        for _ in range(3):
            t0 = time.perf_counter()
            check(lib().sd_cpu_cas_ids(host.data_ptr(), nbytes, sub.ctypes.data, k, cout, None, nt))
            runs.append(time.perf_counter() - t0)
        assert cout.raw == raw, "sd_cpu_cas_ids differs from sd_cas_ids"
        cpu_row = {"files_per_s": k / min(runs[1:]), "threads": nt,
                   "default_over_cpu_path": min(runs[1:]) / e2e_s,
                   "note": "sd_cpu_cas_ids over the same pinned messages, best of 2 after a warm run"}
    res = {"files": k, "bytes": nbytes, "h2d_ms": h2d_ms, "h2d_GBps": nbytes / (h2d_ms * 1e-3) / 1e9,
           "kernel_ms": kernel_ms, "kernel_files_per_s": k / (kernel_ms * 1e-3),
           "end_to_end_ms": e2e_s * 1e3, "end_to_end_files_per_s": k / e2e_s,
           "end_to_end_GBps": nbytes / e2e_s / 1e9,
           "host_cohash_threads": e2e["default"][1], "host_share": e2e["default"][2],
           "gpu_only": {"end_to_end_ms": e2e["gpu_only"][0] * 1e3,
                        "end_to_end_files_per_s": k / e2e["gpu_only"][0],
                        "end_to_end_GBps": nbytes / e2e["gpu_only"][0] / 1e9},
           "parity": par,
           "library_cpu_path": cpu_row,
           "note": "sd_cas_ids from pinned host memory (mean of 2 calls after a warm one, all ranks at once): "
                   "plan + H2D + kernels + D2H + hex, 512 MiB windows on two streams, with the library default "
                   "of host_cohash_threads host threads hashing files from the end of the list meanwhile "
                   "(host_share = their fraction of the files); gpu_only = the same call with 0; h2d_ms = one "
                   "raw copy of the same bytes (HIP events); kernel_ms = the same files device-resident"}
    if DIST:
        rows = [None] * world
        dist.all_gather_object(rows, [e2e_s, k, nbytes])
        per = [{"rank": r, "end_to_end_files_per_s": row[1] / row[0], "end_to_end_GBps": row[2] / row[0] / 1e9}
               for r, row in enumerate(rows)]
        slow = max(row[0] for row in rows)
        res["per_rank"] = per
        res["aggregate"] = {"ranks": world, "files_per_s": sum(row[1] for row in rows) / slow,
                            "GBps": sum(row[2] for row in rows) / slow / 1e9,
                            "note": "all ranks' files and bytes over the slowest rank's time"}
    return res


def cohash_cap(budget: int) -> int:
    """sd_checksums' co-hash thread cap under a host budget (sd_host.h checksum_cohash_cap)"""
    return 0 if budget <= 1 else budget - max(1, (3 * budget + 8) // 16)


def checksum_host(ctx, gib: int, dev, stream):
    """with-H2D checksums: `gib` GiB of pinned host memory (files of 1 GiB) through the
    drop-in sd_checksums, beside the raw H2D copy and the device-resident kernels."""
    from spacedrive_amd import _native
    from spacedrive_amd._native import check, lib
    nf, flen = gib, 1 << 30
    total = nf * flen
    d = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    for i in range(nf):
        ctx.synth_fill(20_000 + i, 0, flen, d[i * flen:])
    host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    host.copy_(d)
    scratch = torch.empty_like(d)
    h2d_ms = min(ev_ms(lambda: scratch.copy_(host, non_blocking=True), stream) for _ in range(2))
    del scratch
    offs = np.arange(nf, dtype=np.uint64) * np.uint64(flen)
    lens = np.full(nf, flen, np.uint64)
    cb = ctx.checksum_batch(offs, lens)
    hs = torch.empty(nf * 32, dtype=torch.uint8, device=dev)
    cb.run(d, hs, stream)
    kernel_ms = ev_ms(lambda: cb.run(d, hs, stream), stream, reps=2)
    want = [hs[32 * i:32 * i + 32].cpu().numpy().tobytes().hex() for i in range(nf)]
    del d, cb
    torch.cuda.empty_cache()
    import spacedrive_amd as sd
    out = ctypes.create_string_buffer(65 * nf)
    keep = sd.get_tuning("host_cohash_threads")
    e2e = {}
    st0, st1 = np.zeros(2, np.uint64), np.zeros(2, np.uint64)
    for mode, h in (("gpu_only", 0), ("default", keep)):
        sd.set_tuning("host_cohash_threads", h)
        try:
            runs = []
            if mode == "default":
                # the library's learned route (co-hashed or the CPU path alone, "checksum_split_adapt"):
                # its four learning calls -- each route's warm-up and first counted call -- first
                for _ in range(4):
                    check(lib().sd_checksums(ctx.handle, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, nf, out))
                check(lib().sd_checksums_stats(ctx.handle, st0.ctypes.data))
            for _ in range(3):  # the first call allocates the context's windows
                ctypes.memset(out, 0, 65 * nf)
                t0 = time.perf_counter()
                check(lib().sd_checksums(ctx.handle, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, nf, out))
                runs.append(time.perf_counter() - t0)
        finally:
            sd.set_tuning("host_cohash_threads", keep)
        if mode == "default":
            check(lib().sd_checksums_stats(ctx.handle, st1.ctypes.data))
        raw = out.raw
        got = [raw[65 * i:65 * i + 64].decode() for i in range(nf)]
        assert got == want, f"sd_checksums ({mode}) differs from the device-resident batch"
        e2e[mode] = min(runs)
    d_gpu, d_host = (int(x) for x in (st1 - st0))
    host_share = d_host / (d_gpu + d_host) if d_gpu + d_host else None
    lv = np.zeros(4, np.float64)  # what this context learned (sd_checksums_learned)
    check(lib().sd_checksums_learned(ctx.handle, lv.ctypes.data))
    learned = {"cohash_GBps": float(lv[0]), "cpu_GBps": float(lv[1]), "cohash_calls": int(lv[2]),
               "cpu_calls": int(lv[3])}
    e2e_s = e2e["default"]
    from oracle import native
    bad = sum(native.checksum_synth_mt(flen, 20_000 + i, 0, nthreads=oracle_threads()).hex() != got[i]
              for i in range(nf))
    # the same bytes as ONE range: shared by the GPU and the host threads block by block
    one_off = np.zeros(1, np.uint64)
    one_len = np.array([total], np.uint64)
    one = {}
    for mode, h in (("gpu_only", 0), ("default", keep)):
        sd.set_tuning("host_cohash_threads", h)
        try:
            runs = []
            for _ in range(3):
                ctypes.memset(out, 0, 65)
                t0 = time.perf_counter()
                check(lib().sd_checksums(ctx.handle, host.data_ptr(), one_off.ctypes.data, one_len.ctypes.data, 1, out))
                runs.append(time.perf_counter() - t0)
        finally:
            sd.set_tuning("host_cohash_threads", keep)
        one[mode] = (min(runs), out.raw[:64].decode())
    one_want = native.checksum_mt(host.numpy(), total, nthreads=oracle_threads()).hex()
    one_bad = sum(v[1] != one_want for v in one.values())
    # the library's CPU path over the same ranges on the host budget's threads (no device)
    cpu_t = effective_cpus()
    h32 = np.zeros((nf, 32), np.uint8)
    cpu_runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        check(lib().sd_cpu_checksums(host.data_ptr(), offs.ctypes.data, lens.ctypes.data, nf, h32.ctypes.data, cpu_t))
        cpu_runs.append(time.perf_counter() - t0)
    cpu_bad = sum(h32[i].tobytes().hex() != got[i] for i in range(nf))
    par = parity(nf, bad, "every file's 64-hex checksum vs the C oracle's chunk-parallel BLAKE3 of the same content")
    return {"files": nf, "bytes": total, "h2d_ms": h2d_ms, "h2d_GBps": total / (h2d_ms * 1e-3) / 1e9, "parity": par,
            "kernel_ms": kernel_ms, "kernel_GBps": total / (kernel_ms * 1e-3) / 1e9,
            "end_to_end_ms": e2e_s * 1e3, "end_to_end_GBps": total / e2e_s / 1e9,
            "host_cohash_threads": max(0, min(keep, cohash_cap(_native.host_cpu_budget()["budget"]))),
            "host_share": host_share, "learned": learned,
            "gpu_only": {"end_to_end_ms": e2e["gpu_only"] * 1e3, "end_to_end_GBps": total / e2e["gpu_only"] / 1e9},
            "library_cpu_path": {"threads": cpu_t, "GBps": total / min(cpu_runs) / 1e9,
                                 "parity": parity(nf, cpu_bad, "sd_cpu_checksums of each range vs sd_checksums' "
                                                               "oracle-checked output"),
                                 "note": "sd_cpu_checksums over the same ranges (1 MiB blocks as tasks), best of 3"},
            "default_over_cpu_path": min(cpu_runs) / e2e_s,
            "one_range": {"bytes": total, "end_to_end_GBps": total / one["default"][0] / 1e9,
                          "gpu_only_GBps": total / one["gpu_only"][0] / 1e9,
                          "parity": parity(2, one_bad, "the one range's checksum (default and GPU only) vs the C "
                                                       "oracle's chunk-parallel BLAKE3 of the same bytes"),
                          "note": "the same bytes as one range: its 1 MiB blocks shared between the GPU (windows "
                                  "from the front) and the host threads (from the back), best of 3"},
            "note": f"sd_checksums over {nf} x 1 GiB of pinned host memory (best of 3): 256 MiB windows, H2D on one "
                    "copy queue overlapping the kernels on two slot streams, with the library default of "
                    "host_cohash_threads host threads hashing ranges from the end meanwhile, one range shared "
                    "block by block where the two sides meet (gpu_only: 0; host_share = the bytes those threads "
                    "hashed over the 3 default calls, sd_checksums_stats); "
                    "h2d_ms = one raw copy; kernel_ms = device-resident"}


# ------------------------------------------------------------------ configs[1] / [2]
def warm(fn, stream, ms_target: float) -> float:
    """Runs fn until ~ms_target of GPU time has passed (the clock ramps up over tens of ms
    after the GPU idles: profiles/r2/r2b_whole_ab.json); returns the first launch's ms."""
    first = ev_ms(fn, stream)
    reps = int(max(0, ms_target - first) / max(first, 1e-3))
    if reps:
        ev_ms(fn, stream, reps=reps)
    return first


def config_leg(ctx, which: str, nfiles: int, reps: int, dev, stream, valu_peak: float, warm_ms: float,
               live: bool = False):
    """configs[1] (1 M files <= 100 KiB, whole-content cas_id) or configs[2] (1 M files
    > 100 KiB, sampled cas_id) on this GPU: kernel-only files/s over device-resident
    staged messages, timed with HIP events on the launch stream, plus determinism of the
    full 32-byte hashes across runs and, outside the timing, a 4 096-file even-stride
    sample of the timed output against the oracle (`parity`)."""
    import spacedrive_amd as sd
    from spacedrive_amd import synth
    gen = synth.small_library if which == "small" else synth.sampled_library
    sizes, cids, twins = gen(0, nfiles)
    ext, total = sd.stage_plan(sizes)
    d_staged = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                        torch.from_numpy(twins.astype(np.int32)).to(dev), d_ext, nfiles, d_staged, stream)
    b = ctx.cas_batch(ext)
    h0 = torch.zeros(nfiles * 32, dtype=torch.uint8, device=dev)
    h1 = torch.zeros(nfiles * 32, dtype=torch.uint8, device=dev)
    b.run(d_staged, h0, stream)
    cold_ms = warm(lambda: b.run(d_staged, h1, stream), stream, warm_ms)
    clock = ClockSampler(dev.index if dev.index is not None else 0).start()
    ms = ev_ms(lambda: b.run(d_staged, h1, stream), stream, reps=reps)
    clock_res = clock.result()
    deterministic = bool(torch.equal(h0, h1))
    roof = valu_roof(b.compressions, ms)
    if which == "sampled":
        kernels, grid = SAMPLED_KERNELS, sampled_grids(b.n_sampled)
        tr = pmc_traffic_sum(kernels, grid)
    else:
        kernels, grid = ["k_whole_items", "k_whole_merge8"], whole_grid(b)
        tr = pmc_traffic(kernels[0], grid)
    ps = parity_sample(sizes, cids, twins, h1, 0)
    pf = full_parity(h1, nfiles, config_digest_key(which, nfiles), lambda: (sizes, cids, twins), live)
    res = {"workload": ("configs[1]: 1M files <= 100 KiB, whole-content cas_id (log-uniform sizes 1..102400)"
                        if which == "small" else
                        "configs[2]: 1M files > 100 KiB, sampled cas_id (log-uniform sizes 102401..4 GiB)"),
           "files": nfiles, "kernel_ms": ms, "files_per_s": nfiles / (ms * 1e-3), "reps": reps,
           "first_launch_ms": cold_ms,
           "msg_GBps": b.msg_bytes / (ms * 1e-3) / 1e9, "compressions": b.compressions,
           "valu_frac": roof["frac"], "valu_frac_full_rate": roof["frac_full_rate"],
           "valu_frac_of_measured_peak": roof["achieved"] * 1e12 / valu_peak if valu_peak else None,
           "clock": clock_res,
           "valu_frac_at_clock": (roof["achieved"] * 1e12
                                  / (G_MIX_LANE_OPS_PER_CLK * N_CUS * clock_res["sclk_mhz_median"] * 1e6)
                                  if clock_res else None),
           "kernels": kernels, "launch_grid": grid,
           "issue_rate_pmc": pmc_issue_rate(kernels[0], grid[0] if isinstance(grid, list) else grid),
           "traffic": tr["bytes"] if tr else None, "deterministic": deterministic,
           "parity": parity(ps["files"], ps["mismatches"], "full 32-byte hashes of an even-stride sample (+ the first "
                            "32) vs the C oracle (oracle/sd_oracle.c) on the same generator"),
           "parity_full": parity(pf["files"], pf["mismatches"], pf["oracle"], expected_from=pf["expected_from"])}
    del d_staged, h0, h1, b
    torch.cuda.empty_cache()
    assert deterministic, which
    return res


# ------------------------------------------------------------------ file-backed legs
def _fs_type(path: str) -> str:
    best, fstype = "", "?"
    try:
        for line in open("/proc/mounts"):
            parts = line.split()
            if len(parts) > 2 and path.startswith(parts[1]) and len(parts[1]) > len(best):
                best, fstype = parts[1], parts[2]
    except OSError:
        pass
    return fstype


def _cpu_s() -> float:
    """user + system CPU seconds of this process so far (every thread, the library's included)"""
    import resource
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def _scratch_dir(need: int) -> str:
    import tempfile
    base = "/dev/shm"
    try:
        st = os.statvfs(base)
        if st.f_bavail * st.f_frsize < 4 * need:
            base = None
    except OSError:
        base = None
    return tempfile.mkdtemp(prefix="sd_fb_", dir=base)


def latency(ctx, paths, sizes, calls: int) -> dict:
    """Single-call latency (p50 / p99, microseconds) of generate_cas_id for the reference's
    per-file callers (watcher/utils.rs:235,393; non_indexed.rs:168): idle (one caller) and
    with 64 concurrent callers, for the GPU-coalesced path (latency_cpu_max = 0), the CPU
    path (sd_cpu_cas_id_path) and the default policy (CPU below 16 calls in flight)."""
    from spacedrive_amd._native import check, lib
    L = lib()
    enc = [os.fsencode(p) for p in paths]
    n = len(enc)

    def gpu_call(i, out, st):
        return L.sd_cas_id_path(ctx.handle, enc[i % n], int(sizes[i % n]), out, ctypes.byref(st))

    def cpu_call(i, out, st):
        return L.sd_cpu_cas_id_path(enc[i % n], int(sizes[i % n]), out, ctypes.byref(st))

    def run(fn, callers, per_caller):
        lat = [[] for _ in range(callers)]
        barrier = threading.Barrier(callers)

        def worker(c):
            out = ctypes.create_string_buffer(17)
            st = ctypes.c_int32(0)
            barrier.wait()
            for j in range(per_caller):
                t0 = time.perf_counter()
                check(fn(c * per_caller + j, out, st))
                lat[c].append(time.perf_counter() - t0)
                assert st.value == 0

        t0 = time.perf_counter()
        th = [threading.Thread(target=worker, args=(c,)) for c in range(callers)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        v = np.array([x for row in lat for x in row]) * 1e6
        return {"p50_us": float(np.percentile(v, 50)), "p99_us": float(np.percentile(v, 99)),
                "calls": int(v.size), "calls_per_s": v.size / wall}

    res = {}
    keep = ctypes.c_int32(0)
    check(L.sd_cas_get_tuning(b"batch_cpu_max", ctypes.byref(keep)))
    # gpu_coalesced: every call coalesced AND every coalesced batch on the GPU (both policies
    # off); policy_default: the library's defaults (CPU below 16 calls in flight, coalesced
    # batches through sd_cas_ids_files' batch policy)
    for mode, cpu_max, batch_max in (("gpu_coalesced", 0, 0), ("policy_default", 16, keep.value)):
        check(L.sd_cas_set_tuning(b"latency_cpu_max", cpu_max))
        check(L.sd_cas_set_tuning(b"batch_cpu_max", batch_max))
        try:
            run(gpu_call, 1, 20)  # warm
            res[mode] = {"idle": run(gpu_call, 1, calls), "concurrent_64": run(gpu_call, 64, max(4, calls // 16))}
        finally:
            check(L.sd_cas_set_tuning(b"latency_cpu_max", 16))
            check(L.sd_cas_set_tuning(b"batch_cpu_max", keep.value))
    res["cpu_path"] = {"idle": run(cpu_call, 1, calls), "concurrent_64": run(cpu_call, 64, max(4, calls // 16))}
    res["note"] = ("files of the file-backed leg on tmpfs (page cache warm), one generate_cas_id per call through "
                   "ctypes from Python threads; gpu_coalesced = sd_cas_id_path with latency_cpu_max 0 and "
                   "batch_cpu_max 0 (every call coalesced, 200 us window, every batch on the GPU); policy_default = "
                   "the defaults (latency_cpu_max 16; coalesced batches of <= 4096 on the CPU path); "
                   "cpu_path = sd_cpu_cas_id_path")
    return res


def identifier_leg(paths, k: int) -> dict:
    """The identifier job (file_identifier_job.rs:80-309, mod.rs:100-392) over the first k
    files: 100-row steps by cursor, Object link/create per step.  (a) look-ahead: each
    hashing call covers the next 32768 orphans (spacedrive_amd/identifier.py IdentifierJob;
    generate_cas_ids -> sd_cas_ids_files, the GPU route); (b) per step: each step hashes
    its own 100 files with the library's CPU path on 16 threads (the reference's per-step
    structure, integration/rust/core/cas.rs without a GPU).  Both give the same Objects.
    hash_s = time inside the batched hashing calls; job_s = the whole job, whose stat calls
    (FileMetadata::new's fs::metadata, mod.rs:65-67) and Object bookkeeping are Python here
    (the reference's bookkeeping is DB writes, out of scope).  Each job runs twice and the
    second, warm run is reported (`first_run` keeps the cold one)."""
    from spacedrive_amd import cas as sdcas
    from spacedrive_amd import cpu, identifier
    paths = paths[:k]
    res = {"files": len(paths), "steps": (len(paths) + 99) // 100}
    owners = {}
    for name, k_ahead, hash_batch in (
            ("lookahead_gpu", identifier.LOOKAHEAD, sdcas.generate_cas_ids),
            ("per_step_cpu_path", identifier.CHUNK_SIZE, lambda p, s: cpu.generate_cas_ids(p, s, nthreads=16))):
        for run in range(2):  # the whole job twice; the second (warm) run is reported
            acc = [0.0]

            def timed(p, s, fn=hash_batch, acc=acc):
                t0 = time.perf_counter()
                r = fn(p, s)
                acc[0] += time.perf_counter() - t0
                return r
            t0 = time.perf_counter()
            job = identifier.IdentifierJob(paths, lookahead=k_ahead,
                                           metadata=identifier._stat_then_hash(timed)).run()
            job_s = time.perf_counter() - t0
            if run == 0:
                first = {"job_s": job_s, "hash_s": acc[0]}
        owners[name] = job.owner
        res[name] = {"job_s": job_s, "hash_s": acc[0], "hash_calls": len(job.hash_calls),
                     "hash_files_per_s": len(paths) / acc[0], "job_files_per_s": len(paths) / job_s,
                     "created": sum(c for c, _ in job.step_stats), "linked": sum(x for _, x in job.step_stats),
                     "first_run": first}
    res["same_objects"] = owners["lookahead_gpu"] == owners["per_step_cpu_path"]
    res["hash_speedup"] = res["per_step_cpu_path"]["hash_s"] / res["lookahead_gpu"]["hash_s"]
    assert res["same_objects"], "look-ahead and per-step identifier jobs disagree"
    return res


def file_backed(ctx, sizes, ext, d_staged, k: int, with_cpu: bool, latency_calls: int, ident_files: int = 0):
    """The drop-in path from files on disk, as identifier_job_step would drive it
    (file_identifier/mod.rs:107-134): the first k files of this shard are written to a
    scratch directory (sampled files sparse: only the windows cas.rs reads are
    materialised), then timed end to end through sd_cas_ids_files (read stager pool
    overlapped with H2D + kernels + D2H), beside the reference's own read schedule
    (open, read_exact, seek; cas.rs:27-58) + the SIMD C restatement on 1, 16 and all
    threads and the library's CPU path on 16 and all threads.  All read from the page cache
    (files just written); the outputs are asserted equal."""
    import shutil
    import spacedrive_amd as sd
    from spacedrive_amd import synth
    from spacedrive_amd._native import check, lib
    k = min(k, len(sizes))
    sub_sizes = np.ascontiguousarray(sizes[:k])
    nbytes = int(ext["msg_offset"][k - 1]) + int(ext["msg_len"][k - 1])
    host = d_staged[:nbytes].cpu().numpy()  # messages in the shard layout (same offsets)
    d = _scratch_dir(nbytes)
    try:
        t0 = time.perf_counter()
        paths = synth.write_files(d, sub_sizes, host, ext[:k])
        write_s = time.perf_counter() - t0
        del host
        L = lib()
        arr = (ctypes.c_char_p * k)(*[os.fsencode(p) for p in paths])
        from spacedrive_amd._native import host_cpu_budget
        threads = min(16, host_cpu_budget()["budget"])  # the library caps every call at its host budget
        nA = effective_cpus()
        out = ctypes.create_string_buffer(17 * k)
        st = np.zeros(k, np.int32)
        sz = np.ascontiguousarray(sub_sizes, np.uint64)
        # the GPU route and the CPU path (the C calls alone, paths encoded once, outside) in
        # interleaved rounds -- the host's load drifts between boxes and within a run -- the
        # first round warming the stager's threads and the context's slots
        cpu_out = ctypes.create_string_buffer(17 * k)
        cpu_st = np.zeros(k, np.int32)
        pipe, pipe_cpu, lib_runs, lib_cpu = [], [], [], []
        gpu_ids = None
        for _ in range(4):
            c0, t0 = _cpu_s(), time.perf_counter()
            check(L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, out, st.ctypes.data, threads))
            pipe.append(time.perf_counter() - t0)
            pipe_cpu.append(_cpu_s() - c0)
            assert (st == 0).all(), np.unique(st)
            if gpu_ids is None:
                raw = out.raw
                gpu_ids = [raw[17 * i:17 * i + 16].decode() for i in range(k)]
            c0, t0 = _cpu_s(), time.perf_counter()
            check(L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, cpu_out, cpu_st.ctypes.data, threads))
            lib_runs.append(time.perf_counter() - t0)
            lib_cpu.append(_cpu_s() - c0)
        assert (cpu_st == 0).all(), np.unique(cpu_st)
        craw = cpu_out.raw
        assert [craw[17 * i:17 * i + 16].decode() for i in range(k)] == gpu_ids, \
            "the library's CPU path differs from its GPU path"
        pipe_s, lib_s = float(np.median(pipe[1:])), float(np.median(lib_runs[1:]))
        res = {"files": k, "dir_fs": _fs_type(d), "write_s": write_s,
               "message_bytes": int(ext["msg_len"][:k].astype(np.int64).sum()),
               "gpu": {"files_per_s": k / pipe_s, "files_per_s_best": k / min(pipe[1:]), "ms": pipe_s * 1e3,
                       "stage_threads": threads, "host_cpu_us_per_file": float(np.median(pipe_cpu[1:])) / k * 1e6,
                       "note": "sd_cas_ids_files: read by the library's stager threads into a ring of pinned "
                               "windows, overlapped with H2D + kernels + D2H + hex; median of 3 warm rounds, "
                               "interleaved with the CPU path's"},
               "library_cpu_path": {"files_per_s": k / lib_s, "files_per_s_best": k / min(lib_runs[1:]),
                                    "threads": threads, "lanes": sd.cpu.simd_lanes(),
                                    "host_cpu_us_per_file": float(np.median(lib_cpu[1:])) / k * 1e6,
                                    "note": "sd_cpu_cas_ids_files, median of 3 warm rounds, interleaved with the "
                                            "GPU route's"}}
        if nA != threads:
            runs = []
            for _ in range(3):
                t0 = time.perf_counter()
                check(L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, cpu_out, cpu_st.ctypes.data, nA))
                runs.append(time.perf_counter() - t0)
            assert (cpu_st == 0).all() and cpu_out.raw == craw
            res["library_cpu_path_all_cores"] = {"files_per_s": k / min(runs[1:]), "threads": nA,
                                                 "note": "sd_cpu_cas_ids_files, best of 2 warm runs"}
        else:
            res["library_cpu_path_all_cores"] = {"same_as": "library_cpu_path", "threads": nA,
                                                 "note": "every usable CPU is the 16-thread row's (quota)"}
        res["gpu_over_cpu_path_16_threads"] = lib_s / pipe_s
        # the GPU route's cas_ids against the oracle reading the same files with the reference's
        # read schedule, on an even-stride sample (the whole set too when with_cpu, below)
        from oracle import native
        idx = sample_idx(k)
        o8, ost = native.cas_ids_files([paths[i] for i in idx], sub_sizes[idx], nthreads=oracle_threads())
        bad = int(sum((ost[j] != 0) or (o8[j].tobytes().hex() != gpu_ids[i]) for j, i in enumerate(idx)))
        res["parity"] = parity(len(idx), bad, "cas_ids of an even-stride sample of the files vs the C oracle's "
                                              "reference read schedule (cas.rs:27-58) + BLAKE3")
        if with_cpu:
            from oracle import native
            ol = native.lib()
            got = np.zeros((k, 8), np.uint8)
            cst = np.zeros(k, np.int32)
            cpu = {}
            for nt, runs in sorted({(1, 1), (threads, 2), (nA, 2)}):  # (all cores == 16 under a 16-CPU quota)
                dts = []
                kk = min(k, 50000) if nt == 1 else k  # one thread: a bounded sample (~0.5 s)
                for _ in range(runs):
                    t0 = time.perf_counter()
                    ol.sdo_cas_ids_files(arr, native._p(sz), kk, native._p(got), native._p(cst), nt, -1)
                    dts.append(time.perf_counter() - t0)
                cpu[f"threads_{nt}"] = {"files_per_s": kk / min(dts), "seconds": min(dts), "files": kk}
                assert (cst[:kk] == 0).all()
            want = [got[i].tobytes().hex() for i in range(k)]
            res["cpu_reference_schedule"] = cpu
            res["equal_to_cpu"] = want == gpu_ids
            assert res["equal_to_cpu"], "file-backed GPU cas_ids differ from the CPU restatement"
        if ident_files > 0:
            res["identifier_job"] = identifier_leg(paths, ident_files)
        if latency_calls > 0:
            res["latency"] = latency(ctx, paths[:2000], sub_sizes[:2000], latency_calls)
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def file_checksums_leg(ctx, mib: int, with_cpu: bool, dev):
    """file_checksum from files on tmpfs (hash.rs:10-24): 256 MiB files through the drop-in
    sd_file_checksums -- its GPU route alone ("checksum_cpu_max" = 0: 1 MiB reads streamed
    into pinned windows, overlapped with H2D + kernels) and its default policy (a call this
    large is split between the GPU route on 4 readers and the CPU path on the rest) -- and
    the library's CPU path on 16 threads, interleaved over 4 rounds (the first warms; the
    host's load drifts, so the routes alternate), medians reported; then the CPU path on
    every usable CPU and the reference's read schedule + the SIMD C restatement (oracle, 1,
    16 and all threads).  Outputs asserted equal, and checked against the oracle."""
    import shutil
    import spacedrive_amd as sd
    nf = max(1, mib // 256)
    flen = 256 << 20
    d = _scratch_dir(nf * flen)
    try:
        buf = torch.empty(flen, dtype=torch.uint8, device=dev)
        paths = []
        for i in range(nf):
            ctx.synth_fill(30_000 + i, 0, flen, buf)
            torch.cuda.synchronize()
            p = os.path.join(d, f"ck{i}")
            buf.cpu().numpy().tofile(p)
            paths.append(p)
        del buf
        total = nf * flen
        res = {"files": nf, "bytes": total, "dir_fs": _fs_type(d)}
        default_cpu_max = sd.get_tuning("checksum_cpu_max")
        want = sd.cpu.file_checksums(paths, nthreads=16)  # every leg must return these (and the oracle)

        def route(cpu_max):
            def f():
                sd.set_tuning("checksum_cpu_max", cpu_max)
                try:
                    return sd.file_checksums(paths)
                finally:
                    sd.set_tuning("checksum_cpu_max", default_cpu_max)
            return f
        legs = {"gpu": route(0), "policy_default": route(default_cpu_max),
                "library_cpu_path": lambda: sd.cpu.file_checksums(paths, nthreads=16)}
        runs = {k: [] for k in legs}
        routes0 = sd.file_checksums_stats()
        split_bytes = {"gpu": 0, "cpu_in_split": 0}
        per_call = []  # policy_default: the route each call took ("checksum_split_adapt") and its GB/s
        # the policy's learning calls first: each route's uncounted warm-up call and one counted
        # call (sd_host.h split_route_choose), so the timed rounds see the route it settled on
        for _ in range(4):
            r0 = sd.file_checksums_stats()
            t0 = time.perf_counter()
            assert legs["policy_default"]() == want
            r1 = sd.file_checksums_stats()
            per_call.append({"round": "learn", "route": "split" if r1["hybrid"] > r0["hybrid"] else
                             ("cpu" if r1["cpu"] > r0["cpu"] else "gpu"), "GBps": total / (time.perf_counter() - t0) / 1e9})
        for rnd in range(4):  # round 0 warms the windows, the pools and the page cache
            for k, f in legs.items():
                b0, r0 = sd.file_checksums_bytes(), sd.file_checksums_stats()
                t0 = time.perf_counter()
                got = f()
                dt = time.perf_counter() - t0
                assert got == want, k
                if k == "policy_default":
                    r1 = sd.file_checksums_stats()
                    per_call.append({"round": rnd, "route": "split" if r1["hybrid"] > r0["hybrid"] else
                                     ("cpu" if r1["cpu"] > r0["cpu"] else "gpu"), "GBps": total / dt / 1e9})
                if rnd:
                    runs[k].append(dt)
                    if k == "policy_default":
                        b1 = sd.file_checksums_bytes()
                        for x in split_bytes:
                            split_bytes[x] += b1[x] - b0[x]
        routes1 = sd.file_checksums_stats()
        for k in legs:
            res[k] = {"GBps": total / float(np.median(runs[k])) / 1e9, "GBps_best": total / min(runs[k]) / 1e9,
                      "seconds_median": float(np.median(runs[k])), "rounds": len(runs[k])}
        res["library_cpu_path"]["threads"] = 16
        res["policy_default"]["route"] = {k: routes1[k] - routes0[k] for k in routes1}
        res["policy_default"]["per_call"] = per_call
        res["policy_default"]["split_adapt"] = sd.get_tuning("checksum_split_adapt")
        res["policy_default"]["learned"] = sd.file_checksums_learned()
        res["policy_default"]["hybrid_threads"] = sd.get_tuning("checksum_hybrid_threads")
        tot = split_bytes["gpu"] + split_bytes["cpu_in_split"]
        res["policy_default"]["gpu_share"] = split_bytes["gpu"] / tot if tot else None
        res["policy_default_over_cpu_path"] = res["policy_default"]["GBps"] / res["library_cpu_path"]["GBps"]
        res["note"] = ("medians of 3 interleaved rounds after a warm one; policy_default splits this call between "
                       "the GPU route (hybrid_threads GPU slots) and the CPU path, or runs the CPU path alone where "
                       "this context measured it faster (split_adapt: after 4 learning calls -- each route's "
                       "uncounted warm-up and one counted call --, the faster, the other every split_adapt-th "
                       "call; per_call; DESIGN.md §4.1)")
        from oracle import native
        bad = sum(native.checksum_synth_mt(flen, 30_000 + i, 0, nthreads=oracle_threads()).hex() != want[i]
                  for i in range(nf))
        res["parity"] = parity(nf, bad, "every file's checksum vs the C oracle's chunk-parallel BLAKE3 of the same "
                                        "content")
        res["gpu"]["note"] = ("sd_file_checksums, GPU route: hash.rs's 1 MiB reads as parallel preads streamed into "
                              "256 MiB pinned windows, two slots alternating (reads overlap H2D + kernels)")
        for nt, key in ((effective_cpus(), "library_cpu_path_all_cores"),):
            cpu_runs = []
            for _ in range(2):
                t0 = time.perf_counter()
                lib_cpu = sd.cpu.file_checksums(paths, nthreads=nt)
                cpu_runs.append(time.perf_counter() - t0)
            res[key] = {"GBps": total / min(cpu_runs) / 1e9, "threads": nt, "note": "best of 2"}
            assert lib_cpu == want
        if with_cpu:
            from oracle import native
            cpu = {}
            for nt in sorted({1, 16, effective_cpus()}):
                sub = paths[:4] if nt == 1 else paths  # one thread: a bounded sample (1 GiB)
                t0 = time.perf_counter()
                got, st = native.file_checksums(sub, nthreads=nt, simd=-1)
                dt = time.perf_counter() - t0
                cpu[f"threads_{nt}"] = {"GBps": len(sub) * flen / dt / 1e9, "seconds": dt, "files": len(sub)}
                assert (st == 0).all() and [g.tobytes().hex() for g in got] == want[:len(sub)]
            res["cpu_reference_schedule"] = cpu
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def split_leg(ctx, comm, gib: int, rank: int, world: int, dev, stream, reps: int, warm_ms: float, tm=None,
              live: bool = False):
    """file_checksum (hash.rs:10-24) of ONE file spread over the ranks: rank r
    holds its contiguous run of 1 MiB blocks (sd_split_range), hashes them to block CVs, the
    CVs are all-gathered in place over libsdcas's RCCL communicator (32 B per MiB), and every
    rank reduces them to the file's hash (sd_split_checksum_mgpu).  Strong scaling: the file
    is the same at every N.  Timed with a barrier on both sides, max over ranks."""
    from spacedrive_amd.device import SplitChecksum
    total = (gib << 30) + 12345  # not block-aligned: the last rank's final block is partial
    sc = SplitChecksum(ctx, total, world, rank)
    d_slice = torch.zeros(sc.len + 128, dtype=torch.uint8, device=dev)
    if sc.len:
        ctx.synth_fill(20_000, 0, sc.len, d_slice, offset=sc.offset)
    cvs = torch.zeros(sc.cv_bytes, dtype=torch.uint8, device=dev)
    out32 = torch.zeros(32, dtype=torch.uint8, device=dev)
    if comm is not None:
        def run():
            sc.mgpu(comm, d_slice, cvs, out32, stream)
    elif world == 1:
        def run():
            sc.leaves(d_slice, cvs, stream)
            sc.root(cvs, out32, stream)
    else:  # rehearsal transport (gloo): the CV slots gathered through host memory
        from spacedrive_amd.split import _gather_slots
        q = sc.cv_bytes // (32 * world)

        def run():
            sc.leaves(d_slice, cvs, stream)
            h = cvs.cpu()
            _gather_slots(h, rank, world, q, None)
            cvs.copy_(h)
            sc.root(cvs, out32, stream)
    run()
    if world == 1:
        warm(run, stream, warm_ms)
    else:  # run() is a collective: every rank must call it the same number of times
        for _ in range(3):
            run()
    torch.cuda.synchronize()
    if DIST:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev if comm is not None else "cpu")
    if DIST:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    wall_ms = float(dt.item()) / reps * 1e3
    leaves_ms = ev_ms(lambda: sc.leaves(d_slice, cvs, stream), stream, reps=reps)
    res = {"file_bytes": total, "ranks": world, "blocks": (total + (1 << 20) - 1) >> 20,
           "ms_per_file": wall_ms, "GBps": total / (wall_ms * 1e-3) / 1e9, "scaling": "strong",
           "rank0_leaves_ms": leaves_ms, "rank0_bytes": sc.len,
           "rank0_leaves_GBps": sc.len / (leaves_ms * 1e-3) / 1e9 if sc.len else None,
           "transport": "rccl" if comm is not None else ("none (N=1)" if world == 1 else
                                                         f"{dist.get_backend()} via host (rehearsal)"),
           "note": "one file over all ranks: per-rank block CVs, the CV slots gathered in rank order ("
                   + ("in-place ncclAllGather inside sd_split_checksum_mgpu over RCCL" if comm is not None else
                      "no gather at N = 1" if world == 1 else
                      "through host memory over the process group: a rehearsal transport, not RCCL")
                   + "), reduce on every rank; wall time with barriers, max over ranks"}
    h = out32.clone() if comm is not None else out32.cpu()
    if DIST:  # every rank must hold the same hash
        allh = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(allh, h)
        res["ranks_agree"] = all(torch.equal(x, h) for x in allh)
        assert res["ranks_agree"], "the ranks' split checksums differ"
    res["hash"] = bytes(h.cpu().numpy()).hex()
    if tm is not None:
        tm.lap("split")
    if rank == 0:  # the file's hash against the oracle's BLAKE3 of the same content
        want, src = synth_checksum_expected(20_000, total, live)
        res["parity"] = parity(1, int(want != res["hash"]), "the file's checksum vs the C oracle's chunk-parallel "
                                                             "BLAKE3 of the same content (rank 0)", expected_from=[src])
    if tm is not None:
        tm.lap("split_oracle_check")
    sc.close()
    del d_slice, cvs
    torch.cuda.empty_cache()
    return res


# ------------------------------------------------------------------ wall time per leg
class Timing(dict):
    """Wall seconds per leg of this rank's run: lap(name) charges the
    time since the previous lap to `name`."""

    def __init__(self):
        super().__init__()
        self._t = time.perf_counter()

    def lap(self, name: str) -> None:
        now = time.perf_counter()
        self[name] = round(self.get(name, 0.0) + now - self._t, 3)
        self._t = now


# ------------------------------------------------------------------ multi-GiB oracle checks
GOLDEN_CHECKSUMS = os.path.join(ROOT, "tests", "golden", "bench_checksums.json")
_golden = None


def golden_checksums() -> dict:
    """tests/golden/bench_checksums.json: the C oracle's checksums of the bench's multi-GiB
    synthetic files (configs[3]'s files 0 and 15 of every rank's shard, each rank's shortest
    mixed file, the split file), written by tests/golden/make_bench_golden.py from the same
    deterministic generator; tests/test_bench_helpers.py re-derives some of them with the
    oracle on every CPU run.  Empty when absent."""
    global _golden
    if _golden is None:
        try:
            with open(GOLDEN_CHECKSUMS) as f:
                _golden = json.load(f)
        except OSError:
            _golden = {}
    return _golden


def mixed_layout(start: int, total: int):
    """configs[3]'s mixed variant: files of 2..8 GiB (unaligned lengths) packed at 128-B
    starts (SD_STAGE_ALIGN, profiles/r2/r2z5_ck_align.json) in the first `total` bytes of the
    buffer that holds the rank's 16 generated files; seeded by the rank's first file index."""
    rng = np.random.default_rng(7 + start)
    offs, lens, pos = [], [], 0
    while True:
        ln = int(rng.integers(2 << 30, (8 << 30) + 1))
        if pos + ln > total:
            break
        offs.append(pos)
        lens.append(ln)
        pos = (pos + ln + 127) // 128 * 128
    return offs, lens


def cas_digest(ids8: np.ndarray) -> str:
    """SHA-256 of n cas_ids (the first 8 hash bytes of each file, in file order): one value
    that equals the oracle's only if every one of the n cas_ids does."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(ids8, np.uint8).tobytes()).hexdigest()


def library_digest_key(start: int, n: int, n_total: int) -> str:
    return f"library:{start}:{n}:{n_total}"


def config_digest_key(which: str, n: int) -> str:
    return f"configs:{which}:{n}"


def full_parity(d_hash: torch.Tensor, n: int, key: str, gen, live: bool) -> dict:
    """ALL n cas_ids of a timed output against the oracle (a 4 096-file sample
    is 0.4 % of a leg): their SHA-256 against the committed digest of the oracle's cas_ids
    (tests/golden/bench_checksums.json, make_bench_golden.py), or -- for a workload the
    goldens do not hold, with --oracle-live, or to locate a mismatch -- the oracle's own
    cas_ids computed here from gen() = (sizes, cids, twins)."""
    got = d_hash.view(-1, 32)[:n, :8].cpu().numpy()
    want_digest = golden_checksums().get("cas_digest", {}).get(key)
    if want_digest and not live:
        ok = cas_digest(got) == want_digest
        if ok:
            return {"files": n, "mismatches": 0, "oracle": "SHA-256 of all n cas_ids == the committed digest of "
                                                             "the C oracle's (oracle/sd_oracle_simd.c)",
                    "expected_from": "golden", "key": key}
    from oracle import native
    s, c, t = gen()
    want = native.cas_ids_synth_simd(s, c, t, nthreads=oracle_threads())
    bad = np.nonzero((got != want).any(axis=1))[0]
    return {"files": n, "mismatches": int(len(bad)), "first_bad_index": int(bad[0]) if len(bad) else None,
            "oracle": "all n cas_ids vs the C oracle's (oracle/sd_oracle_simd.c) on the same generator",
            "expected_from": "oracle (live)", "key": key,
            "digest_mismatch": bool(want_digest) and not live}


def synth_checksum_expected(cid: int, length: int, live: bool):
    """(hex, source) of BLAKE3 over synthetic file `cid`'s first `length` bytes: the committed
    oracle output when it holds this file, else the C oracle on this host (this rank's share
    of its threads)."""
    g = golden_checksums().get("synth", {}).get(f"{cid}:{length}")
    if g and not live:
        return g, "golden"
    from oracle import native
    return native.checksum_synth_mt(length, cid, 0, nthreads=oracle_threads()).hex(), "oracle (live)"


def mixed_expected(start: int, total: int, mi: int, off: int, ln: int, flen: int, live: bool):
    """(hex, source) of mixed file `mi` -- bytes [off, off + ln) of the concatenation of the
    rank's 16 generated files of flen bytes (cids 10000 + start + i)."""
    g = golden_checksums().get("mixed", {}).get(f"{start}:{total}")
    if g and not live and g["index"] == mi and g["offset"] == off and g["len"] == ln:
        return g["hash"], "golden"
    from oracle import native
    return mixed_host_checksum(start, off, ln, flen, oracle_threads()).hex(), "oracle (live)"


def mixed_host_checksum(start: int, off: int, ln: int, flen: int, nthreads: int) -> bytes:
    """The oracle's checksum of a mixed file, its bytes generated on the host piece by piece
    from the generated files it spans."""
    from oracle import native
    buf = np.empty(ln, np.uint8)
    pos = off
    while pos < off + ln:
        i, o = divmod(pos, flen)
        n = min(flen - o, off + ln - pos)
        native.lib().sdo_synth_fill(10_000 + start + i, 0, o, n, buf[pos - off:].ctypes.data)
        pos += n
    return native.checksum_mt(buf, ln, nthreads=nthreads)


def end_to_end_summary(out: dict) -> dict:
    """The end-to-end rows beside the library's own CPU path on the same host threads, with
    the share of the work host threads did in each, copied into
    cpu_baseline so the driver's record keeps them."""
    s = {}
    h = out.get("with_h2d", {})
    if "cas" in h and "library_cpu_path" in h["cas"]:
        c = h["cas"]
        s["with_h2d_cas"] = {"unit": "files/s", "default": c["end_to_end_files_per_s"],
                             "gpu_only": c["gpu_only"]["end_to_end_files_per_s"],
                             "library_cpu_path": c["library_cpu_path"]["files_per_s"],
                             "ratio": c["library_cpu_path"]["default_over_cpu_path"],
                             "host_share": c.get("host_share"), "host_threads": c.get("host_cohash_threads")}
    if "checksum" in h and "library_cpu_path" in h["checksum"]:
        c = h["checksum"]
        s["with_h2d_checksum"] = {"unit": "GB/s", "default": c["end_to_end_GBps"],
                                  "gpu_only": c["gpu_only"]["end_to_end_GBps"],
                                  "library_cpu_path": c["library_cpu_path"]["GBps"],
                                  "ratio": c["default_over_cpu_path"], "host_share": c.get("host_share"),
                                  "host_threads": c.get("host_cohash_threads")}
    fb = out.get("file_backed", {})
    if "gpu" in fb and "library_cpu_path" in fb:
        s["file_backed_cas"] = {"unit": "files/s", "gpu_route": fb["gpu"]["files_per_s"],
                                "library_cpu_path": fb["library_cpu_path"]["files_per_s"],
                                "ratio": fb.get("gpu_over_cpu_path_16_threads"), "host_share_of_hashing": 0.0,
                                "note": "the GPU route hashes every file on the device; its host threads read"}
    fc = out.get("file_backed_checksum", {})
    if "policy_default" in fc and "library_cpu_path" in fc:
        s["file_backed_checksum"] = {"unit": "GB/s", "default": fc["policy_default"]["GBps"],
                                     "gpu_route": fc.get("gpu", {}).get("GBps"),
                                     "library_cpu_path": fc["library_cpu_path"]["GBps"],
                                     "ratio": fc.get("policy_default_over_cpu_path"),
                                     "host_share": (1.0 - fc["policy_default"]["gpu_share"])
                                     if fc["policy_default"].get("gpu_share") is not None else None}
    return s


# ------------------------------------------------------------------ the stdout line
# The driver lost round 5's 24.4 KB line (BENCH_r05 "parsed": null) and keeps an 8.4 KB
# stdout tail: stdout carries a compact line well inside both, the full record goes to a file.
LINE_BUDGET = 16384
LINE_TARGET = 8000
STD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _sig(o, digits: int = 4):
    """floats to `digits` significant digits, recursively (the line's size, not its meaning)"""
    if isinstance(o, float):
        return float(f"{o:.{digits}g}")
    if isinstance(o, dict):
        return {k: _sig(v, digits) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_sig(v, digits) for v in o]
    return o


def _g(d, *path):
    for k in path:
        if not isinstance(d, dict):
            return None
        d = d.get(k)
    return d


def _par(p):
    """a parity record as [files, mismatches]"""
    return [p.get("files"), p.get("mismatches")] if isinstance(p, dict) else None


def _prune(d):
    return {k: v for k, v in d.items() if v is not None and v != {}}


def compact_line(out: dict, full_path: str = None) -> dict:
    """The stdout line: the driver's standard keys complete and first, then `roofline`, then
    `cpu_baseline`, then one short record per leg.  Every prose note lives in DESIGN.md §6
    (the field glossary); `basis` codes name the peak's evidence.  Values are the full
    record's, rounded to 4 significant digits (the ones the value and ms_per_step keep)."""
    c = {k: out.get(k) for k in STD_KEYS}
    r = out.get("roofline") or {}
    clock = r.get("clock") or {}
    c["roofline"] = _prune({
        "bound": r.get("bound"), "achieved": r.get("achieved"), "peak": r.get("peak"), "unit": r.get("unit"),
        "frac": r.get("frac"), "frac_full_rate": r.get("frac_full_rate"), "peak_full_rate": r.get("peak_full_rate"),
        "basis": "probe7 G-mix 64 lane-ops/clk/CU; full rate 128", "traffic": r.get("traffic"),
        "algorithmic_bytes": _g(r, "algorithmic", "bytes_per_launch"),
        "kernel": r.get("kernel"), "kernel_ms": r.get("kernel_ms"), "kernel_events": r.get("kernel_events"),
        "issue_rate_pmc_frac": _g(r, "issue_rate_pmc", "frac"),
        "lane_ops_per_clk_cu": _g(r, "issue_rate_pmc", "lane_ops_per_clk_cu"),
        "sclk_mhz_median": clock.get("sclk_mhz_median"), "board_power_w": clock.get("board_power_w_median"),
        "frac_at_clock": r.get("frac_of_issue_ceiling_at_clock"), "frac_of_measured_peak": r.get("frac_of_measured_peak"),
        "hbm_GBps": _g(r, "hbm", "achieved"), "hbm_frac": _g(r, "hbm", "frac"),
        "phase": _prune({k: _g(r, "phase", k) for k in ("ms", "achieved", "frac", "frac_full_rate")})})
    cb = out.get("cpu_baseline")
    if cb:
        e2e = {}
        for k, v in (cb.get("end_to_end_vs_library_cpu_path") or {}).items():
            e2e[k] = _prune({"unit": v.get("unit"), "default": v.get("default", v.get("gpu_route")),
                             "gpu_only": v.get("gpu_only"), "cpu_path": v.get("library_cpu_path"),
                             "ratio": v.get("ratio"), "host_share": v.get("host_share", v.get("host_share_of_hashing"))})
        c["cpu_baseline"] = _prune({
            "value": cb.get("value"), "unit": cb.get("unit"), "cores": cb.get("cores"), "kind": cb.get("kind"),
            "sample": (f"first {cb['sample_files']} files of the shard" if cb.get("sample_files") else
                       "a prefix of the shard") + ", messages in host RAM, hash only (oracle AVX-512 hash_many)",
            "single_thread": _g(cb, "single_thread", "value"), "all_cores": _g(cb, "all_cores", "value"),
            "all_cores_threads": _g(cb, "all_cores", "cores"), "simd": cb.get("simd"),
            "host_cpu": _g(cb, "host_cpu", "model"), "cgroup_cpu_quota": _g(cb, "host_cpu", "cgroup_cpu_quota"),
            "file_backed_16t": _g(cb, "file_backed", "threads_16", "files_per_s"),
            "end_to_end": e2e or None})
    legs = {}
    for k, v in (out.get("configs") or {}).items():
        legs["configs_" + k] = _prune({
            "files_per_s": v.get("files_per_s"), "kernel_ms": v.get("kernel_ms"), "valu_frac": v.get("valu_frac"),
            "frac_full_rate": v.get("valu_frac_full_rate"), "issue_rate_pmc_frac": _g(v, "issue_rate_pmc", "frac"),
            "sclk_mhz": _g(v, "clock", "sclk_mhz_median"), "traffic": v.get("traffic"),
            "msg_GBps": v.get("msg_GBps"), "parity": _par(v.get("parity")), "parity_full": _par(v.get("parity_full"))})
    ck = out.get("checksum")
    if ck:
        legs["checksum"] = _prune({
            "GBps": ck.get("GBps"), "per_gpu_GBps": ck.get("per_gpu_GBps"), "ms": ck.get("ms_per_run"),
            "valu_frac": _g(ck, "roofline", "frac"), "frac_full_rate": _g(ck, "roofline", "frac_full_rate"),
            "issue_rate_pmc_frac": _g(ck, "roofline", "issue_rate_pmc", "frac"),
            "hbm_frac": _g(ck, "roofline", "hbm", "frac"), "traffic": ck.get("traffic"),
            "parity": _par(ck.get("parity")), "mixed_GBps": _g(ck, "mixed", "GBps"),
            "mixed_parity": _par(_g(ck, "mixed", "parity"))})
    sp = out.get("checksum_one_file")
    if sp:
        legs["checksum_one_file"] = _prune({"GBps": sp.get("GBps"), "ms": sp.get("ms_per_file"),
                                            "bytes": sp.get("file_bytes"), "ranks": sp.get("ranks"),
                                            "transport": sp.get("transport"), "parity": _par(sp.get("parity"))})
    h = out.get("with_h2d") or {}
    for k, v in h.items():
        legs["with_h2d_" + k] = _prune({
            "end_to_end": v.get("end_to_end_files_per_s", v.get("end_to_end_GBps")),
            "unit": "files/s" if "end_to_end_files_per_s" in v else "GB/s",
            "gpu_only": _g(v, "gpu_only", "end_to_end_files_per_s") or _g(v, "gpu_only", "end_to_end_GBps"),
            "h2d_GBps": v.get("h2d_GBps"), "kernel_ms": v.get("kernel_ms"), "host_share": v.get("host_share"),
            "host_threads": v.get("host_cohash_threads"),
            # N > 1: every rank at once, all ranks' files over the slowest rank's time
            "aggregate_files_per_s": _g(v, "aggregate", "files_per_s"), "aggregate_GBps": _g(v, "aggregate", "GBps"),
            "parity": _par(v.get("parity"))})
    fb = out.get("file_backed")
    if fb:
        legs["file_backed"] = _prune({"files_per_s": _g(fb, "gpu", "files_per_s"),
                                      "cpu_path": _g(fb, "library_cpu_path", "files_per_s"),
                                      "ratio": fb.get("gpu_over_cpu_path_16_threads"), "parity": _par(fb.get("parity")),
                                      "identifier_hash_speedup": _g(fb, "identifier_job", "hash_speedup"),
                                      "identifier_same_objects": _g(fb, "identifier_job", "same_objects")})
    fc = out.get("file_backed_checksum")
    if fc:
        legs["file_backed_checksum"] = _prune({"GBps": _g(fc, "policy_default", "GBps"), "gpu": _g(fc, "gpu", "GBps"),
                                               "cpu_path": _g(fc, "library_cpu_path", "GBps"),
                                               "ratio": fc.get("policy_default_over_cpu_path"),
                                               "parity": _par(fc.get("parity"))})
    lat = out.get("latency")
    if lat:
        legs["latency_us"] = {k: [_g(v, "idle", "p50_us"), _g(v, "idle", "p99_us"),
                                  _g(v, "concurrent_64", "p50_us"), _g(v, "concurrent_64", "p99_us")]
                              for k, v in lat.items() if isinstance(v, dict)}
    c["legs"] = legs
    ps, pf = out.get("parity_sample") or {}, out.get("parity_full") or {}
    c["parity"] = _prune({"sample": _par(ps), "full": _par(pf), "full_from": pf.get("expected_from"),
                          "ranks": pf.get("ranks")})
    d = out.get("dedup") or {}
    c["dedup"] = _prune({"records": d.get("records"), "groups": d.get("groups"), "valid_files": d.get("valid_files"),
                         "records_per_rank": d.get("records_per_rank"), "transport": d.get("transport"),
                         "parity": d.get("parity"), "phases_ms_max": d.get("phases_ms_max_over_ranks"),
                         "transport_note": d.get("transport_note")})
    di = out.get("distributed") or {}
    rl = di.get("rccl_libs") or {}
    c["distributed"] = _prune({"world": di.get("world"), "backend": di.get("backend"),
                               "dedup_transport": di.get("dedup_transport"), "force_dist": di.get("force_dist"),
                               "rccl_libs": _prune({"one_rccl": rl.get("one_rccl"),
                                                    "version": _g(rl, "sdcas_comm", "version"),
                                                    "mapped": len(rl.get("mapped") or [])}) if rl else None})
    pl, se = out.get("steps_pipelined") or {}, out.get("steps_serial") or {}
    c["steps"] = out.get("steps")
    c["kernels"] = _prune({"pipelined_value": pl.get("value"), "serial_value": se.get("value"),
                           **{k: v for k, v in (out.get("kernels") or {}).items() if k != "note"}})
    t = out.get("timing") or {}
    c["timing"] = _prune({"rank0_total_s": t.get("rank0_total_s"), "rank0_process_s": t.get("rank0_process_s"),
                          "total_s_max_over_ranks": t.get("total_s_max_over_ranks"),
                          "host_threads_budget": t.get("host_threads_budget")})
    c["launch"] = out.get("launch")
    if full_path:
        c["full_record"] = full_path
    c = _sig(c)
    # the contract's numbers keep full precision (the driver's own consistency checks use them)
    c["value"], c["ms_per_step"] = out.get("value"), out.get("ms_per_step")
    return c


def emit(out: dict, stream, full_path: str = None) -> str:
    """Writes the full record to `full_path` (when given and writable) and the compact line to
    `stream`; returns the line.  Fails loudly when the line outgrows LINE_BUDGET."""
    if full_path:
        try:
            os.makedirs(os.path.dirname(full_path) or ".", exist_ok=True)
            with open(full_path, "w") as f:
                json.dump(out, f)
        except OSError as e:
            log(f"bench.py: could not write the full record to {full_path}: {e}")
            full_path = None
    line = json.dumps(compact_line(out, full_path), separators=(",", ":"))
    if len(line) > LINE_BUDGET:
        raise SystemExit(f"bench.py: the stdout line is {len(line)} B, over the {LINE_BUDGET} B budget")
    if len(line) > LINE_TARGET:
        log(f"bench.py: the stdout line is {len(line)} B (target {LINE_TARGET} B)")
    print(line, file=stream, flush=True)
    return line


# ------------------------------------------------------------------ main
def main():
    args = parse()
    mode = launch_mode(args.gpus, os.environ)
    if mode == "spawn":  # before any torch.cuda call: the ranks are children
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    t_main = time.perf_counter()
    if os.environ.get("SD_BENCH_STACKS_AFTER"):  # debugging a stuck run: dump every thread's stack
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["SD_BENCH_STACKS_AFTER"]), repeat=True)
    # stdout carries exactly one JSON line: anything native libraries print there (RCCL's
    # version banner at communicator init) goes to stderr instead
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    tm = Timing()
    if args.share_gpu:  # rehearsal of the N-rank path on a box with fewer GPUs
        local = local % torch.cuda.device_count()
    elif world > 1 and local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: local rank {local} of {world} but {torch.cuda.device_count()} visible GPUs "
                         f"(--share-gpu maps several ranks onto one GPU: a rehearsal)")
    torch.cuda.set_device(local)
    global DIST
    if world > 1 or args.force_dist:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
        DIST = True
    # collectives' tensors live where the backend wants them
    cdev = torch.device("cuda", local) if DIST and args.dist_backend == "nccl" else torch.device("cpu")
    transport = args.dedup or ("rccl" if args.dist_backend == "nccl" else "torch")
    import spacedrive_amd as sd
    from spacedrive_amd import _native, dedup, synth
    if args.host_cpu_budget > 0:
        sd.set_tuning("host_cpu_budget", args.host_cpu_budget)

    ctx = sd.Context(local)
    n = args.files_per_gpu
    start, n_total = rank * n, world * n
    t_setup = time.time()
    sizes, cids, twins = synth.library(start, n, n_total)
    ext, total = sd.stage_plan(sizes)
    dev = torch.device("cuda", local)
    d_staged = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                        torch.from_numpy(twins.astype(np.int32)).to(dev), d_ext, n, d_staged)
    batch = ctx.cas_batch(ext)
    d_hash = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    d_valid = torch.from_numpy((sizes != 0).astype(np.uint8)).to(dev)  # size 0: no cas_id (mod.rs:80-88)
    comm = rccl = None
    transport_note = None
    if transport == "rccl":
        err = None
        try:
            comm = dedup.make_comm(ctx)
            rccl = dedup.RcclDedup(ctx, comm, dev, capacity=n * 5 // 4 + 4096)
        except Exception as e:  # noqa: BLE001 -- recorded in the output line, never silent
            err = f"sd_comm_create failed on rank {rank}: {e}"
        ok = torch.tensor([0 if err else 1], device=cdev)
        if DIST:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)  # every rank takes the same transport
        if not int(ok.item()):
            log(f"[rank {rank}] {err or 'a peer rank failed sd_comm_create'}; exchanging through torch.distributed")
            transport, transport_note = "torch", err or "a peer rank failed sd_comm_create"
            comm = rccl = None
    if rccl is None:
        ascending = dedup.shards_ascend(n, start, None, cdev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.time() - t_setup:.1f}s: {n} files ({batch.n_sampled} sampled), "
        f"{batch.msg_bytes / 1e9:.2f} GB of messages, {batch.compressions / 1e9:.3f} G compressions, "
        f"dedup transport {transport}")

    stream = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]

    def step(k=None):
        if k is not None:
            ev[k][0].record(stream)
        batch.run_part(1, d_staged, d_hash, stream)  # the sampled kernels, timed on their own
        if k is not None:
            ev[k][1].record(stream)
        batch.run_part(2, d_staged, d_hash, stream)  # k_whole_items + 2 x k_whole_merge8
        if k is not None:
            ev[k][2].record(stream)
        if rccl is not None:
            r = rccl(d_hash.view(n, 32), d_valid, n, start, stream=stream)
        else:
            r = dedup.dedup_shard(ctx, d_hash.view(n, 32), d_valid, n, start, index_sorted=ascending)
        if k is not None:
            ev[k][3].record(stream)
        return r

    tm.lap("setup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if DIST:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        res = step(k)
    torch.cuda.synchronize()
    if DIST:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if DIST:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    def avg(a, b):
        return sum(ev[k][a].elapsed_time(ev[k][b]) for k in range(args.steps)) / args.steps

    hash_ms, sampled_ms, dedup_ms = avg(0, 2), avg(0, 1), avg(2, 3)
    recs, rep, n_groups, owners = res
    # every valid file lands on exactly one rank; groups never straddle ranks
    tot = torch.tensor([recs.shape[0], n_groups, int((sizes != 0).sum())], dtype=torch.int64, device=cdev)
    if DIST:
        dist.all_reduce(tot)
    # the exchange's balance: records each rank groups after the prefix all-to-all
    per_rank = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(world)]
    mine = torch.tensor([recs.shape[0]], dtype=torch.int64, device=cdev)
    if DIST:
        dist.all_gather(per_rank, mine)
    else:
        per_rank = [mine]
    dedup_totals = {"records": int(tot[0]), "groups": int(tot[1]), "valid_files": int(tot[2]),
                    "records_per_rank": [int(x.item()) for x in per_rank],
                    "records_on_rank0": int(recs.shape[0]),
                    "objects_created_on_rank0": int((owners == recs[:, 1]).sum()), "transport": transport}
    if transport_note:
        dedup_totals["transport_note"] = transport_note
    assert dedup_totals["records"] == dedup_totals["valid_files"], dedup_totals
    files_total = n_total * args.steps
    s_hash_ms, s_sampled_ms = hash_ms, sampled_ms
    serial = {"value": files_total / elapsed, "ms_per_step": elapsed / args.steps * 1e3,
              "note": "each step's hashing, then its dedup, on one stream (the kernel breakdown below)"}
    value = serial["value"]
    pipelined = None
    clock_res = None
    if rccl is not None and not args.no_overlap:
        # The same K steps as an indexer runs consecutive batches: batch k's exchange and
        # grouping (sd_cas_dedup_mgpu, its host syncs, the RCCL collectives) on one stream
        # while batch k+1 hashes on another; two hash buffers alternate.
        # The hashing stream has the higher priority: the exchange's small kernels then fill in
        # around the hash kernels' workgroups instead of taking CUs from them first (A/B,
        # profiles/r4/r4u_stream_prio_ab/: 107.5-107.7 M files/s against 103.9-104.3 M with equal
        # priorities and 103.6-104.0 M with the exchange first; the serial steps 105.2-105.6 M)
        hs = torch.cuda.Stream(device=dev, priority=-1)
        ds = torch.cuda.Stream(device=dev, priority=0)
        d_hash2 = [d_hash, torch.empty_like(d_hash)]
        ser = (recs.clone(), owners.clone())  # the runner's output buffers are reused by every call
        e_hash = [torch.cuda.Event() for _ in range(2)]
        e_ded = [torch.cuda.Event() for _ in range(2)]
        ded_seen = [False, False]

        pev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

        def hash_into(b, k=None):  # k: the timed step whose kernel events to record
            if ded_seen[b]:  # the exchange that read this buffer is done with it
                hs.wait_event(e_ded[b])
            if k is not None:
                pev[k][0].record(hs)
            batch.run_part(1, d_staged, d_hash2[b], hs)  # the sampled kernels, timed on their own
            if k is not None:
                pev[k][1].record(hs)
            batch.run_part(2, d_staged, d_hash2[b], hs)
            if k is not None:
                pev[k][2].record(hs)
            e_hash[b].record(hs)

        def pipelined_steps(K, timed=False):
            r = None
            hash_into(0, 0 if timed else None)
            for k in range(K):
                b = k & 1
                if k + 1 < K:
                    hash_into(b ^ 1, k + 1 if timed else None)
                ds.wait_event(e_hash[b])
                r = rccl(d_hash2[b].view(n, 32), d_valid, n, start, stream=ds)
                e_ded[b].record(ds)
                ded_seen[b] = True
            return r

        tm.lap("steps_serial")
        pipelined_steps(args.warmup)
        torch.cuda.synchronize()
        if DIST:
            dist.barrier()
        torch.cuda.synchronize()
        clock = ClockSampler(dev.index if dev.index is not None else 0).start()
        t0 = time.perf_counter()
        pres = pipelined_steps(args.steps, timed=True)
        torch.cuda.synchronize()
        if DIST:
            dist.barrier()
        p_elapsed = time.perf_counter() - t0
        clock_res = clock.result()
        if DIST:
            t = torch.tensor([p_elapsed], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            p_elapsed = float(t.item())
        # the last batch's exchange gives the serial pass's result exactly
        same = (pres[2] == n_groups and pres[0].shape == ser[0].shape and torch.equal(pres[0], ser[0])
                and torch.equal(pres[3], ser[1]))
        del d_hash2, ser
        p_sampled = sum(pev[k][0].elapsed_time(pev[k][1]) for k in range(args.steps)) / args.steps
        p_hash = sum(pev[k][0].elapsed_time(pev[k][2]) for k in range(args.steps)) / args.steps
        pipelined = {"value": files_total / p_elapsed, "ms_per_step": p_elapsed / args.steps * 1e3,
                     "equal_to_serial": bool(same), "sampled_ms": p_sampled, "hash_ms": p_hash,
                     "note": "batch k's dedup (sd_cas_dedup_mgpu) on one stream while batch k+1 hashes on "
                             "another; the value"}
        assert same, "the pipelined steps' dedup differs from the serial steps'"
        value, elapsed = pipelined["value"], p_elapsed
        # the roofline comes from the timed region that gives `value`: these steps' own events
        sampled_ms, hash_ms = p_sampled, p_hash

    # roofline of the dominant kernels, the sampled pair k_cas_sampled_lanes + _merge (81 % of
    # the shard's compressions, one unit: the merge finishes what the lanes kernel starts),
    # timed on its own with HIP events on its launch stream: 953 compressions x 672 VALU
    # lane-ops per sampled file; bytes = 57 352 B message read + 32 B hash written per file
    valu_peak = ctx.valu_peak()
    dom_comp = 953 * batch.n_sampled
    dom_bytes = batch.n_sampled * (SAMPLED_MSG + 32)
    dom = valu_roof(dom_comp, sampled_ms)
    dom_gbps = dom_bytes / (sampled_ms * 1e-3) / 1e9
    hash_bytes = batch.msg_bytes + 32 * n
    phase_roof = valu_roof(batch.compressions, hash_ms)
    s_grid, w_grid = sampled_grids(batch.n_sampled), whole_grid(batch)
    tr = pmc_traffic_sum(SAMPLED_KERNELS, s_grid)
    tr_w = pmc_traffic("k_whole_items", w_grid)
    out = {
        "metric": "cas_id files/sec (10M synthetic files) + checksum GB/s at 1/2/4/8 MI355X",
        "value": value, "unit": "files/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic (device-generated, SURVEY.md 8(d) generator)",
        "config": {"workload": f"10M-file library mixture (configs[0] mix: 60% <=100KiB whole-content, 40% sampled; "
                               f"10% dups, 1% sample twins), {n} files per GPU, step = hash shard + "
                               f"cas_id-prefix all-to-all dedup ({transport}) + Object owners (chunk-of-100 rule)",
                   "files_per_gpu": n, "global_files": n_total, "parallelism": f"file-sharded x{world}"},
        "roofline": {"bound": "valu", "achieved": dom["achieved"], "peak": VALU_PEAK_TOPS,
                     "unit": "T int32 VALU lane-ops/s", "frac": dom["frac"], "peak_basis": PEAK_BASIS,
                     "peak_full_rate": VALU_FULL_RATE_TOPS, "frac_full_rate": dom["frac_full_rate"],
                     "traffic": tr["bytes"] if tr else None, "traffic_source": tr,
                     "kernel": " + ".join(SAMPLED_KERNELS), "kernel_ms": sampled_ms, "launch_grid": s_grid,
                     "kernel_events": "steps_pipelined" if pipelined else "steps_serial",
                     "algorithmic": {"compressions_per_launch": dom_comp, "lane_ops_per_compression": 672,
                                     "bytes_per_launch": dom_bytes,
                                     "per_unit": "sampled file: 953 compressions, 57352 B read + 32 B written"},
                     "clock": clock_res,
                     "frac_of_issue_ceiling_at_clock": (
                         dom["achieved"] * 1e12 / (G_MIX_LANE_OPS_PER_CLK * N_CUS * clock_res["sclk_mhz_median"] * 1e6)
                         if clock_res else None),
                     "measured_valu_peak": valu_peak / 1e12,
                     "frac_of_measured_peak": dom["achieved"] * 1e12 / valu_peak if valu_peak else None,
                     "issue_rate_pmc": pmc_issue_rate(SAMPLED_KERNELS[0], s_grid[0]),
                     "hbm": {"achieved": dom_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                             "frac": dom_gbps / HBM_PEAK_GBPS},
                     "phase": {"kernels": SAMPLED_KERNELS + ["k_whole_items", "k_whole_merge8"], "ms": hash_ms,
                               "compressions": batch.compressions, "bytes": hash_bytes,
                               "achieved": phase_roof["achieved"], "frac": phase_roof["frac"],
                               "frac_full_rate": phase_roof["frac_full_rate"],
                               "whole_items_grid": w_grid, "whole_items_traffic": tr_w["bytes"] if tr_w else None}},
        "steps_serial": serial, "steps_pipelined": pipelined,
        "distributed": {"dist_initialized": DIST, "backend": dist.get_backend() if DIST else None, "world": world,
                        "force_dist": bool(args.force_dist), "dedup_transport": transport,
                        "rccl_libs": rccl_libs() if transport == "rccl" or args.dist_backend == "nccl" else None},
        "host_threads": dict(_native.host_cpu_budget(), numa=_native.host_numa(),
                             cohash_threads=min(sd.get_tuning("host_cohash_threads"),
                                                                         _native.host_cpu_budget()["budget"] - 1),
                             read_threads=min(sd.get_tuning("read_threads"), _native.host_cpu_budget()["budget"]),
                             note="the library's host thread budget (sd_host_cpu_budget): min(affinity, cgroup quota) "
                                  "/ LOCAL_WORLD_SIZE; every call's readers, CPU-path workers and co-hashing threads "
                                  "are capped by it"),
        "kernels": {"hash_ms": s_hash_ms, "sampled_ms": s_sampled_ms, "whole_ms": s_hash_ms - s_sampled_ms,
                    "dedup_and_exchange_ms": dedup_ms,
                    "host_overhead_ms": serial["ms_per_step"] - s_hash_ms - dedup_ms,
                    "sampled_files": batch.n_sampled, "whole_files": batch.n_whole,
                    "note": "the serial steps' event breakdown (steps_serial)"},
        "dedup": dedup_totals,
    }
    tm.lap("steps_pipelined" if pipelined else "steps_serial")
    # ---- the timed steps' output, checked (outside the timed regions) --------------------
    # (1) hashes: a fixed sample of every rank's shard against the C oracle
    ps = parity_sample(sizes, cids, twins, d_hash, start)
    bad = torch.tensor([ps["mismatches"], ps["files"]], dtype=torch.int64, device=cdev)
    if DIST:
        dist.all_reduce(bad)
    out["parity_sample"] = dict(ps, files=int(bad[1]), mismatches=int(bad[0]), ranks=world,
                                rank0_first_bad_global_index=ps["first_bad_global_index"])
    out["parity_sample"].pop("first_bad_global_index")
    # (1b) all of every rank's cas_ids: one digest per shard against the oracle's
    pf = full_parity(d_hash, n, library_digest_key(start, n, n_total), lambda: (sizes, cids, twins), args.oracle_live)
    bad = torch.tensor([pf["mismatches"], pf["files"], int(pf["expected_from"] == "golden")], dtype=torch.int64,
                       device=cdev)
    if DIST:
        dist.all_reduce(bad)
    out["parity_full"] = dict(pf, files=int(bad[1]), mismatches=int(bad[0]), ranks=world,
                              ranks_from_golden=int(bad[2]))
    assert out["parity_full"]["mismatches"] == 0, out["parity_full"]
    # (2) the exchange, grouping and Object owners: a key slice from every rank, on rank 0
    out["dedup"]["parity_slice"] = dedup_parity(d_hash, d_valid, n, start, recs, rep, owners, world, dev, transport)
    out["dedup"]["parity"] = out["dedup"]["parity_slice"]["parity"]
    # (3) where one exchange's time goes (one more serial call, events at its phases)
    if rccl is not None:
        comm.set_timing(True)
        torch.cuda.synchronize()
        if DIST:
            dist.barrier()
        rccl(d_hash.view(n, 32), d_valid, n, start, stream=stream)
        ph = comm.last_phases()
        comm.set_timing(False)
        pt = torch.tensor([ph[k] for k in comm.PHASES], dtype=torch.float64, device=cdev)
        if DIST:
            dist.all_reduce(pt, op=dist.ReduceOp.MAX)
        out["dedup"]["phases_ms"] = dict(ph, note="rank 0's call: partition, all-gather of the count rows + their "
                                                  "copy to the host, the stream's idle gap while the host reads them "
                                                  "and queues the exchange (the mid-call sync), grouped send/recv, "
                                                  "group + owners (HIP events on the call's stream)")
        out["dedup"]["phases_ms_max_over_ranks"] = {k: float(v) for k, v in zip(comm.PHASES, pt.tolist())}
    assert out["parity_sample"]["mismatches"] == 0, out["parity_sample"]
    assert out["dedup"]["parity"], out["dedup"]["parity_slice"]

    tm.lap("parity_steps")
    solo = rank == 0 and not DIST and not args.no_extras
    with_h2d = {}
    if args.host_staged_files > 0 and not args.no_extras:  # every rank: one PCIe link per GPU
        k_h2d = args.host_staged_files if not DIST else min(args.host_staged_files, 150_000)
        with_h2d["cas"] = host_staged(ctx, ext, d_staged, k_h2d, dev, stream, world, lib_=(sizes, cids, twins))
        tm.lap("with_h2d_cas")
    if solo and args.file_backed_files > 0:
        out["file_backed"] = file_backed(ctx, sizes, ext, d_staged, args.file_backed_files,
                                         with_cpu=not args.no_cpu_baseline, latency_calls=args.latency_calls,
                                         ident_files=args.identifier_files)
        if "latency" in out["file_backed"]:
            out["latency"] = out["file_backed"].pop("latency")
        tm.lap("file_backed")
    del d_staged, recs, rep, owners
    torch.cuda.empty_cache()

    tm.lap("release")
    # configs[3]: validator checksums, 16 files of (G/16) GiB per GPU
    if args.checksum_gib > 0:
        nf = 16
        flen = (args.checksum_gib << 30) // nf
        d_data = torch.empty(nf * flen + 128, dtype=torch.uint8, device=dev)
        offs = [i * flen for i in range(nf)]
        for i in range(nf):
            ctx.synth_fill(10_000 + start + i, 0, flen, d_data[offs[i]:])
        cb = ctx.checksum_batch(offs, [flen] * nf)
        d_sum = torch.empty(nf * 32, dtype=torch.uint8, device=dev)
        cb.run(d_data, d_sum, stream)
        warm(lambda: cb.run(d_data, d_sum, stream), stream, args.warm_ms)
        ck_clock = ClockSampler(dev.index if dev.index is not None else 0).start()
        ck_ms = ev_ms(lambda: cb.run(d_data, d_sum, stream), stream, reps=args.checksum_steps)
        ck_clock = ck_clock.result()
        gbps = cb.total_bytes / (ck_ms * 1e-3) / 1e9
        tot = torch.tensor([gbps], dtype=torch.float64, device=cdev)
        if DIST:
            dist.all_reduce(tot)
        roof = valu_roof(cb.compressions, ck_ms)
        tr_ck = pmc_traffic("k_ck_leaf", ck_leaf_grid(cb.blocks))
        out["checksum"] = {"GBps": float(tot.item()), "unit": "GB/s", "per_gpu_GBps": gbps, "ms_per_run": ck_ms,
                           "workload": f"configs[3]: {nf} x {flen >> 20} MiB files per GPU, full-file BLAKE3",
                           "roofline": {"bound": "valu", "achieved": roof["achieved"], "peak": VALU_PEAK_TOPS,
                                        "unit": "T int32 VALU lane-ops/s", "frac": roof["frac"],
                                        "frac_full_rate": roof["frac_full_rate"], "peak_basis": PEAK_BASIS,
                                        "clock": ck_clock,
                                        "frac_of_issue_ceiling_at_clock": (
                                            roof["achieved"] * 1e12
                                            / (G_MIX_LANE_OPS_PER_CLK * N_CUS * ck_clock["sclk_mhz_median"] * 1e6)
                                            if ck_clock else None),
                                        "issue_rate_pmc": pmc_issue_rate("k_ck_leaf", ck_leaf_grid(cb.blocks)),
                                        "hbm": {"achieved": gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                                "frac": gbps / HBM_PEAK_GBPS}},
                           "launch_grid": ck_leaf_grid(cb.blocks), "traffic": tr_ck["bytes"] if tr_ck else None}
        tm.lap("checksum")
        # the timed output against the oracle: two of the 16 files (the first and the last)
        sums = d_sum.cpu().numpy().reshape(nf, 32)
        chk = [0, nf - 1]
        exp = [synth_checksum_expected(10_000 + start + i, flen, args.oracle_live) for i in chk]
        bad = sum(e[0] != sums[i].tobytes().hex() for e, i in zip(exp, chk))
        out["checksum"]["parity"] = parity(len(chk), bad, "files 0 and 15 of the timed batch vs the C oracle's "
                                                          "chunk-parallel BLAKE3 of the same content", checked=chk,
                                           expected_from=sorted({e[1] for e in exp}))
        tm.lap("checksum_oracle_check")
        # configs[3]'s mixed variant: files of 2..8 GiB (unaligned lengths) in the same buffer
        m_offs, m_lens = mixed_layout(start, nf * flen)
        if m_lens:
            cbm = ctx.checksum_batch(m_offs, m_lens)
            d_msum = torch.empty(len(m_lens) * 32, dtype=torch.uint8, device=dev)
            cbm.run(d_data, d_msum, stream)
            mx_ms = ev_ms(lambda: cbm.run(d_data, d_msum, stream), stream, reps=args.checksum_steps)
            mroof = valu_roof(cbm.compressions, mx_ms)
            tm.lap("checksum_mixed")
            # one mixed file (the shortest: each spans parts of two generated files) against
            # the oracle hashing the same bytes, generated on the host
            mi = int(np.argmin(m_lens))
            want_m, src_m = mixed_expected(start, nf * flen, mi, m_offs[mi], m_lens[mi], flen, args.oracle_live)
            mbad = int(want_m != d_msum[32 * mi:32 * mi + 32].cpu().numpy().tobytes().hex())
            out["checksum"]["mixed"] = {
                "workload": f"configs[3] mixed: {len(m_lens)} files of 2..8 GiB, unaligned lengths, "
                            f"packed at 128-B (SD_STAGE_ALIGN) starts",
                "files": len(m_lens), "bytes": cbm.total_bytes, "ms_per_run": mx_ms,
                "GBps": cbm.total_bytes / (mx_ms * 1e-3) / 1e9, "frac": mroof["frac"],
                "frac_full_rate": mroof["frac_full_rate"],
                "parity": parity(1, mbad, f"mixed file {mi} ({m_lens[mi]} B, the shortest) vs the C oracle's "
                                          "chunk-parallel BLAKE3 of the same bytes", expected_from=[src_m])}
            del cbm, d_msum
            tm.lap("checksum_mixed_oracle_check")
        del d_data, cb
        torch.cuda.empty_cache()

    if args.split_gib > 0:
        out["checksum_one_file"] = split_leg(ctx, comm, args.split_gib, rank, world, dev, stream,
                                             args.checksum_steps, args.warm_ms, tm=tm, live=args.oracle_live)

    if solo and args.host_checksum_gib > 0:
        with_h2d["checksum"] = checksum_host(ctx, args.host_checksum_gib, dev, stream)
        tm.lap("with_h2d_checksum")
    if solo and args.file_checksum_mib > 0:
        out["file_backed_checksum"] = file_checksums_leg(ctx, args.file_checksum_mib,
                                                         with_cpu=not args.no_cpu_baseline, dev=dev)
        tm.lap("file_backed_checksum")
    if with_h2d:
        out["with_h2d"] = with_h2d

    if not DIST and args.config_files > 0:
        out["configs"] = {k: config_leg(ctx, k, args.config_files, args.config_reps, dev, stream, valu_peak,
                                        args.warm_ms, live=args.oracle_live)
                          for k in ("small", "sampled")}
        tm.lap("configs_1_2")

    if rank == 0 and not DIST and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sizes, cids, twins, args.cpu_seconds)
        if "cpu_reference_schedule" in out.get("file_backed", {}):
            out["cpu_baseline"]["file_backed"] = dict(out["file_backed"]["cpu_reference_schedule"],
                                                      files=out["file_backed"]["files"],
                                                      note="reference read schedule from files (page cache)")
        tm.lap("cpu_baseline")
        out["cpu_baseline"]["end_to_end_vs_library_cpu_path"] = end_to_end_summary(out)
    if comm is not None:
        comm.close()
    total_s = time.perf_counter() - t_main
    tot = torch.tensor([total_s], dtype=torch.float64, device=cdev)
    if DIST:
        dist.all_reduce(tot, op=dist.ReduceOp.MAX)
    try:  # the process's whole life so far: interpreter start, imports, launch included
        import psutil
        proc_s = round(time.time() - psutil.Process().create_time(), 3)
    except Exception:  # noqa: BLE001 -- a diagnostic
        proc_s = None
    out["timing"] = {"rank0_s": dict(tm), "rank0_total_s": round(total_s, 3), "rank0_process_s": proc_s,
                     "total_s_max_over_ranks": round(float(tot.item()), 3),
                     "host_threads_budget": _native.host_cpu_budget()["budget"],
                     "note": "wall seconds per leg on rank 0, from main() to the line (the process's import and "
                             "launch before main() excluded); *_oracle_check legs compare with the committed "
                             "oracle goldens unless --oracle-live"}
    out["launch"] = {"requested_gpus": args.gpus, "mode": mode,
                     "spawned_by_bench": os.environ.get("SD_BENCH_SPAWNED") == "1",
                     "share_gpu": bool(args.share_gpu),
                     "devices_used": len({(r % torch.cuda.device_count()) if args.share_gpu else r
                                          for r in range(world)}) if world > 1 else 1}
    if DIST:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        emit(out, json_out, args.full_out or None)


if __name__ == "__main__":
    main()
