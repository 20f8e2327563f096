"""Is the container's CPU quota throttling the host side?  The GPU box's cgroup allows 16
CPUs of time per period while the affinity mask holds 256 CPUs, so 16 busy threads plus any
other runnable thread of the process can spend a period's quota early and the whole cgroup
then waits for the next period.  For file checksums from tmpfs (32 x 256 MiB, the bench's
set) this times the library's CPU path at T threads and the split policy at read budgets B,
each with the cgroup's cpu.stat deltas (periods, throttled periods, throttled time).
Interleaved rounds; every output asserted equal.
python scripts/throttle_probe.py [rounds] -> one JSON line (per-round rows on stderr)"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch  # noqa: F401  (the device, for the synthetic files)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib, path_array  # noqa: E402
from scripts.hybrid_checksum_probe2 import write_set  # noqa: E402


def cpu_stat():
    for p in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            with open(p) as f:
                return {k: int(v) for k, v in (ln.split() for ln in f if len(ln.split()) == 2)}
        except OSError:
            continue
    return {}


def cpu_max():
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            pass
    return None


def main():
    rounds_n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = sd.default_context(0)
    L = lib()
    knobs = ("checksum_cpu_max", "checksum_hybrid_threads", "read_threads")
    keep = {k: sd.get_tuning(k) for k in knobs}
    d = tempfile.mkdtemp(dir="/dev/shm")
    lens = [256 << 20] * 32
    res = {"cpu.max": cpu_max(), "affinity": len(os.sched_getaffinity(0)), "rounds": []}
    try:
        paths = write_set(ctx, d, lens, 40_000)
        n, total = len(paths), sum(lens)
        _keep, arr = path_array(paths)
        out = ctypes.create_string_buffer(65 * n)
        st = np.zeros(n, np.int32)
        check(L.sd_cpu_file_checksums(arr, n, out, st.ctypes.data, 16))
        want = out.raw

        def timed(fn, reps=3):
            best, s0 = None, cpu_stat()
            for _ in range(reps):
                ctypes.memset(out, 0, 65 * n)
                t0 = time.perf_counter()
                fn()
                dt = time.perf_counter() - t0
                assert out.raw == want and (st == 0).all()
                best = dt if best is None else min(best, dt)
            s1 = cpu_stat()
            delta = {k: s1[k] - s0.get(k, 0) for k in s1 if k in ("nr_periods", "nr_throttled", "throttled_usec",
                                                                   "usage_usec", "throttled_time")}
            return {"GBps": total / best / 1e9, **delta}

        def cpu(t):
            return lambda: check(L.sd_cpu_file_checksums(arr, n, out, st.ctypes.data, t))

        def split(budget, g=4):
            def f():
                sd.set_tuning("checksum_cpu_max", 2147483647)
                sd.set_tuning("checksum_hybrid_threads", g)
                sd.set_tuning("read_threads", budget)
                try:
                    check(L.sd_file_checksums(ctx.handle, arr, n, out, st.ctypes.data))
                finally:
                    for k, v in keep.items():
                        sd.set_tuning(k, v)
            return f

        legs = [(f"cpu_{t}", cpu(t)) for t in (16, 15, 14, 12)]
        legs += [(f"split_b{b}", split(b)) for b in (16, 15, 14)]
        for rnd in range(rounds_n):
            r = {k: timed(f) for k, f in legs}
            res["rounds"].append(r)
            print(json.dumps({"round": rnd, **{k: round(v["GBps"], 1) for k, v in r.items()},
                              "throttled": {k: v.get("nr_throttled") for k, v in r.items()}}),
                  file=sys.stderr, flush=True)
        res["median_GBps"] = {k: float(np.median([r[k]["GBps"] for r in res["rounds"]])) for k, _ in legs}
        print(json.dumps(res))
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
