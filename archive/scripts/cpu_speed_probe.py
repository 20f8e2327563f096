"""Host BLAKE3 speeds on this machine: the library's CPU path (libsdcas sd_cpu_*) beside the
oracle's SIMD restatement (the bench's cpu_baseline, oracle/sd_oracle_simd.c), on the same
inputs -- one 512 MiB range (checksum) and the cas messages of 100 000 library files staged
in host memory (hash only) -- at 1 and 16 threads, best of 3.  Outputs asserted equal.
python scripts/cpu_speed_probe.py -> one JSON line"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import native  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402
from spacedrive_amd.device import stage_plan  # noqa: E402


def best(fn, reps=3):
    b = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        b = min(b, time.perf_counter() - t0)
    return b


def main():
    res = {"cpu": os.uname().machine}
    n = 512 << 20
    d = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
    offs, lens = np.zeros(1, np.uint64), np.array([n], np.uint64)
    out = np.zeros(32, np.uint8)
    for t in (1, 16):
        s = best(lambda: check(lib().sd_cpu_checksums(d.ctypes.data, offs.ctypes.data, lens.ctypes.data, 1,
                                                      out.ctypes.data, t)))
        o = best(lambda: native.checksum_mt(d, n, nthreads=t, simd=-1))
        assert native.checksum_mt(d, n, nthreads=t, simd=-1) == out.tobytes()
        res[f"checksum_{t}t_GBps"] = {"library": n / s / 1e9, "oracle": n / o / 1e9}
    k = 100_000
    sizes, cids, twins = synth.library(0, k, 10_000_000)
    ext, total = stage_plan(sizes)
    buf = native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    ext_c = np.ascontiguousarray(ext)
    hexo = ctypes.create_string_buffer(17 * k)
    for t in (1, 16):
        s = best(lambda: check(lib().sd_cpu_cas_ids(buf.ctypes.data, total + 64, ext_c.ctypes.data, k, hexo, None, t)))
        o = best(lambda: native.cas_ids_staged(buf, ext, nthreads=t, simd=-1))
        want = native.cas_ids_staged(buf, ext, nthreads=t, simd=-1)
        raw = hexo.raw
        assert [raw[17 * i:17 * i + 16].decode() for i in range(0, k, 997)] == \
            [want[i][:8].tobytes().hex() for i in range(0, k, 997)]
        res[f"cas_{t}t_files_per_s"] = {"library": k / s, "oracle": k / o, "msg_GBps_library": total / s / 1e9}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
