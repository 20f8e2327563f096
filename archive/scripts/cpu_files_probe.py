"""The library's CPU path from files (sd_cpu_cas_ids_files) beside the oracle's reference
read schedule (sdo_cas_ids_files), same files, same thread counts, C calls only (paths
encoded outside the timed region), best of `reps`.  Files: the configs[0] mixture on
tmpfs, sampled files sparse.  python scripts/cpu_files_probe.py [files] [threads...]"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import native  # noqa: E402  (checker and CPU baseline only)
from spacedrive_amd._native import lib  # noqa: E402
from spacedrive_amd.synth import sample_windows  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    threads = [int(a) for a in sys.argv[2:]] or [1, 8]
    reps = 3
    rng = np.random.default_rng(5)
    small = rng.random(n) < 0.6
    sizes = np.where(small, np.exp(rng.uniform(0, np.log(102400), n)),
                     np.exp(rng.uniform(np.log(102401), np.log(4 << 30), n))).astype(np.uint64)
    sizes = np.maximum(sizes, 1)
    d = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        paths = []
        for i, s in enumerate(sizes.tolist()):
            p = os.path.join(d, f"f{i:07d}")
            fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            if s > 102400:
                os.ftruncate(fd, s)
            for fo, ln in sample_windows(s):
                if ln:
                    os.pwrite(fd, rng.integers(0, 256, ln, np.uint8).tobytes(), fo)
            os.close(fd)
            paths.append(p)
        arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
        sz = np.ascontiguousarray(sizes, np.uint64)
        out = ctypes.create_string_buffer(17 * n)
        st = np.zeros(n, np.int32)
        o_out = np.zeros((n, 8), np.uint8)
        o_st = np.zeros(n, np.int32)
        ol = native.lib()
        res = {"files": n, "msg_bytes": int(sum(min(int(s), 102400) + 8 if s <= 102400 else 57352 for s in sizes))}
        for nt in threads:
            lt, ot = [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                lib().sd_cpu_cas_ids_files(arr, sz.ctypes.data, n, out, st.ctypes.data, nt)
                lt.append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                ol.sdo_cas_ids_files(arr, native._p(sz), n, native._p(o_out), native._p(o_st), nt, -1)
                ot.append(time.perf_counter() - t0)
            raw = out.raw
            assert (st == 0).all() and (o_st == 0).all()
            assert all(raw[17 * i:17 * i + 16].decode() == o_out[i].tobytes().hex() for i in range(n))
            res[f"threads_{nt}"] = {"library_files_per_s": n / min(lt), "oracle_files_per_s": n / min(ot),
                                    "library_us_per_file_thread": min(lt) * nt / n * 1e6,
                                    "oracle_us_per_file_thread": min(ot) * nt / n * 1e6}
        print(json.dumps(res))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
