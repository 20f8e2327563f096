"""Per-call cost of the path-based entry points at small batch sizes (the latency path and
the identifier's 100-file steps): sd_cas_ids_files and sd_file_checksums (GPU), and the
library's CPU path on 16 threads beside them, with n = 1, 16, 100 files (or the sizes given) of the bench's file-backed mixture on tmpfs,
200 calls each after a warm-up (fewer for large n); median / p90 wall time per call.
Sampled files are capped on disk (4 MiB, or 1 MiB past 100 files), which moves only their
sample offsets.  Prints one JSON object.
python scripts/small_batch_probe.py [calls] [n,n,...]"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402


def _with_policy(fn, cpu_max=4096):
    sd.set_tuning("batch_cpu_max", cpu_max)
    try:
        return fn()
    finally:
        sd.set_tuning("batch_cpu_max", 0)
    sd.set_tuning("checksum_cpu_max", 0)  # "file_checksums" times the GPU route (the default policy is the CPU path)


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    ctx = sd.Context(0)
    # "cas_ids_files" times the GPU route: the batch-size policy would send these calls to
    # the CPU path ("policy_cas_ids_files" times the default policy beside it)
    sd.set_tuning("batch_cpu_max", 0)
    root = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        ks = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 16, 100]
        n = max(ks)
        cap = (4 << 20) if n <= 100 else (1 << 20)
        sizes, cids, twins = synth.library(0, n, n)
        rng = np.random.default_rng(3)
        paths = []
        for i in range(n):
            p = os.path.join(root, f"f{i}")
            s = int(min(sizes[i], cap))  # keep the sampled files small on disk
            sizes[i] = s
            with open(p, "wb") as f:
                f.write(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
            paths.append(p.encode())
        res = {}
        for k in ks:
            reps = max(10, min(calls, 20000 // k))
            arr = (ctypes.c_char_p * k)(*paths[:k])
            sz = np.ascontiguousarray(sizes[:k], np.uint64)
            st = np.zeros(k, np.int32)
            hex17 = ctypes.create_string_buffer(17 * k)
            hex65 = ctypes.create_string_buffer(65 * k)
            for name, fn in (("cas_ids_files", lambda: lib().sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, hex17,
                                                                                st.ctypes.data, 16)),
                             ("policy_cas_ids_files", lambda: _with_policy(lambda: lib().sd_cas_ids_files(
                                 ctx.handle, arr, sz.ctypes.data, k, hex17, st.ctypes.data, 16))),
                             ("file_checksums", lambda: lib().sd_file_checksums(ctx.handle, arr, k, hex65,
                                                                                st.ctypes.data)),
                             ("cpu_cas_ids_files_16t", lambda: lib().sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, hex17,
                                                                                         st.ctypes.data, 16)),
                             ("cpu_file_checksums_16t", lambda: lib().sd_cpu_file_checksums(arr, k, hex65,
                                                                                           st.ctypes.data, 16))):
                for _ in range(10):
                    check(fn())
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    check(fn())
                    ts.append((time.perf_counter() - t0) * 1e6)
                ts.sort()
                res[f"{name}_n{k}"] = {"p50_us": ts[len(ts) // 2], "p90_us": ts[int(len(ts) * 0.9)], "min_us": ts[0]}
        print(json.dumps(res))
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
