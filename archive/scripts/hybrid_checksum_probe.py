"""Can the GPU route and the CPU path of file_checksum (hash.rs:10-24) share one call?
From the page cache the GPU route is PCIe-bound (~54 GB/s on 16 reader threads) and the CPU
path is bound by its 16 threads (~89 GB/s); the GPU route needs few threads to fill PCIe,
so a call whose files are split between the two -- g reader threads for the GPU route,
16 - g for the CPU path, running at once -- might beat both.  Prototype from Python: the
two C entry points on disjoint file subsets, on two host threads (ctypes releases the
GIL), 32 x 256 MiB files on tmpfs; outputs asserted equal to the CPU path's.  Then the
library's own split (sd_file_checksums' default policy: a shared cursor over the large
files, "checksum_hybrid_threads" g = 0 (off: the CPU path), 4, 6, 8), interleaved rounds.
python scripts/hybrid_checksum_probe.py [nfiles] -> one JSON line"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib, path_array  # noqa: E402


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    flen = 256 << 20
    ctx = sd.default_context(0)
    d = tempfile.mkdtemp(dir="/dev/shm")
    L = lib()
    try:
        buf = torch.empty(flen, dtype=torch.uint8, device="cuda")
        paths = []
        for i in range(nf):
            ctx.synth_fill(30_000 + i, 0, flen, buf)
            torch.cuda.synchronize()
            p = os.path.join(d, f"ck{i}")
            buf.cpu().numpy().tofile(p)
            paths.append(p)
        del buf
        total = nf * flen
        keep, arr = path_array(paths)
        ptrs = np.ctypeslib.as_array((ctypes.c_uint64 * nf).from_address(arr))
        out = ctypes.create_string_buffer(65 * nf)
        st = np.zeros(nf, np.int32)
        check(L.sd_cpu_file_checksums(arr, nf, out, st.ctypes.data, 16))
        want = out.raw

        def gpu(a, b, g):
            check(L.sd_cas_set_tuning(b"read_threads", g))
            check(L.sd_file_checksums(ctx.handle, ptrs[a:].ctypes.data, b - a, ctypes.byref(out, 65 * a),
                                      st[a:].ctypes.data))

        def cpu(a, b, c):
            check(L.sd_cpu_file_checksums(ptrs[a:].ctypes.data, b - a, ctypes.byref(out, 65 * a),
                                          st[a:].ctypes.data, c))

        def timed(fn, reps=3):
            best = None
            for _ in range(reps):
                ctypes.memset(out, 0, 65 * nf)
                t0 = time.perf_counter()
                fn()
                dt = time.perf_counter() - t0
                assert out.raw == want and (st == 0).all()
                best = dt if best is None else min(best, dt)
            return total / best / 1e9

        def policy(g):  # the library's own split (sd_file_checksums, default checksum_cpu_max)
            check(L.sd_cas_set_tuning(b"checksum_cpu_max", 2147483647))
            check(L.sd_cas_set_tuning(b"read_threads", 16))
            check(L.sd_cas_set_tuning(b"checksum_hybrid_threads", g))
            try:
                check(L.sd_file_checksums(ctx.handle, arr, nf, out, st.ctypes.data))
            finally:
                check(L.sd_cas_set_tuning(b"checksum_hybrid_threads", 0))
                check(L.sd_cas_set_tuning(b"checksum_cpu_max", 0))

        check(L.sd_cas_set_tuning(b"checksum_cpu_max", 0))  # sd_file_checksums: its GPU route
        res = {"files": nf, "bytes": total, "rows": [], "policy": []}
        for rnd in range(2):  # interleaved rounds: the box's clocks and page cache drift
            r = {"cpu_16": timed(lambda: cpu(0, nf, 16)), "gpu_16": timed(lambda: gpu(0, nf, 16))}
            for g in (0, 4, 6, 8):
                r[f"policy_hybrid_{g}"] = timed(lambda g=g: policy(g))
            res["policy"].append(r)
            print(json.dumps(r), file=sys.stderr, flush=True)
        res["cpu_16"] = max(r["cpu_16"] for r in res["policy"])
        res["gpu_16"] = max(r["gpu_16"] for r in res["policy"])
        for g in (6,):
            for k in (nf * 3 // 8, nf // 2, nf * 5 // 8):
                def hyb(g=g, k=k):
                    t = threading.Thread(target=gpu, args=(0, k, g))
                    t.start()
                    cpu(k, nf, 16 - g)
                    t.join()
                row = {"gpu_threads": g, "gpu_files": k, "GBps": timed(hyb)}
                res["rows"].append(row)
                print(json.dumps(row), file=sys.stderr, flush=True)
        print(json.dumps(res))
    finally:
        L.sd_cas_set_tuning(b"checksum_cpu_max", 2147483647)
        L.sd_cas_set_tuning(b"read_threads", 16)
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
