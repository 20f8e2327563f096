"""Per-call cost of sd_cas_ids_files (GPU route) at the identifier look-ahead's batch sizes,
from tmpfs: the same 100 000 files hashed in consecutive calls of K files, K from 4096 to
100 000, the C ABI called directly (paths encoded once) and through the Python wrapper
(spacedrive_amd.cas.generate_cas_ids), beside the library's CPU path at the same K.
Set SD_PROFILE_FILES=1 for the library's per-call breakdown on stderr.
python scripts/lookahead_probe.py [nfiles]  -> one JSON line"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib, path_array  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    ctx = sd.default_context(0)
    sizes, cids, twins = synth.library(0, k, 1_250_000)
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), k, d)
    host = d.cpu().numpy()
    del d
    tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    sd.set_tuning("batch_cpu_max", 0)  # the GPU route at every K
    try:
        paths = synth.write_files(tmp, sizes, host, ext)
        del host
        keep, arr_all = path_array(paths)
        ptrs = np.ctypeslib.as_array((ctypes.c_uint64 * k).from_address(arr_all))
        sz = np.ascontiguousarray(sizes, np.uint64)
        out = ctypes.create_string_buffer(17 * k)
        st = np.zeros(k, np.int32)
        L = lib()
        res = {"files": k, "rows": []}
        for K in (4096, 8192, 16384, 32768, 65536, k):
            row = {"K": K}
            for route in ("gpu", "cpu", "gpu_python"):
                best = None
                for _ in range(3):
                    t0 = time.perf_counter()
                    for a in range(0, k, K):
                        b = min(k, a + K)
                        if route == "gpu":
                            check(L.sd_cas_ids_files(ctx.handle, ptrs[a:].ctypes.data, sz[a:].ctypes.data, b - a,
                                                     ctypes.byref(out, 17 * a), st[a:].ctypes.data, 16))
                        elif route == "cpu":
                            check(L.sd_cpu_cas_ids_files(ptrs[a:].ctypes.data, sz[a:].ctypes.data, b - a,
                                                         ctypes.byref(out, 17 * a), st[a:].ctypes.data, 16))
                        else:
                            sd.generate_cas_ids(paths[a:b], sizes[a:b])
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                assert (st == 0).all()
                row[route] = {"files_per_s": k / best, "ms_per_call": best * 1e3 / ((k + K - 1) // K)}
            res["rows"].append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
        print(json.dumps(res))
    finally:
        sd.set_tuning("batch_cpu_max", 4096)
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
