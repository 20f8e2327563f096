"""sd_cas_ids_files on the bench's file-backed set (20 000 library files on tmpfs) across the
files_window_mb knob and stager thread counts, beside the library's CPU path and the
oracle's reference read schedule: where does the file-backed cas path lose time?
python scripts/cas_files_probe.py [nfiles]  -> one JSON line"""
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
from spacedrive_amd._native import check, lib  # noqa: E402


REPS = 5


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    ctx = sd.default_context(0)
    sizes, cids, twins = synth.library(0, k, 1_250_000)
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), k, d)
    host = d.cpu().numpy()
    tmp = tempfile.mkdtemp(dir="/dev/shm")
    out = {"files": k}
    try:
        paths = synth.write_files(tmp, sizes, host, ext)
        L = lib()
        arr = (ctypes.c_char_p * k)(*[os.fsencode(p) for p in paths])
        sz = np.ascontiguousarray(sizes, np.uint64)
        buf = ctypes.create_string_buffer(17 * k)
        st = np.zeros(k, np.int32)
        ref = None
        for mb in (32, 64):
            check(L.sd_cas_set_tuning(b"files_window_mb", mb))
            for th in (16, 32):
                best = 1e9
                for _ in range(REPS):
                    t0 = time.perf_counter()
                    check(L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, buf, st.ctypes.data, th))
                    best = min(best, time.perf_counter() - t0)
                assert (st == 0).all()
                ids = buf.raw
                assert ref is None or ids == ref
                ref = ids
                out[f"gpu_w{mb}_t{th}_files_per_s"] = round(k / best)
        check(L.sd_cas_set_tuning(b"files_window_mb", 32))
        # staging alone (the pread pool into pinned memory, no GPU)
        ext2 = ext.copy()
        stage = np.zeros(total + 64, np.uint8)
        for th in (16, 32):
            best = 1e9
            for _ in range(REPS):
                t0 = time.perf_counter()
                check(L.sd_cas_stage_files(arr, ext2.ctypes.data, k, stage.ctypes.data, st.ctypes.data, th))
                best = min(best, time.perf_counter() - t0)
            out[f"stage_only_t{th}_files_per_s"] = round(k / best)
        for th in (16, 32):
            t0 = time.perf_counter()
            sd.cpu.generate_cas_ids(paths, sizes, nthreads=th)
            out[f"cpu_path_t{th}_files_per_s"] = round(k / (time.perf_counter() - t0))
        from oracle import native
        for th in (16, 32):
            t0 = time.perf_counter()
            native.cas_ids_files(paths, sizes, nthreads=th, simd=-1)
            out[f"oracle_t{th}_files_per_s"] = round(k / (time.perf_counter() - t0))
        out["cpus_affinity"] = len(os.sched_getaffinity(0))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
