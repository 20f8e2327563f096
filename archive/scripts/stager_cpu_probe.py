"""Host-only probe (no GPU needed): why does the GPU route's stager read files more slowly
than the library's CPU path reads *and hashes* them?  Times, on the same tmpfs file set and
at equal thread counts:
  * sd_cas_stage_files into one large buffer (the shape cas_files uses: consecutive files
    packed at 128-B starts), fresh and re-used;
  * sd_cpu_cas_ids_files (read into a per-thread scratch buffer + hash);
python scripts/stager_cpu_probe.py [nfiles] [threads]   -> one JSON line"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import native  # noqa: E402  -- only to build the synthetic file contents
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402
from spacedrive_amd.device import stage_plan  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    th = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    sizes, cids, twins = synth.library(0, k, 1_250_000)
    ext, total = stage_plan(sizes)
    host = native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    tmp = tempfile.mkdtemp(dir="/dev/shm")
    out = {"files": k, "threads": th}
    try:
        paths = synth.write_files(tmp, sizes, host, ext)
        L = lib()
        arr = (ctypes.c_char_p * k)(*[os.fsencode(p) for p in paths])
        sz = np.ascontiguousarray(sizes, np.uint64)
        st = np.zeros(k, np.int32)

        def best(fn, reps=5):
            b = 1e9
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                b = min(b, time.perf_counter() - t0)
            return b

        stage = np.zeros(total + 64, np.uint8)
        ext2 = ext.copy()
        out["stage_reused_files_per_s"] = k / best(lambda: check(
            L.sd_cas_stage_files(arr, ext2.ctypes.data, k, stage.ctypes.data, st.ctypes.data, th)))

        def fresh():
            s2 = np.empty(total + 64, np.uint8)
            check(L.sd_cas_stage_files(arr, ext2.ctypes.data, k, s2.ctypes.data, st.ctypes.data, th))
        out["stage_fresh_files_per_s"] = k / best(fresh)
        # the same reads into a small, cache-resident region: file i at slot i % R of 128 KiB
        # (a timing probe only: slots are overwritten; a slot holds the longest message,
        # 8 + 102400 B + padding) -- what do cold destinations cost?
        slot = 131072
        assert int(ext["msg_len"].max()) + 64 <= slot
        for R in (32, 128, 512):
            ring_ext = ext.copy()
            ring_ext["msg_offset"] = (np.arange(k, dtype=np.uint64) % np.uint64(R)) * np.uint64(slot)
            small = np.zeros(R * slot + 64, np.uint8)
            out[f"stage_ring{R}x128k_files_per_s"] = k / best(lambda: check(
                L.sd_cas_stage_files(arr, ring_ext.ctypes.data, k, small.ctypes.data, st.ctypes.data, th)))
        buf = ctypes.create_string_buffer(17 * k)
        out["cpu_path_files_per_s"] = k / best(lambda: check(
            L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, buf, st.ctypes.data, th)))
        try:
            import torch
            gpu = torch.cuda.is_available()
        except ImportError:
            gpu = False
        if gpu:  # the stager's real destination: hipHostMalloc'd (pinned) memory
            pinned = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
            pinned.zero_()
            out["stage_pinned_files_per_s"] = k / best(lambda: check(
                L.sd_cas_stage_files(arr, ext2.ctypes.data, k, pinned.data_ptr(), st.ctypes.data, th)))
            import spacedrive_amd as sd
            ctx = sd.default_context(0)
            check(L.sd_cas_set_tuning(b"batch_cpu_max", 0))
            out["gpu_route_files_per_s"] = k / best(lambda: check(
                L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, buf, st.ctypes.data, th)))
            ref = buf.raw
            sweep = os.environ.get("SWEEP", "")  # "window_mb:ring,..." -> the GPU route per setting
            for item in filter(None, sweep.split(",")):
                wmb, ring = (int(v) for v in item.split(":"))
                check(L.sd_cas_set_tuning(b"files_window_mb", wmb))
                check(L.sd_cas_set_tuning(b"files_ring", ring))
                out[f"gpu_route_w{wmb}_r{ring}_files_per_s"] = k / best(lambda: check(
                    L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, buf, st.ctypes.data, th)))
                assert buf.raw == ref, item
            check(L.sd_cas_set_tuning(b"files_window_mb", 32))
            check(L.sd_cas_set_tuning(b"files_ring", 4))
        out["cpus_affinity"] = len(os.sched_getaffinity(0))
        out["message_GB"] = float(ext["msg_len"].astype(np.float64).sum()) / 1e9
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
