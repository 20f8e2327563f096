"""Where does the file-backed cas GPU route spend host CPU?  On the bench's file-backed set
(library mixture, tmpfs) this measures wall time and process CPU time per file, in
interleaved rounds, for:
  stage_only   sd_cas_stage_files: the stager's reads into one pageable host buffer (no GPU)
  gpu_route    sd_cas_ids_files: the same reads into the pinned ring + H2D + kernels + hex
  cpu_path     sd_cpu_cas_ids_files: the same reads + the CPU hash
all on 16 threads; and the process's thread count and per-thread CPU (from /proc) over a
gpu_route call, to see whether any thread besides the readers burns CPU.
python scripts/files_cpu_cost_probe.py [nfiles] [rounds] -> one JSON line"""
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


def _cpu_s():
    t = os.times()
    return t.user + t.system


def thread_cpu():
    """{tid: (name, utime+stime ticks)} of this process's threads."""
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                s = f.read()
            name = s[s.index("(") + 1:s.rindex(")")]
            rest = s[s.rindex(")") + 2:].split()
            out[tid] = (name, int(rest[11]) + int(rest[12]))
        except OSError:
            pass
    return out


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = sd.default_context(0)
    sizes, cids, twins = synth.library(0, k, 1_250_000)
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), k, d)
    host = d.cpu().numpy()
    del d
    tmp = tempfile.mkdtemp(dir="/dev/shm")
    res = {"files": k, "rounds": []}
    try:
        paths = synth.write_files(tmp, sizes, host, ext)
        del host
        L = lib()
        arr = (ctypes.c_char_p * k)(*[os.fsencode(p) for p in paths])
        sz = np.ascontiguousarray(sizes, np.uint64)
        out = ctypes.create_string_buffer(17 * k)
        st = np.zeros(k, np.int32)
        stage = np.zeros(total + 64, np.uint8)
        ext2 = ext.copy()

        legs = {
            "stage_only": lambda: check(L.sd_cas_stage_files(arr, ext2.ctypes.data, k, stage.ctypes.data,
                                                             st.ctypes.data, 16)),
            "gpu_route": lambda: check(L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, out, st.ctypes.data, 16)),
            "cpu_path": lambda: check(L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, out, st.ctypes.data, 16)),
        }
        for f in legs.values():
            f()
        for rnd in range(rounds):
            row = {}
            for name, f in legs.items():
                ext2[:] = ext
                c0, t0 = _cpu_s(), time.perf_counter()
                f()
                dt = time.perf_counter() - t0
                assert (st == 0).all(), name
                row[name] = {"files_per_s": k / dt, "cpu_us_per_file": (_cpu_s() - c0) / k * 1e6}
            res["rounds"].append(row)
            print(json.dumps({n: (round(v["files_per_s"] / 1e6, 3), round(v["cpu_us_per_file"], 2))
                              for n, v in row.items()}), file=sys.stderr, flush=True)
        # per-thread CPU over one gpu_route call
        a = thread_cpu()
        legs["gpu_route"]()
        b = thread_cpu()
        hz = os.sysconf("SC_CLK_TCK")
        per = sorted(((b[t][1] - a.get(t, ("", 0))[1]) / hz * 1e3, b[t][0]) for t in b)
        res["gpu_route_threads_cpu_ms"] = [(round(ms, 1), n) for ms, n in per[::-1] if ms > 0]
        res["threads"] = len(b)
        print(json.dumps(res))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
