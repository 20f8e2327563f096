"""A/B of the two from-files cas_id routes on one file set, alternated in one process:
sd_cas_ids_files (GPU route: stager threads -> pinned windows -> kernels) and
sd_cpu_cas_ids_files (the library's CPU path: read + hash on the same thread count), with
the wall time and the process's CPU time (user + system, every thread) of each call.
python scripts/files_ab.py [nfiles] [threads] [rounds]  -> one JSON line"""
import ctypes
import json
import os
import resource
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


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    th = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
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
    out = {"files": k, "threads": th, "rounds": rounds}
    try:
        paths = synth.write_files(tmp, sizes, host, ext)
        del host
        L = lib()
        arr = (ctypes.c_char_p * k)(*[os.fsencode(p) for p in paths])
        sz = np.ascontiguousarray(sizes, np.uint64)
        st = np.zeros(k, np.int32)
        a, b = ctypes.create_string_buffer(17 * k), ctypes.create_string_buffer(17 * k)
        keep = sd.get_tuning("batch_cpu_max")
        sd.set_tuning("batch_cpu_max", 0)
        def gpu(hot):
            def run():
                sd.set_tuning("files_stage_hot", hot)
                try:
                    return L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, a, st.ctypes.data, th)
                finally:
                    sd.set_tuning("files_stage_hot", 0)
            return run
        routes = {"gpu": gpu(0), "gpu_stage_hot": gpu(1),
                  "cpu_path": lambda: L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, b, st.ctypes.data, th)}
        res = {r: {"s": [], "cpu_s": []} for r in routes}
        for r in routes:  # warm both
            check(routes[r]())
        for _ in range(rounds):
            for r, fn in routes.items():
                c0, t0 = cpu_s(), time.perf_counter()
                check(fn())
                res[r]["s"].append(time.perf_counter() - t0)
                res[r]["cpu_s"].append(cpu_s() - c0)
        sd.set_tuning("batch_cpu_max", keep)
        assert a.raw == b.raw
        check(routes["gpu_stage_hot"]())
        assert a.raw == b.raw
        for r, v in res.items():
            s = np.array(v["s"])
            out[r] = {"files_per_s_median": k / float(np.median(s)), "files_per_s_best": k / float(s.min()),
                      "files_per_s_all": [round(k / x) for x in s],
                      "cpu_us_per_file_median": float(np.median(v["cpu_s"])) / k * 1e6}
        out["gpu_over_cpu_median"] = out["gpu"]["files_per_s_median"] / out["cpu_path"]["files_per_s_median"]
        try:
            out["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
        except OSError:
            pass
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
