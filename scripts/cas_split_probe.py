"""Would a split help sd_cas_ids_files from the page cache?  Both routes are bound by host
work (opens, preads, closes; the GPU route then copies each message into a pinned window,
the CPU path hashes it), so the question is whether they contend for the same host
resource.  On the bench's file-backed set (the library mixture, tmpfs) this times, in
interleaved rounds: the GPU route alone and the CPU path alone on 16 threads, and static
splits that run both at once on disjoint parts of the list (the GPU route on g stager
threads over the first fraction f of the files, the CPU path on 16 - g threads over the
rest; the wall time is the slower half's).  Every output is asserted equal.
python scripts/cas_split_probe.py [nfiles] [rounds] -> one JSON line (rows on stderr)"""
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
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402


def _cpu_s():
    t = os.times()
    return t.user + t.system


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
        check(L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, out, st.ctypes.data, 16))
        want = out.raw
        P = ctypes.sizeof(ctypes.c_char_p)

        def gpu(a, b, t):
            check(L.sd_cas_ids_files(ctx.handle, ctypes.addressof(arr) + P * a, sz.ctypes.data + 8 * a, b - a,
                                     ctypes.addressof(out) + 17 * a, st.ctypes.data + 4 * a, t))

        def cpu(a, b, t):
            check(L.sd_cpu_cas_ids_files(ctypes.addressof(arr) + P * a, sz.ctypes.data + 8 * a, b - a,
                                         ctypes.addressof(out) + 17 * a, st.ctypes.data + 4 * a, t))

        def split(g, f):
            def run():
                a = int(k * f)
                th = threading.Thread(target=gpu, args=(0, a, g))
                th.start()
                cpu(a, k, 16 - g)
                th.join()
            return run

        legs = [("gpu_16", lambda: gpu(0, k, 16)), ("cpu_16", lambda: cpu(0, k, 16))]
        legs += [(f"split_g{g}_f{f}", split(g, f)) for g, f in ((8, 0.5), (10, 0.6), (6, 0.4), (12, 0.7))]
        for leg in legs:  # warm
            leg[1]()
        for rnd in range(rounds):
            row = {}
            for name, fn in legs:
                ctypes.memset(out, 0, 17 * k)
                c0, t0 = _cpu_s(), time.perf_counter()
                fn()
                dt = time.perf_counter() - t0
                assert out.raw == want and (st == 0).all(), name
                row[name] = {"files_per_s": k / dt, "host_cpu_us_per_file": (_cpu_s() - c0) / k * 1e6}
            res["rounds"].append(row)
            print(json.dumps({n: round(v["files_per_s"] / 1e6, 3) for n, v in row.items()}), file=sys.stderr,
                  flush=True)
        res["median_M_files_per_s"] = {n: float(np.median([r[n]["files_per_s"] for r in res["rounds"]])) / 1e6
                                       for n, _ in legs}
        print(json.dumps(res))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
