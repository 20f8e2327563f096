"""Does placing libsdcas's own threads on the GPU's NUMA node ("numa_pin", sd_host.h) help
its host-side paths?  Interleaved rounds, numa_pin 1 vs 0, in one process on the box:
  ck_cpu_16      sd_cpu_file_checksums, 32 x 256 MiB on tmpfs, 16 threads
  ck_policy      sd_file_checksums with its default policy (the split)
  cas_gpu        sd_cas_ids_files, 200 000 library-mixture files on tmpfs (the GPU route)
  cas_cpu_16     sd_cpu_cas_ids_files, the same files, 16 threads
The files are written from this (unplaced) main thread, as an indexer's would be.
python scripts/numa_lib_probe.py [rounds] -> one JSON line (rounds on stderr)"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, host_numa, lib, path_array  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ctx = sd.default_context(0)
    L = lib()
    d = tempfile.mkdtemp(dir="/dev/shm")
    keep = sd.get_tuning("numa_pin")
    try:
        # checksum files
        flen, nf = 256 << 20, 32
        buf = torch.empty(flen, dtype=torch.uint8, device="cuda")
        ck_paths = []
        for i in range(nf):
            ctx.synth_fill(60_000 + i, 0, flen, buf)
            torch.cuda.synchronize()
            p = os.path.join(d, f"ck{i}")
            buf.cpu().numpy().tofile(p)
            ck_paths.append(p)
        del buf
        # library files (the bench's file-backed set)
        n = 200_000
        sizes, cids, twins = synth.library(0, n, 8 * n)
        ext, total = sd.stage_plan(sizes)
        d_staged = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        d_ext = torch.from_numpy(ext.view(np.uint8).copy()).cuda()
        ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                            torch.from_numpy(twins.astype(np.int32)).cuda(), d_ext, n, d_staged)
        torch.cuda.synchronize()
        host = d_staged.cpu().numpy()
        del d_staged
        lib_dir = os.path.join(d, "lib")
        os.makedirs(lib_dir)
        paths = synth.write_files(lib_dir, sizes, host, ext)
        del host
        _k1, ck_arr = path_array(ck_paths)
        _k2, arr = path_array(paths)
        sz = np.ascontiguousarray(sizes, np.uint64)
        ck_out = ctypes.create_string_buffer(65 * nf)
        ck_st = np.zeros(nf, np.int32)
        out = ctypes.create_string_buffer(17 * n)
        st = np.zeros(n, np.int32)

        def ck_cpu():
            check(L.sd_cpu_file_checksums(ck_arr, nf, ck_out, ck_st.ctypes.data, 16))

        def ck_policy():
            check(L.sd_file_checksums(ctx.handle, ck_arr, nf, ck_out, ck_st.ctypes.data))

        def cas_gpu():
            check(L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, n, out, st.ctypes.data, 16))

        def cas_cpu():
            check(L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, n, out, st.ctypes.data, 16))

        legs = {"ck_cpu_16": (ck_cpu, nf * flen, "GBps"), "ck_policy": (ck_policy, nf * flen, "GBps"),
                "cas_gpu": (cas_gpu, n, "Mfiles_per_s"), "cas_cpu_16": (cas_cpu, n, "Mfiles_per_s")}
        want = {}
        res = {k: {1: [], 0: []} for k in legs}
        for rnd in range(rounds + 1):  # round 0 warms
            for pin in (1, 0):
                sd.set_tuning("numa_pin", pin)
                for k, (fn, units, _) in legs.items():
                    t0 = time.perf_counter()
                    fn()
                    dt = time.perf_counter() - t0
                    o = (ck_out if k.startswith("ck") else out).raw
                    if k not in want:
                        want[k] = o
                    assert o == want[k], k
                    if rnd:
                        res[k][pin].append(units / dt / 1e9 if legs[k][2] == "GBps" else units / dt / 1e6)
            if rnd:
                print(json.dumps({"round": rnd, **{f"{k}_pin{p}": res[k][p][-1] for k in legs for p in (1, 0)}}),
                      file=sys.stderr, flush=True)
        summary = {k: {"unit": legs[k][2], "median_pinned": float(np.median(res[k][1])),
                       "median_unpinned": float(np.median(res[k][0]))} for k in legs}
        for k in summary:
            summary[k]["pinned_over_unpinned"] = summary[k]["median_pinned"] / summary[k]["median_unpinned"]
        print(json.dumps({"numa": host_numa(), "rounds": rounds, "summary": summary, "raw": {k: res[k] for k in res}}))
    finally:
        sd.set_tuning("numa_pin", keep)
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
