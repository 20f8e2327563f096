"""How many host threads the from-files routes should run under the box's 16-CPU quota (round
5): at 15 co-hashing threads sd_checksums lost 12-17 % against 13 (the calling thread and
the runtime's threads left no core free).  The same question for the file
routes, in interleaved rounds on tmpfs:
  cas_gpu_T / cas_cpu_T   sd_cas_ids_files (GPU route, T stager threads) and
                          sd_cpu_cas_ids_files (T threads) over 200 000 library files
  ck_cpu_T / ck_split_T   sd_cpu_file_checksums on T threads and sd_file_checksums' default
                          split with "read_threads" T, over 32 x 256 MiB
every output asserted equal to the first leg's (the cas ids to the oracle's on a sample).
python scripts/files_threads_probe.py [rounds] -> one JSON line (per-round rows on stderr)"""
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
from scripts.hybrid_checksum_probe2 import write_set  # noqa: E402

THREADS = (12, 13, 14, 15, 16)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = sd.default_context(0)
    L = lib()
    k = 200_000
    sizes, cids, twins = synth.library(0, k, 1_250_000)
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), k, d)
    host = d.cpu().numpy()
    del d
    tmp = tempfile.mkdtemp(dir="/dev/shm")
    keep = {key: sd.get_tuning(key) for key in ("batch_cpu_max", "read_threads")}
    try:
        paths = synth.write_files(tmp, sizes, host, ext)
        del host
        _keep_a, arr = path_array(paths)
        sz = np.ascontiguousarray(sizes, np.uint64)
        st = np.zeros(k, np.int32)
        out = ctypes.create_string_buffer(17 * k)
        from oracle import native  # the reference answer for the probe's own check
        idx = np.linspace(0, k - 1, 2048).astype(np.int64)
        want_ids, _ = native.cas_ids_files([paths[i] for i in idx], sizes[idx], nthreads=16)
        ck_dir = os.path.join(tmp, "ck")
        os.mkdir(ck_dir)
        ck_paths = write_set(ctx, ck_dir, [256 << 20] * 32, 60_000)
        ck_total = 32 * (256 << 20)
        _keep_b, ck_arr = path_array(ck_paths)
        ck_st = np.zeros(32, np.int32)
        ck_out = ctypes.create_string_buffer(65 * 32)
        ck_want, _ = native.file_checksums(ck_paths, nthreads=16)
        ck_want = [w.tobytes().hex() for w in ck_want]

        def cas_gpu(T):
            def f():
                sd.set_tuning("batch_cpu_max", 0)
                try:
                    check(L.sd_cas_ids_files(ctx.handle, arr, sz.ctypes.data, k, out, st.ctypes.data, T))
                finally:
                    sd.set_tuning("batch_cpu_max", keep["batch_cpu_max"])
                return "cas"
            return f

        def cas_cpu(T):
            def f():
                check(L.sd_cpu_cas_ids_files(arr, sz.ctypes.data, k, out, st.ctypes.data, T))
                return "cas"
            return f

        def ck_cpu(T):
            def f():
                check(L.sd_cpu_file_checksums(ck_arr, 32, ck_out, ck_st.ctypes.data, T))
                return "ck"
            return f

        def ck_split(T):
            def f():
                sd.set_tuning("read_threads", T)
                try:
                    check(L.sd_file_checksums(ctx.handle, ck_arr, 32, ck_out, ck_st.ctypes.data))
                finally:
                    sd.set_tuning("read_threads", keep["read_threads"])
                return "ck"
            return f

        legs = [(f"cas_gpu_{T}", cas_gpu(T)) for T in THREADS] + [(f"cas_cpu_{T}", cas_cpu(T)) for T in THREADS]
        legs += [(f"ck_cpu_{T}", ck_cpu(T)) for T in THREADS] + [(f"ck_split_{T}", ck_split(T)) for T in THREADS]
        for _, f in legs:  # warm: pools, windows, page cache
            f()
        rows = []
        for rnd in range(rounds):
            r = {}
            for name, f in legs:
                t0 = time.perf_counter()
                what = f()
                dt = time.perf_counter() - t0
                if what == "cas":
                    assert (st == 0).all(), name
                    got = [out.raw[17 * i:17 * i + 16].decode() for i in idx]
                    assert got == [w.tobytes().hex() for w in want_ids], name
                    r[name] = k / dt
                else:
                    assert (ck_st == 0).all(), name
                    assert [ck_out.raw[65 * i:65 * i + 64].decode() for i in range(32)] == ck_want, name
                    r[name] = ck_total / dt / 1e9
            rows.append(r)
            print(json.dumps({"round": rnd, **{key: round(v, 1) if v < 1e4 else round(v) for key, v in r.items()}}),
                  file=sys.stderr, flush=True)
        med = {name: float(np.median([r[name] for r in rows])) for name, _ in legs}
        print(json.dumps({"cas_files": k, "ck_bytes": ck_total, "units": {"cas": "files/s", "ck": "GB/s"},
                          "rounds": rows, "median": med, "host_budget": sd.host_cpu_budget()}))
    finally:
        for key, v in keep.items():
            sd.set_tuning(key, v)
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
