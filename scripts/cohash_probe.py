"""sd_cas_ids from pinned host memory with h host threads co-hashing ("host_cohash_threads"),
h in {0, 8, 11..15}, against the library's CPU path alone on 16 threads (sd_cpu_cas_ids):
the bench's with-H2D leg (300 000 files of the library mixture, 8.55 GB of messages),
interleaved rounds, outputs asserted equal.
python scripts/cohash_probe.py [files] [rounds] -> one JSON line"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = sd.default_context(0)
    sizes, cids, twins = synth.library(0, k, 10_000_000)
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), k, d)
    host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    host.copy_(d)
    del d
    L = lib()
    out = ctypes.create_string_buffer(17 * k)
    want = None
    res = {"files": k, "bytes": total, "rounds": []}
    keep = sd.get_tuning("host_cohash_threads")
    try:
        for _ in range(rounds):
            row = {}
            for h in ((0, 8, 11, 12, 13, 14, 15) if k >= 100_000 else (0, 15)):
                sd.set_tuning("host_cohash_threads", h)
                check(L.sd_cas_ids(ctx.handle, host.data_ptr(), total + 64, ext.ctypes.data, k, out, None))  # warm
                s0 = np.zeros(2, np.uint64)
                s1 = np.zeros(2, np.uint64)
                check(L.sd_cas_ids_stats(ctx.handle, s0.ctypes.data))
                reps = max(1, 200_000 // k)
                t0 = time.perf_counter()
                for _ in range(reps):
                    check(L.sd_cas_ids(ctx.handle, host.data_ptr(), total + 64, ext.ctypes.data, k, out, None))
                dt = (time.perf_counter() - t0) / reps
                check(L.sd_cas_ids_stats(ctx.handle, s1.ctypes.data))
                raw = out.raw
                want = want or raw
                assert raw == want
                row[f"cohash_{h}"] = {"files_per_s": k / dt, "GBps": total / dt / 1e9, "ms_per_call": dt * 1e3,
                                      "host_share": float((s1 - s0)[1]) / (k * reps)}
            t0 = time.perf_counter()
            check(L.sd_cpu_cas_ids(host.data_ptr(), total + 64, ext.ctypes.data, k, out, None, 16))
            dt = time.perf_counter() - t0
            assert out.raw == want
            row["cpu_path_16"] = {"files_per_s": k / dt, "GBps": total / dt / 1e9}
            res["rounds"].append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    finally:
        sd.set_tuning("host_cohash_threads", keep)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
