"""sd_checksums over ONE range of `gib` GiB of pinned host memory (the bench's with-H2D
one_range leg): GPU only (host_cohash_threads 0) against shared block by block with h host
threads, h in {4, 8, 15}; also the same bytes as gib ranges of 1 GiB and as 4 gib ranges
of 256 MiB, and the CPU path alone
(sd_cpu_checksums).  Outputs asserted equal.
python scripts/shared_range_probe.py [gib] [rounds] -> one JSON line"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402


def main():
    gib = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = sd.default_context(0)
    total = gib << 30
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    for i in range(gib):
        ctx.synth_fill(20_000 + i, 0, 1 << 30, d[i << 30:])
    host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    host.copy_(d)
    del d
    L = lib()
    out = ctypes.create_string_buffer(65 * 4 * gib)
    keep = sd.get_tuning("host_cohash_threads")
    one_off, one_len = np.zeros(1, np.uint64), np.array([total], np.uint64)
    many_off = np.arange(gib, dtype=np.uint64) << np.uint64(30)
    many_len = np.full(gib, 1 << 30, np.uint64)
    q_off = np.arange(4 * gib, dtype=np.uint64) << np.uint64(28)
    q_len = np.full(4 * gib, 1 << 28, np.uint64)
    res = {"bytes": total, "rounds": []}
    want = {}
    try:
        for _ in range(rounds):
            row = {}
            for h in (0, 4, 8, 15):
                sd.set_tuning("host_cohash_threads", h)
                for name, offs, lens in (("one", one_off, one_len), ("ranges", many_off, many_len),
                                         ("quarters", q_off, q_len)):
                    check(L.sd_checksums(ctx.handle, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, len(offs),
                                         out))
                    t0 = time.perf_counter()
                    check(L.sd_checksums(ctx.handle, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, len(offs),
                                         out))
                    dt = time.perf_counter() - t0
                    got = out.raw[:65 * len(offs)]
                    assert want.setdefault(name, got) == got, (name, h)
                    row[f"{name}_cohash_{h}_GBps"] = total / dt / 1e9
            h32 = ctypes.create_string_buffer(32)
            t0 = time.perf_counter()
            check(L.sd_cpu_checksums(host.data_ptr(), one_off.ctypes.data, one_len.ctypes.data, 1, h32, 16))
            dt = time.perf_counter() - t0
            assert h32.raw.hex() == want["one"][:64].decode()
            row["cpu_path_16_GBps"] = total / dt / 1e9
            res["rounds"].append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    finally:
        sd.set_tuning("host_cohash_threads", keep)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
