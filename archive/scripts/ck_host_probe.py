"""sd_checksums over pinned host memory (the bench's with-H2D checksum leg): 4 x 1 GiB
ranges, timed several times; run under rocprofv3 --kernel-trace --memory-copy-trace to see
the copy / kernel timeline.  python scripts/ck_host_probe.py [gib] [reps]"""
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    ctx = sd.default_context(0)
    flen = 1 << 30
    total = gib * flen
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    for i in range(gib):
        ctx.synth_fill(20_000 + i, 0, flen, d[i * flen:])
    host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    host.copy_(d)
    del d
    torch.cuda.empty_cache()
    out = ctypes.create_string_buffer(65 * gib)
    res = {}
    for name, offs, lens in (("1GiB_ranges", np.arange(gib, dtype=np.uint64) * np.uint64(flen),
                              np.full(gib, flen, np.uint64)),
                             ("one_range", np.zeros(1, np.uint64), np.array([total], np.uint64))):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            check(lib().sd_checksums(ctx.handle, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, len(lens), out))
            ts.append(time.perf_counter() - t0)
        res[name] = [round(total / t / 1e9, 2) for t in ts]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
