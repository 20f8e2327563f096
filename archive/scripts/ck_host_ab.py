"""A/B of sd_checksums over pinned host memory between two builds of libsdcas (raw ctypes,
so an older build with fewer exports loads too): python scripts/ck_host_ab.py LIB [gib]"""
import ctypes
import json
import sys
import time

import numpy as np
import torch


def main():
    L = ctypes.CDLL(sys.argv[1])
    gib = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    P = ctypes.c_void_p
    L.sd_cas_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
    L.sd_checksums.argtypes = [P, P, P, P, ctypes.c_size_t, P]
    ctx = P()
    assert L.sd_cas_ctx_create(0, ctypes.byref(ctx)) == 0
    flen = 1 << 30
    total = gib * flen
    host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    host[:total].copy_(torch.randint(0, 256, (total,), dtype=torch.uint8))
    offs = np.arange(gib, dtype=np.uint64) * np.uint64(flen)
    lens = np.full(gib, flen, np.uint64)
    out = ctypes.create_string_buffer(65 * gib)
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        assert L.sd_checksums(ctx, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, gib, out) == 0
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"lib": sys.argv[1].split("/")[-2], "GBps": [round(total / t / 1e9, 2) for t in ts],
                      "first_hash": out.raw[:16].decode()}))


if __name__ == "__main__":
    main()
