"""What bounds the co-hashed checksum call over pinned memory (round 5; DESIGN.md section
4.2): the host's hashing against the device's DMA from host memory.  4 GiB of pinned memory A (the bench's with-H2D checksum input: 4 x 1 GiB), a second
pinned buffer B of 4 GiB and a device buffer; legs, in interleaved rounds:
  cpu_T          sd_cpu_checksums over A on T threads (T = 13, 16), nothing else running
  dma            one 4 GiB H2D copy B -> device, alone
  cpu_T+dma      the same CPU call while that copy runs (the copy queued first); both rates
  cohash_13      sd_checksums over A (the library default: the GPU + 13 host threads)
Every CPU-path output asserted equal to the first.  Also the NUMA node of A's and B's pages
(move_pages) and the GPU's node, so the contention can be put on DRAM or on the fabric.
python scripts/cohash_contention_probe.py [rounds] -> one JSON line (rows on stderr)"""
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


def page_nodes(ptr: int, nbytes: int, samples: int = 256) -> dict:
    """NUMA node of `samples` evenly spaced pages of [ptr, ptr + nbytes) (move_pages with no
    target nodes only reports where each page is)."""
    libc = ctypes.CDLL(None, use_errno=True)
    page = os.sysconf("SC_PAGE_SIZE")
    addrs = (ctypes.c_void_p * samples)(*[(ptr + (nbytes - page) * i // (samples - 1)) & ~(page - 1)
                                           for i in range(samples)])
    status = (ctypes.c_int * samples)()
    SYS_move_pages = 279  # x86_64
    rc = libc.syscall(SYS_move_pages, 0, ctypes.c_ulong(samples), addrs, None, status, 0)
    if rc != 0:
        return {"error": os.strerror(ctypes.get_errno())}
    out = {}
    for s in status:
        out[str(s)] = out.get(str(s), 0) + 1
    return out


def host_numa() -> list:
    """sd_host_numa: [placed, CPUs on the device's node, the device's node]"""
    v = (ctypes.c_int * 3)()
    check(lib().sd_host_numa(v))
    return list(v)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    sd.set_tuning("checksum_split_adapt", 0)  # cohash_13 is always the co-hashed call (round 6's learned route off)
    ctx = sd.default_context(0)
    nf, flen = 4, 1 << 30
    total = nf * flen
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    for i in range(nf):
        ctx.synth_fill(20_000 + i, 0, flen, d[i * flen:])
    a = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    b = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    a.copy_(d)
    b.fill_(7)
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    L = lib()
    offs = np.arange(nf, dtype=np.uint64) * np.uint64(flen)
    lens = np.full(nf, flen, np.uint64)
    h32 = np.zeros((nf, 32), np.uint8)
    out = ctypes.create_string_buffer(65 * nf)
    side = torch.cuda.Stream()
    want = None

    def cpu(T):
        t0 = time.perf_counter()
        check(L.sd_cpu_checksums(a.data_ptr(), offs.ctypes.data, lens.ctypes.data, nf, h32.ctypes.data, T))
        dt = time.perf_counter() - t0
        return dt, [h32[i].tobytes().hex() for i in range(nf)]

    def dma_start():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            e0.record(side)
            dst.copy_(b, non_blocking=True)
            e1.record(side)
        return e0, e1

    def leg(name):
        nonlocal want
        r = {}
        if name.startswith("cpu_"):
            T = int(name.split("_")[1].split("+")[0])
            ev = dma_start() if name.endswith("+dma") else None
            if ev:
                time.sleep(0.002)  # the copy under way before the hashing starts
            dt, got = cpu(T)
            if want is None:
                want = got
            assert got == want, name
            r["cpu_GBps"] = total / dt / 1e9
            if ev:
                side.synchronize()
                r["dma_GBps"] = total / (ev[0].elapsed_time(ev[1]) / 1e3) / 1e9
        elif name == "dma":
            ev = dma_start()
            side.synchronize()
            r["dma_GBps"] = total / (ev[0].elapsed_time(ev[1]) / 1e3) / 1e9
        else:  # cohash_13: the library default
            t0 = time.perf_counter()
            check(L.sd_checksums(ctx.handle, a.data_ptr(), offs.ctypes.data, lens.ctypes.data, nf, out))
            dt = time.perf_counter() - t0
            assert [out.raw[65 * i:65 * i + 64].decode() for i in range(nf)] == want, name
            r["GBps"] = total / dt / 1e9
        return r

    legs = ["cpu_16", "cpu_13", "dma", "cpu_13+dma", "cpu_16+dma", "cohash_13"]
    for n in legs:  # warm
        leg(n)
    rows = []
    for rnd in range(rounds):
        row = {n: leg(n) for n in legs}
        rows.append(row)
        print(json.dumps({"round": rnd, **{n: {k: round(v, 1) for k, v in x.items()} for n, x in row.items()}}),
              file=sys.stderr, flush=True)
    med = {n: {k: float(np.median([r[n][k] for r in rows])) for k in rows[0][n]} for n in legs}
    print(json.dumps({"bytes": total, "rounds": rows, "median": med, "host_budget": sd.host_cpu_budget(),
                      "numa": {"a_pages": page_nodes(a.data_ptr(), total), "b_pages": page_nodes(b.data_ptr(), total),
                               "sd_host_numa": host_numa(),
                               "affinity": len(os.sched_getaffinity(0))}}))


if __name__ == "__main__":
    main()
