"""Zero-copy H2D from the page cache: can the GPU route of file_checksum skip the host's
memcpy?  A regular file is mmap'ed read-only, the mapping is page-locked with
hipHostRegister (read-only flag), and one hipMemcpyAsync DMA-reads the page-cache pages
straight into HBM -- no host thread copies the bytes.  Per file: the register cost, the DMA
rate, the unregister cost and the process CPU time, against a pread into pinned memory of
the same bytes.  The device copy is checked against the file (torch equality).
python scripts/zerocopy_probe.py [nfiles] [MiB per file] -> one JSON line"""
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

PROT_READ, MAP_SHARED = 1, 1
MAP_FAILED = ctypes.c_void_p(-1).value


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    flen = mib << 20
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    d = tempfile.mkdtemp(dir="/dev/shm")
    res = {"files": nf, "bytes_per_file": flen, "flags": {}}
    try:
        rng = np.random.default_rng(3)
        paths = []
        for i in range(nf):
            p = os.path.join(d, f"z{i}")
            rng.integers(0, 255, flen, dtype=np.uint8).tofile(p)
            paths.append(p)
        dev = torch.empty(flen, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for flags in (0x08, 0x00, 0x08 | 0x01):  # ReadOnly, Default, ReadOnly|Portable
            rows = []
            for i, p in enumerate(paths):
                fd = os.open(p, os.O_RDONLY)
                c0, t0 = cpu_s(), time.perf_counter()
                addr = libc.mmap(None, flen, PROT_READ, MAP_SHARED, fd, 0)
                if addr in (None, MAP_FAILED):
                    os.close(fd)
                    rows.append({"error": f"mmap errno {ctypes.get_errno()}"})
                    break
                t1 = time.perf_counter()
                rc = hip.hipHostRegister(addr, flen, flags)
                t2 = time.perf_counter()
                if rc != 0:
                    libc.munmap(addr, flen)
                    os.close(fd)
                    rows.append({"error": f"hipHostRegister rc {rc}"})
                    break
                rc = hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr()), addr, flen, 1, ctypes.c_void_p(stream))
                hip.hipStreamSynchronize(ctypes.c_void_p(stream))
                t3 = time.perf_counter()
                hip.hipHostUnregister(addr)
                libc.munmap(addr, flen)
                os.close(fd)
                t4 = time.perf_counter()
                cpu = cpu_s() - c0
                ok = bool(torch.equal(dev[:1 << 20].cpu(), torch.from_numpy(np.fromfile(p, np.uint8, 1 << 20))))
                tail = np.fromfile(p, np.uint8)[-4096:]
                ok = ok and bool(torch.equal(dev[-4096:].cpu(), torch.from_numpy(tail)))
                rows.append({"mmap_ms": (t1 - t0) * 1e3, "register_ms": (t2 - t1) * 1e3, "dma_ms": (t3 - t2) * 1e3,
                             "unregister_ms": (t4 - t3) * 1e3, "total_GBps": flen / (t4 - t0) / 1e9,
                             "dma_GBps": flen / (t3 - t2) / 1e9, "cpu_ms": cpu * 1e3, "equal": ok, "memcpy_rc": rc})
            res["flags"][hex(flags)] = rows
            print(hex(flags), json.dumps(rows[-1] if rows else None), file=sys.stderr, flush=True)
        # baseline: pread into pinned memory, then the same DMA
        pinned = torch.empty(flen, dtype=torch.uint8, pin_memory=True)
        rows = []
        for p in paths:
            c0, t0 = cpu_s(), time.perf_counter()
            with open(p, "rb", buffering=0) as f:
                f.readinto(memoryview(pinned.numpy()))
            t1 = time.perf_counter()
            dev.copy_(pinned, non_blocking=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rows.append({"read_ms": (t1 - t0) * 1e3, "dma_ms": (t2 - t1) * 1e3, "total_GBps": flen / (t2 - t0) / 1e9,
                         "cpu_ms": (cpu_s() - c0) * 1e3})
        res["pread_pinned"] = rows
        print("pread", json.dumps(rows[-1]), file=sys.stderr, flush=True)
        print(json.dumps(res))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
