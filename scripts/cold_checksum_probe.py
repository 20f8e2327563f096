"""The validator's checksums from COLD files (round 5): every file's pages dropped from the
page cache before each leg (fsync + posix_fadvise(DONTNEED), residency checked with
mincore), on the box's own filesystem (an overlay; scripts/cold_read_probe.py measured
17-18 GB/s for cold buffered reads against 29-34 GB/s with O_DIRECT on 8 threads).
Legs, in interleaved rounds over NF x 256 MiB in /tmp:
  cpu16 / split / gpu    sd_cpu_file_checksums on 16 threads / sd_file_checksums' default
                         (the split by blocks) / its GPU route alone ("checksum_cpu_max" 0)
  raw_buffered / raw_direct   16 threads reading every file in 1 MiB preads, page-cache
                         reads / O_DIRECT into aligned buffers, no hashing: the read floors
  *_hot                  cpu16 and split again without dropping the pages
Every checksum asserted equal to the first leg's.
python scripts/cold_checksum_probe.py [rounds] [nf] -> one JSON line (rows on stderr)"""
import ctypes
import json
import mmap
import os
import shutil
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib, path_array  # noqa: E402
from scripts.cold_read_probe import evict, resident_fraction  # noqa: E402

MiB = 1 << 20


def write_files(d: str, nf: int, flen: int) -> list:
    paths = []
    block = bytearray(os.urandom(MiB))
    for i in range(nf):
        p = os.path.join(d, f"c{i}")
        with open(p, "wb") as f:
            for k in range(flen // MiB):
                block[:8] = (i * 100000 + k).to_bytes(8, "little")  # every block distinct
                f.write(block)
            os.fsync(f.fileno())
        paths.append(p)
    return paths


def raw_read(paths: list, threads: int, direct: bool) -> float:
    units = [(p, o) for p in paths for o in range(0, os.path.getsize(p), MiB)]
    nxt = [0]
    lock = threading.Lock()
    total = [0]

    def work():
        m = mmap.mmap(-1, MiB)
        fds = {}
        got = 0
        try:
            while True:
                with lock:
                    if nxt[0] >= len(units):
                        break
                    p, o = units[nxt[0]]
                    nxt[0] += 1
                if p not in fds:
                    fds[p] = os.open(p, os.O_RDONLY | (os.O_DIRECT if direct else 0))
                got += os.preadv(fds[p], [m], o)
        finally:
            for fd in fds.values():
                os.close(fd)
            m.close()
            with lock:
                total[0] += got
    t0 = time.perf_counter()
    th = [threading.Thread(target=work) for _ in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    return total[0] / (time.perf_counter() - t0) / 1e9


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    flen = 256 * MiB
    ctx = sd.default_context(0)
    L = lib()
    d = f"/tmp/sd_cold_ck_{os.getpid()}"
    os.makedirs(d)
    keep = sd.get_tuning("checksum_cpu_max")
    try:
        paths = write_files(d, nf, flen)
        total = nf * flen
        _keep, arr = path_array(paths)
        st = np.zeros(nf, np.int32)
        out = ctypes.create_string_buffer(65 * nf)
        want = None

        def drop():
            for p in paths:
                evict(p)
            return float(np.mean([resident_fraction(p) for p in paths[:4]]))

        def lib_leg(kind):
            nonlocal want
            if kind == "cpu16":
                check(L.sd_cpu_file_checksums(arr, nf, out, st.ctypes.data, 16))
            else:
                sd.set_tuning("checksum_cpu_max", 0 if kind == "gpu" else keep)
                try:
                    check(L.sd_file_checksums(ctx.handle, arr, nf, out, st.ctypes.data))
                finally:
                    sd.set_tuning("checksum_cpu_max", keep)
            assert (st == 0).all(), kind
            got = [out.raw[65 * i:65 * i + 64] for i in range(nf)]
            if want is None:
                want = got
            assert got == want, kind

        legs = ["cpu16", "split", "gpu", "raw_buffered", "raw_direct", "cpu16_hot", "split_hot"]
        rows = []
        for rnd in range(rounds):
            r = {}
            for name in legs:
                hot = name.endswith("_hot")
                res = None if hot else drop()
                t0 = time.perf_counter()
                if name.startswith("raw_"):
                    gbps = raw_read(paths, 16, name == "raw_direct")
                else:
                    lib_leg(name.replace("_hot", ""))
                    gbps = total / (time.perf_counter() - t0) / 1e9
                r[name] = {"GBps": gbps, "resident_before": res}
            rows.append(r)
            print(json.dumps({"round": rnd, **{k: round(v["GBps"], 1) for k, v in r.items()}}), file=sys.stderr,
                  flush=True)
        med = {k: float(np.median([r[k]["GBps"] for r in rows])) for k in legs}
        print(json.dumps({"bytes": total, "files": nf, "rounds": rows, "median_GBps": med,
                          "fs": open("/proc/mounts").read().split("\n")[0], "host_budget": sd.host_cpu_budget()}))
    finally:
        sd.set_tuning("checksum_cpu_max", keep)
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
