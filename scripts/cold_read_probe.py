"""Can the validator's cold-storage case be measured on the GPU box?  (round 5; DESIGN.md
section 9 "reads from cold storage")  For each candidate directory (the repo copy, /tmp,
$TMPDIR, /dev/shm): its filesystem (/proc/mounts), whether O_DIRECT opens and reads, and
whether posix_fadvise(DONTNEED) on a written, fsync'ed file evicts it from the page cache
(mincore residency before / after) -- then the read rate of a 1 GiB file cold (evicted) and
hot, buffered 1 MiB reads on 1 and 8 threads, and O_DIRECT 1 MiB reads on 8 threads.
python scripts/cold_read_probe.py -> one JSON line"""
import ctypes
import json
import mmap
import os
import threading
import time

GiB = 1 << 30
MiB = 1 << 20
libc = ctypes.CDLL(None, use_errno=True)


def fs_of(path: str) -> str:
    best, fs = "", "?"
    real = os.path.realpath(path)
    with open("/proc/mounts") as f:
        for ln in f:
            dev, mnt, typ = ln.split()[:3]
            if real.startswith(mnt) and len(mnt) > len(best):
                best, fs = mnt, f"{typ} ({dev} on {mnt})"
    return fs


def resident_fraction(path: str) -> float:
    """fraction of the file's pages in the page cache (mmap + mincore, nothing touched)"""
    size = os.path.getsize(path)
    page = os.sysconf("SC_PAGE_SIZE")
    n = (size + page - 1) // page
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    fd = os.open(path, os.O_RDONLY)
    try:
        addr = libc.mmap(None, size, 1, 1, fd, 0)  # PROT_READ, MAP_SHARED
        if addr in (None, ctypes.c_void_p(-1).value):
            return -1.0
        vec = (ctypes.c_ubyte * n)()
        rc = libc.mincore(ctypes.c_void_p(addr), ctypes.c_size_t(size), vec)
        libc.munmap(ctypes.c_void_p(addr), ctypes.c_size_t(size))
        return -1.0 if rc != 0 else sum(v & 1 for v in vec) / n
    finally:
        os.close(fd)


def evict(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def read_rate(path: str, threads: int, direct: bool) -> float:
    size = os.path.getsize(path)
    per = size // threads

    def work(t):
        flags = os.O_RDONLY | (os.O_DIRECT if direct else 0)
        fd = os.open(path, flags)
        m = mmap.mmap(-1, MiB)  # page-aligned buffer (O_DIRECT needs alignment)
        try:
            off = t * per
            end = off + per
            while off < end:
                n = os.preadv(fd, [m], off)
                if n <= 0:
                    break
                off += n
        finally:
            m.close()
            os.close(fd)
    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    return size / (time.perf_counter() - t0) / 1e9


def probe(d: str) -> dict:
    r = {"dir": d, "fs": fs_of(d)}
    path = os.path.join(d, f"sd_cold_probe_{os.getpid()}")
    try:
        with open(path, "wb") as f:
            block = os.urandom(MiB)
            for _ in range(GiB // MiB):
                f.write(block)
            f.flush()
            os.fsync(f.fileno())
        try:
            fd = os.open(path, os.O_RDONLY | os.O_DIRECT)
            m = mmap.mmap(-1, MiB)
            r["o_direct"] = os.preadv(fd, [m], 0) == MiB
            m.close()
            os.close(fd)
        except OSError as e:
            r["o_direct"] = f"no: {e.strerror}"
        r["resident_after_write"] = resident_fraction(path)
        evict(path)
        r["resident_after_fadvise"] = resident_fraction(path)
        r["cold_buffered_1t_GBps"] = read_rate(path, 1, False)
        r["hot_buffered_1t_GBps"] = read_rate(path, 1, False)
        evict(path)
        r["cold_buffered_8t_GBps"] = read_rate(path, 8, False)
        r["hot_buffered_8t_GBps"] = read_rate(path, 8, False)
        if r["o_direct"] is True:
            r["direct_8t_GBps"] = read_rate(path, 8, True)
    except OSError as e:
        r["error"] = str(e)
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
    return r


def main():
    dirs = []
    for d in (os.environ.get("GRAFT_REPO_ROOT") or os.getcwd(), "/tmp", os.environ.get("TMPDIR"), "/dev/shm"):
        if d and os.path.isdir(d) and os.path.realpath(d) not in [os.path.realpath(x) for x in dirs]:
            dirs.append(d)
    print(json.dumps({"probes": [probe(d) for d in dirs]}))


if __name__ == "__main__":
    main()
