"""Every host entry point of libsdcas at once on one context (round 5), for `seconds`:
  A  sd_file_checksums over a split-eligible file set (the split or the CPU path, learned)
  B  sd_cas_ids_files over 20 000 library files (the stager's private-fd readers)
  C  sd_checksums over 1.25 GiB of pinned host memory (the GPU and 13 co-hashing threads)
  D  single-file calls (sd_cas_id_path: the coalescer and the latency policy), 4 threads
Every result is compared with the C oracle's (A, C: every checksum; B, D: every cas_id).
Prints one JSON line: calls and mismatches per kind, errors; exits 1 on any of them or a hang.
python scripts/mixed_stress.py [seconds=60]"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402
from spacedrive_amd.device import stage_plan  # noqa: E402
from oracle import native  # noqa: E402  (the checker)

MiB = 1 << 20


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    ctx = sd.default_context(0)
    d = tempfile.mkdtemp(prefix="sd_mixed_stress_")
    try:
        # A: large files
        ck_paths = []
        for i in range(10):
            size = (40 + 9 * i) * MiB + 17 * i
            p = os.path.join(d, f"big{i}")
            with open(p, "wb") as f:
                pos = 0
                while pos < size:
                    k = min(32 * MiB, size - pos)
                    f.write(native.synth_bytes(41000 + i, 0, pos, k))
                    pos += k
            ck_paths.append(p)
        ck_want = [h.tobytes().hex() for h in native.file_checksums(ck_paths, nthreads=16)[0]]
        # B, D: library files
        n = 20000
        sizes, cids, twins = synth.library(0, n, n)
        sizes = np.minimum(sizes, np.uint64(1 << 34))
        ext, total = stage_plan(sizes)
        staged = native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
        lib_dir = os.path.join(d, "lib")
        os.mkdir(lib_dir)
        lib_paths = synth.write_files(lib_dir, sizes, staged, ext)
        nz = [i for i in range(n) if int(sizes[i])]  # (an empty file has no cas_id, mod.rs:80-88)
        lib_paths = [lib_paths[i] for i in nz]
        sizes = sizes[nz]
        n = len(nz)
        ids_want, _ = native.cas_ids_files(lib_paths, sizes, nthreads=16)
        ids_want = [w.tobytes().hex() for w in ids_want]
        # C: pinned host ranges
        nr, rlen = 5, 256 * MiB
        dev = torch.empty(nr * rlen + 64, dtype=torch.uint8, device="cuda")
        for i in range(nr):
            ctx.synth_fill(42000 + i, 0, rlen, dev[i * rlen:])
        host = torch.empty(nr * rlen + 64, dtype=torch.uint8, pin_memory=True)
        torch.cuda.synchronize()
        host.copy_(dev)
        del dev
        offs = np.arange(nr, dtype=np.uint64) * np.uint64(rlen)
        lens = np.full(nr, rlen, np.uint64)
        rng_want = [h.tobytes().hex() for h in native.checksums(host.numpy(), offs, lens, nthreads=16)]

        stop = time.time() + seconds
        calls = {"A": 0, "B": 0, "C": 0, "D": 0}
        bad = {"A": 0, "B": 0, "C": 0, "D": 0}
        errors = []
        lock = threading.Lock()

        def count(kind, c, b):
            with lock:
                calls[kind] += c
                bad[kind] += b

        def run(kind, fn):
            try:
                while time.time() < stop:
                    fn()
            except Exception as e:  # noqa: BLE001
                errors.append(f"{kind}: {e!r}")

        def a():
            got = sd.file_checksums(ck_paths)
            count("A", 1, sum(g != w for g, w in zip(got, ck_want)))

        size_list = [int(x) for x in sizes]

        def b():
            got = sd.generate_cas_ids(lib_paths, size_list)
            count("B", 1, sum(g != w for g, w in zip(got, ids_want)))

        L = lib()
        rng_out = ctypes.create_string_buffer(65 * nr)

        def c():
            check(L.sd_checksums(ctx.handle, host.data_ptr(), offs.ctypes.data, lens.ctypes.data, nr, rng_out))
            got = [rng_out.raw[65 * i:65 * i + 64].decode() for i in range(nr)]
            count("C", 1, sum(g != w for g, w in zip(got, rng_want)))

        rs = np.random.default_rng(7)

        def dd():
            i = int(rs.integers(0, n))
            got = sd.generate_cas_id(lib_paths[i], size_list[i])
            count("D", 1, got != ids_want[i])

        th = [threading.Thread(target=run, args=(k, f)) for k, f in (("A", a), ("B", b), ("C", c))]
        th += [threading.Thread(target=run, args=("D", dd)) for _ in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=seconds + 300)
        hung = any(x.is_alive() for x in th)
        print(json.dumps({"seconds": seconds, "calls": calls, "mismatches": bad, "errors": errors, "hung": hung,
                          "routes": sd.file_checksums_stats(), "cas_files_routes": sd.cas_ids_files_stats()}),
              flush=True)
        if hung or errors or sum(bad.values()):
            sys.exit(1)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
