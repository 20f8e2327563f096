"""Times sd_file_checksums on N x 256 MiB tmpfs files (the bench's file_backed_checksum
leg) a few times; run under rocprofv3 --kernel-trace --memory-copy-trace to see where the
host waits.  python scripts/ck_files_probe.py [nfiles] [reps]"""
import json
import os
import shutil
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    flen = 256 << 20
    d = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        ctx = sd.default_context(0)
        buf = torch.empty(flen, dtype=torch.uint8, device="cuda")
        paths = []
        for i in range(nf):
            ctx.synth_fill(30_000 + i, 0, flen, buf)
            torch.cuda.synchronize()
            p = os.path.join(d, f"ck{i}")
            buf.cpu().numpy().tofile(p)
            paths.append(p)
        sd.file_checksums(paths[:1])
        out = {"files": nf, "bytes": nf * flen, "GBps": []}
        ref = None
        for _ in range(reps):
            t0 = time.perf_counter()
            got = sd.file_checksums(paths)
            dt = time.perf_counter() - t0
            out["GBps"].append(round(nf * flen / dt / 1e9, 2))
            assert ref is None or got == ref
            ref = got
        t0 = time.perf_counter()
        cpu = sd.cpu.file_checksums(paths, nthreads=16)
        out["cpu_GBps"] = round(nf * flen / (time.perf_counter() - t0) / 1e9, 2)
        assert cpu == ref
        print(json.dumps(out))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
