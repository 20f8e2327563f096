"""Writes a synthetic library's first N files (random bytes in the windows generate_cas_id
reads; sampled files sparse) to a scratch dir and runs scripts/stage_bench.c over them.

    python scripts/stage_bench.py N THREADS[,THREADS...] [MODES, e.g. 0,2,0,2]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd import synth  # noqa: E402

n, Ts = int(sys.argv[1]), [int(t) for t in sys.argv[2].split(",")]
sizes, _, _ = synth.library(0, n, 1_250_000)
rng = np.random.default_rng(1)
d = tempfile.mkdtemp(prefix="sb_", dir="/dev/shm")
lst = os.path.join(d, "list.txt")
with open(lst, "w") as f:
    f.write(f"{n}\n")
    for i, s in enumerate(sizes.tolist()):
        p = os.path.join(d, f"f{i:07d}")
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        if s > synth.SMALL_MAX:
            os.ftruncate(fd, s)
        for fo, ln in synth.sample_windows(s):
            if ln:
                os.pwrite(fd, rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), fo)
        os.close(fd)
        f.write(f"{p} {s}\n")
exe = os.path.join(tempfile.mkdtemp(prefix="sbx_"), "stage_bench")  # /dev/shm may be noexec
src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stage_bench.c")
subprocess.run(["gcc", "-O2", "-w", "-o", exe, src, "-lpthread"], check=True)
modes = [(int(m), 0) for m in sys.argv[3].split(",")] if len(sys.argv) > 3 else \
    [(0, 0), (1, 16), (1, 64), (0, 0), (1, 64)]
for T in Ts:
    for mode, b in modes:
        args = [exe, lst, str(T), str(mode)] + ([str(b or 64)] if mode == 1 else [])
        print(" ".join(args[2:]), flush=True)
        subprocess.run(args, check=True)
subprocess.run(["rm", "-rf", d])
