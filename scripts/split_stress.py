"""Stress of sd_file_checksums' split (round 5): its threads feed the GPU from the shared-fd
pool and free the slots through host functions on the slot streams.
Three caller threads, one context, each repeatedly checksumming its own split-eligible file
set (>= 512 MiB of files >= 8 MiB, odd sizes, a small file and an unreadable path among
them) for `seconds`, with the GPU slot count and the learned route varied between calls;
every result is compared with the C oracle's.  Prints one JSON line: calls per thread,
mismatches, errors.
python scripts/split_stress.py [seconds=60]"""
import json
import os
import shutil
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from oracle import native  # noqa: E402  (the checker)

MiB = 1 << 20


def write(d, name, cid, size):
    p = os.path.join(d, name)
    with open(p, "wb") as f:
        pos = 0
        while pos < size:
            k = min(32 * MiB, size - pos)
            f.write(native.synth_bytes(cid, 0, pos, k))
            pos += k
    return p


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    sd.default_context(0)
    d = tempfile.mkdtemp(prefix="sd_split_stress_")
    try:
        sets = []
        for t in range(3):
            sizes = [(24 + 7 * i) * MiB + 13 * i + t for i in range(10)] + [5000 + t, 9 * MiB - 1]
            paths = [write(d, f"t{t}_{i}", 40000 + 100 * t + i, s) for i, s in enumerate(sizes)]
            paths.insert(3, os.path.join(d, f"missing_{t}"))
            want = []
            for p in paths:
                if os.path.exists(p):
                    h, st = native.file_checksums([p], nthreads=16)
                    want.append(h[0].tobytes().hex() if st[0] == 0 else None)
                else:
                    want.append(None)
            sets.append((paths, want))
        keep = {k: sd.get_tuning(k) for k in ("checksum_cpu_max", "checksum_hybrid_threads", "checksum_split_adapt")}
        sd.set_tuning("checksum_cpu_max", 2147483647)
        calls = [0, 0, 0]
        bad = [0, 0, 0]
        errors = []
        stop = time.time() + seconds

        def worker(t):
            paths, want = sets[t]
            k = 0
            try:
                while time.time() < stop:
                    got = sd.file_checksums(paths)
                    for g, w in zip(got, want):
                        if w is None:
                            bad[t] += not isinstance(g, OSError)
                        else:
                            bad[t] += g != w
                    calls[t] += 1
                    k += 1
                    if t == 0 and k % 5 == 0:  # vary the policy under the other callers
                        sd.set_tuning("checksum_hybrid_threads", [6, 2, 10, 1, 6][k // 5 % 5])
                        sd.set_tuning("checksum_split_adapt", [8, 0, 2][k // 5 % 3])
            except Exception as e:  # noqa: BLE001
                errors.append(f"thread {t}: {e!r}")

        th = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=seconds + 300)
        alive = any(x.is_alive() for x in th)
        for k, v in keep.items():
            sd.set_tuning(k, v)
        print(json.dumps({"seconds": seconds, "calls": calls, "mismatches": bad, "errors": errors, "hung": alive,
                          "routes": sd.file_checksums_stats()}), flush=True)
        if alive or errors or sum(bad):
            sys.exit(1)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
