"""sd_file_checksums from the page cache, round 4: the GPU route's readers now deliver
through pread_stream (page cache -> a cache-resident buffer -> streaming stores into the
pinned window; "checksum_stage_hot") and every pool run is limited to the call's reader
count, so a split call (the GPU route on g reader threads, the CPU path on 16 - g) no
longer runs its GPU half on the 16 threads an earlier call left in the pools.  Interleaved
rounds on two tmpfs file sets (the bench's 32 x 256 MiB, and 48 files of 8..320 MiB):
  cpu_16                 sd_cpu_file_checksums on 16 threads (the library's CPU path)
  gpu_16[_hot0]          the GPU route alone ("checksum_cpu_max" 0), pread_stream on / off
  hybrid_g[_hot0]        the policy's split, "checksum_hybrid_threads" g
  *_pK                   the same with "cpu_read_piece_kib" K (round 5: the CPU path reads and
                         hashes each 1 MiB block K KiB at a time; 256 the default since)
  hybrid_g / _files      round 5: the split claimed by blocks with g GPU slots (the default) /
                         by whole files (round 4, "checksum_split_blocks" 0)
Every call's output is asserted equal to the CPU path's.
python scripts/hybrid_checksum_probe2.py [rounds] [legs,...] -> one JSON line (per-round rows on stderr)"""
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib, path_array  # noqa: E402

KNOBS = ("checksum_cpu_max", "checksum_hybrid_threads", "checksum_stage_hot", "read_threads", "cpu_read_piece_kib",
         "checksum_split_blocks")


def write_set(ctx, d, lens, cid0):
    buf = torch.empty(max(lens) + 64, dtype=torch.uint8, device="cuda")
    paths = []
    for i, ln in enumerate(lens):
        ctx.synth_fill(cid0 + i, 0, ln, buf)
        torch.cuda.synchronize()
        p = os.path.join(d, f"f{cid0 + i}")
        buf[:ln].cpu().numpy().tofile(p)
        paths.append(p)
    return paths


def main():
    ctx = sd.default_context(0)
    L = lib()
    keep = {k: sd.get_tuning(k) for k in KNOBS}
    d = tempfile.mkdtemp(dir="/dev/shm")
    rng = np.random.default_rng(11)
    sets = {"32x256MiB": [256 << 20] * 32,
            "48_mixed_8_320MiB": [int(x) for x in rng.integers(8 << 20, 320 << 20, 48)]}
    out_all = {}
    try:
        for name, lens in sets.items():
            paths = write_set(ctx, d, lens, 40_000 if name.startswith("32") else 50_000)
            n, total = len(paths), sum(lens)
            _keep, arr = path_array(paths)
            out = ctypes.create_string_buffer(65 * n)
            st = np.zeros(n, np.int32)
            check(L.sd_cpu_file_checksums(arr, n, out, st.ctypes.data, 16))
            want = out.raw
            from oracle import native  # the reference answer for the probe's own check
            ref, _ = native.file_checksums(paths, nthreads=16)
            assert [want[65 * i:65 * i + 64].decode() for i in range(n)] == [r.tobytes().hex() for r in ref]

            def timed(fn, reps=3):
                best = None
                for _ in range(reps):
                    ctypes.memset(out, 0, 65 * n)
                    t0 = time.perf_counter()
                    fn()
                    dt = time.perf_counter() - t0
                    assert out.raw == want and (st == 0).all()
                    best = dt if best is None else min(best, dt)
                return total / best / 1e9

            def cpu16(piece=256):
                def f():
                    sd.set_tuning("cpu_read_piece_kib", piece)
                    try:
                        check(L.sd_cpu_file_checksums(arr, n, out, st.ctypes.data, 16))
                    finally:
                        sd.set_tuning("cpu_read_piece_kib", keep["cpu_read_piece_kib"])
                return f

            def policy(cpu_max, g, hot, piece=256, blocks=1):
                def f():
                    sd.set_tuning("checksum_split_blocks", blocks)
                    sd.set_tuning("checksum_cpu_max", cpu_max)
                    sd.set_tuning("checksum_hybrid_threads", g)
                    sd.set_tuning("checksum_stage_hot", hot)
                    sd.set_tuning("cpu_read_piece_kib", piece)
                    try:
                        check(L.sd_file_checksums(ctx.handle, arr, n, out, st.ctypes.data))
                    finally:
                        for k, v in keep.items():
                            sd.set_tuning(k, v)
                return f

            legs = [("cpu_16", cpu16()), ("cpu_16_p0", cpu16(0)), ("gpu_16", policy(0, 0, 1))]
            legs += [(f"hybrid_{g}", policy(2147483647, g, 1)) for g in (3, 4, 5, 6, 8)]
            legs += [(f"hybrid_{g}_files", policy(2147483647, g, 1, blocks=0)) for g in (4, 6)]
            if len(sys.argv) > 2:
                legs = [lg for lg in legs if lg[0] in sys.argv[2].split(",")]
            rounds = []
            for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):  # interleaved: host load drifts
                r = {k: timed(f) for k, f in legs}
                rounds.append(r)
                print(json.dumps({"set": name, "round": rnd, **r}), file=sys.stderr, flush=True)
            best = {k: max(r[k] for r in rounds) for k, _ in legs}
            med = {k: float(np.median([r[k] for r in rounds])) for k, _ in legs}
            out_all[name] = {"files": n, "bytes": total, "rounds": rounds, "best": best, "median": med,
                             "median_over_cpu_16": {k: med[k] / med["cpu_16"] for k in med}}
            for p in paths:
                os.unlink(p)
        print(json.dumps(out_all))
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
