"""Writes tests/golden/bench_checksums.json: the C oracle's checksums of bench.py's multi-GiB
synthetic files, so a rank with a small host-thread share (2 threads per rank on an 8-GPU
node) compares its timed output with them instead of re-hashing 40+ GiB
on the host.

    python tests/golden/make_bench_golden.py [--threads 8]

Files (the bench's defaults: --files-per-gpu 1 250 000, --checksum-gib 64, --split-gib 32;
ranks 0..7 of the 8-GPU run, so every N in 1/2/4/8 finds its ranks):
  * configs[3]: files 0 and 15 of each rank's 16 x 4 GiB batch (cids 10000 + start + i);
  * configs[3] mixed: each rank's shortest 2..8 GiB file, which spans two generated files
    (bench.mixed_layout);
  * the split file: (32 GiB + 12345) bytes of cid 20000.
Everything is the oracle's output (oracle/sd_oracle_simd.c's chunk-parallel BLAKE3, itself
pinned to the published BLAKE3 vectors, tests/test_oracle.py) on the deterministic generator
of SURVEY.md §8(d); tests/test_bench_helpers.py re-derives entries on every CPU run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import native  # noqa: E402

FILES_PER_GPU = 1_250_000
RANKS = 8
CHECKSUM_GIB = 64
NF = 16
SPLIT_GIB = 32


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    flen = (CHECKSUM_GIB << 30) // NF
    total = NF * flen
    synth, mixed = {}, {}
    t0 = time.time()
    for r in range(RANKS):
        start = r * FILES_PER_GPU
        for i in (0, NF - 1):
            cid = 10_000 + start + i
            synth[f"{cid}:{flen}"] = native.checksum_synth_mt(flen, cid, 0, nthreads=a.threads).hex()
        offs, lens = bench.mixed_layout(start, total)
        mi = min(range(len(lens)), key=lambda k: lens[k])
        mixed[f"{start}:{total}"] = {"index": mi, "offset": offs[mi], "len": lens[mi],
                                     "hash": bench.mixed_host_checksum(start, offs[mi], lens[mi], flen, a.threads).hex()}
        print(f"rank {r}: {time.time() - t0:.1f}s", flush=True)
    split_len = (SPLIT_GIB << 30) + 12345
    synth[f"20000:{split_len}"] = native.checksum_synth_mt(split_len, 20_000, 0, nthreads=a.threads).hex()
    out = {"generator": "SURVEY.md 8(d) splitmix64 synthetic files (oracle/sd_oracle.c sdo_synth_fill)",
           "oracle": "oracle/sd_oracle_simd.c chunk-parallel BLAKE3 (sdo_checksum_synth_mt / sdo_checksum_mt)",
           "made_by": "tests/golden/make_bench_golden.py",
           "bench_defaults": {"files_per_gpu": FILES_PER_GPU, "checksum_gib": CHECKSUM_GIB, "files": NF,
                              "split_gib": SPLIT_GIB, "ranks": RANKS},
           "synth": synth, "mixed": mixed}
    with open(bench.GOLDEN_CHECKSUMS, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {bench.GOLDEN_CHECKSUMS} in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
