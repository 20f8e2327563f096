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
  * the split file: (32 GiB + 12345) bytes of cid 20000;
  * cas_digest: SHA-256 of the concatenated 8-byte cas_ids, in file order, of every
    rank's whole 1.25 M-file shard at N = 1, 2, 4 and 8 (a shard's files depend on the
    library size: duplicates point across it), and of configs[1] / configs[2]'s 1 M files
    -- the bench checks ALL of its timed output against these (a checksum of checksums),
    and still compares a 4 096-file sample's full 32-byte hashes with the oracle live.
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
CONFIG_FILES = 1_000_000


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only-digests", action="store_true", help="keep the checksums, recompute cas_digest")
    a = ap.parse_args()
    if a.only_digests:
        with open(bench.GOLDEN_CHECKSUMS) as f:
            out = json.load(f)
        out["cas_digest"] = digests(a.threads)
        write(out)
        return
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
           "synth": synth, "mixed": mixed, "cas_digest": digests(a.threads)}
    write(out)
    print(f"done in {time.time() - t0:.1f}s")


def digests(threads: int) -> dict:
    from spacedrive_amd import synth as sy
    d = {}
    t0 = time.time()
    for world in (1, 2, 4, 8):
        for r in range(world):
            start, n_total = r * FILES_PER_GPU, world * FILES_PER_GPU
            s, c, tw = sy.library(start, FILES_PER_GPU, n_total)
            ids = native.cas_ids_synth_simd(s, c, tw, nthreads=threads)
            d[bench.library_digest_key(start, FILES_PER_GPU, n_total)] = bench.cas_digest(ids)
            print(f"library shard {r}/{world}: {time.time() - t0:.1f}s", flush=True)
    for which, gen in (("small", sy.small_library), ("sampled", sy.sampled_library)):
        s, c, tw = gen(0, CONFIG_FILES)
        ids = native.cas_ids_synth_simd(s, c, tw, nthreads=threads)
        d[bench.config_digest_key(which, CONFIG_FILES)] = bench.cas_digest(ids)
        print(f"configs {which}: {time.time() - t0:.1f}s", flush=True)
    return d


def write(out: dict) -> None:
    with open(bench.GOLDEN_CHECKSUMS, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {bench.GOLDEN_CHECKSUMS}")


if __name__ == "__main__":
    main()
