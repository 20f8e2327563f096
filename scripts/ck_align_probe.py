"""Does the start alignment of checksum files in device memory cost time?

configs[3]'s mixed variant (12 files of 2..8 GiB, unaligned lengths) packs the files at
16-byte aligned starts, so every file after the first starts mid cache line; its
k_ck_leaf launch fetched 1.33x the algorithmic bytes (profiles/r2z4_pmc.md, grid
16311808) and ran at 0.855 of the VALU bound against 0.90 for the aligned files.
This times the same file lengths over the same device buffer packed at 16, 128, 256
and 4096-byte starts (and, for reference, the aligned 16 x 4 GiB layout), alternating
the layouts so all see the same clock history.  Hashes must not depend on the layout.

    python scripts/ck_align_probe.py [--out gpurun_out/ck_align.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spacedrive_amd.device import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/ck_align.json")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    stream = torch.cuda.current_stream()
    cap = a.gib << 30
    rng = np.random.default_rng(7)
    lens, tot = [], 0
    while True:  # the bench's mixed lengths (bench.py, rank 0)
        ln = int(rng.integers(2 << 30, (8 << 30) + 1))
        if tot + ln + 4096 * 13 > cap:
            break
        lens.append(ln)
        tot += ln
    d_data = torch.empty(cap + 4096, dtype=torch.uint8, device=dev)
    layouts = {}
    for al in (16, 128, 256, 4096):
        offs, pos = [], 0
        for ln in lens:
            offs.append(pos)
            pos = (pos + ln + al - 1) // al * al
        layouts[f"start_align_{al}"] = offs
    res = {"files": len(lens), "bytes": tot, "lens": lens, "runs": {}}
    sums = {}
    for rnd in range(a.rounds):
        for name, offs in layouts.items():
            for i, (o, ln) in enumerate(zip(offs, lens)):  # same content at every layout
                ctx.synth_fill(20_001 + i, 0, ln, d_data[o:])
            cb = ctx.checksum_batch(offs, lens)
            d_sum = torch.empty(len(lens) * 32, dtype=torch.uint8, device=dev)
            cb.run(d_data, d_sum, stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                cb.run(d_data, d_sum, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            sums.setdefault(name, d_sum.cpu().numpy().tobytes().hex())
            res["runs"].setdefault(name, []).append(ms)
            print(f"round {rnd} {name:18s} {ms:8.3f} ms  {tot / ms / 1e6:8.1f} GB/s", flush=True)
            del cb, d_sum
    ref = sums["start_align_16"]
    res["hashes_equal_across_layouts"] = all(v == ref for v in sums.values())
    res["best_ms"] = {k: min(v) for k, v in res["runs"].items()}
    print(json.dumps({k: v for k, v in res.items() if k not in ("lens",)}), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f)
    if not res["hashes_equal_across_layouts"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
