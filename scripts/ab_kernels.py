"""Interleaved A/B timing of kernel variants in one process (cdna_hip_programming.md §5.4
rule 24), with a bit-exactness check of every variant's output against the first.

    python scripts/ab_kernels.py --what sampled --variants 10,11,20,21,40,41
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="sampled", choices=["sampled", "whole", "library", "checksum"])
    ap.add_argument("--variants", default="10,11,20,21,40,41")
    ap.add_argument("--files", type=int, default=500_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--checksum-gib", type=int, default=16)
    ap.add_argument("--key", default=None, help="tuning key the variants set (default: by --what)")
    ap.add_argument("--set", default="", help="extra fixed tuning, e.g. whole_variant=7")
    args = ap.parse_args()
    import spacedrive_amd as sd
    from spacedrive_amd import synth
    from spacedrive_amd._native import lib

    key = {"sampled": b"sampled_variant", "whole": b"whole_variant", "library": b"whole_variant",
           "checksum": b"checksum_variant"}[args.what] if args.key is None else args.key.encode()
    variants = [int(v) for v in args.variants.split(",")]
    for kv in filter(None, args.set.split(",")):
        k, v = kv.split("=")
        assert lib().sd_cas_set_tuning(k.encode(), int(v)) == 0
    ctx = sd.Context(0)
    dev = torch.device("cuda", 0)
    if args.what in ("sampled", "whole", "library"):
        n = args.files
        if args.what == "library":
            sizes, cids, twins = synth.library(0, n, n)
        else:
            gen = synth.sampled_library if args.what == "sampled" else synth.small_library
            sizes, cids, twins = gen(0, n)
        ext, total = sd.stage_plan(sizes)
        data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                            torch.from_numpy(twins.astype(np.int32)).to(dev),
                            torch.from_numpy(ext.view(np.uint8).copy()).to(dev), n, data)
        b = ctx.cas_batch(ext)
        nout = n
    else:
        nf = 16
        flen = (args.checksum_gib << 30) // nf
        data = torch.empty(nf * flen + 128, dtype=torch.uint8, device=dev)
        for i in range(nf):
            ctx.synth_fill(77 + i, 0, flen, data[i * flen:])
        b = ctx.checksum_batch([i * flen for i in range(nf)], [flen] * nf)
        nout = nf
    out = torch.zeros(nout * 32, dtype=torch.uint8, device=dev)
    ref = None
    times = {v: [] for v in variants}
    for r in range(args.rounds):
        for v in variants:
            assert lib().sd_cas_set_tuning(key, v) == 0
            out.zero_()
            b.run(data, out)
            torch.cuda.synchronize()
            h = out.cpu().numpy()
            if ref is None:
                ref = h.copy()
            assert np.array_equal(h, ref), f"variant {v} differs"
            times[v].append(b.time(data, out, args.iters) / args.iters)
    res = {}
    for v in variants:
        t = sorted(times[v])
        ms = t[len(t) // 2]
        comp = b.compressions
        res[v] = {"median_ms": ms, "min_ms": t[0], "Tops": comp * 672 / (ms * 1e-3) / 1e12,
                  "GBps": (b.msg_bytes if hasattr(b, "msg_bytes") else b.total_bytes) / (ms * 1e-3) / 1e9}
    print(json.dumps({"what": args.what, "n": nout, "compressions": b.compressions, "variants": res}, indent=1))


if __name__ == "__main__":
    main()
