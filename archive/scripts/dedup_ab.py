"""A/B of sd_dedup_group variants on one GPU (1.25 M index-sorted records, 10 % dups).

    python scripts/dedup_ab.py [--m 1250000] [--reps 20]

Times each "dedup_variant" with HIP events on the launch stream (the call syncs on the
group count, so per-call wall time is also reported) and asserts identical outputs.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1250000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--library", action="store_true", help="records of bench.py's library shard instead of random keys")
    ap.add_argument("--big", type=int, default=0,
                    help="random keys plus this many groups of 1400 (one rank's share of the 10 M library's size-1 files at N=8)")
    a = ap.parse_args()
    ctx = sd.Context(0)
    if a.library:  # the bench's shard: hash it on the device, then partition (nparts 1)
        from spacedrive_amd import synth
        sizes, cids, twins = synth.library(0, a.m, a.m)
        ext, total = sd.stage_plan(sizes)
        d_staged = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        d_ext = torch.from_numpy(ext.view(np.uint8).copy()).cuda()
        ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                            torch.from_numpy(twins.astype(np.int32)).cuda(), d_ext, a.m, d_staged)
        batch = ctx.cas_batch(ext)
        d_hash = torch.empty(a.m * 32, dtype=torch.uint8, device="cuda")
        batch.run(d_staged, d_hash)
        del d_staged
        counts = torch.empty(1, dtype=torch.int64, device="cuda")
        recs = torch.empty((a.m, 2), dtype=torch.int64, device="cuda")
        nv = ctx.dedup_partition(d_hash.view(a.m, 32), torch.from_numpy((sizes != 0).astype(np.uint8)).cuda(), a.m, 0,
                                 1, counts, recs)
        src = recs[:nv].clone()
        a.m = nv
    else:
        rng = np.random.default_rng(1)
        keys = rng.integers(-2**63, 2**63 - 1, a.m, dtype=np.int64)
        dup = rng.choice(a.m, a.m // 10, replace=False)
        keys[dup] = keys[rng.integers(0, a.m, len(dup))]
        for g in range(a.big):
            keys[rng.choice(a.m, 1400, replace=False)] = keys[g]
        src = torch.from_numpy(np.stack([keys, np.arange(a.m, dtype=np.int64)], axis=1)).cuda()
    k = src[:, 0].cpu().numpy().view(np.uint64)
    lg = 1
    while lg < 24 and (48 << lg) < a.m:
        lg += 1
    span = int(k.max()) - int(k.min())
    sh = max(span.bit_length() - lg, 0)
    bsz = np.bincount(((k - k.min()) >> np.uint64(sh)).astype(np.int64), minlength=1 << lg)
    _, gs = np.unique(k, return_counts=True)
    print(f"records {a.m}: {1 << lg} buckets, mean {a.m / (1 << lg):.1f}, max {bsz.max()}, >128: {(bsz > 128).sum()}, "
          f"sum s^2 {float((bsz.astype(np.float64) ** 2).sum()):.3g}; largest group {gs.max()}", flush=True)
    outs = {}
    for v in (0, 1, 0, 1):
        lib().sd_cas_set_tuning(b"dedup_variant", v)
        rec = torch.empty_like(src)
        rep = torch.empty(a.m, dtype=torch.int64, device="cuda")
        ms, wall = [], []
        for _ in range(a.reps + 3):
            rec.copy_(src)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            ng = ctx.dedup_group(rec, a.m, rep, index_sorted=True)
            e1.record()
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e3)
            ms.append(e0.elapsed_time(e1))
        print(f"dedup_variant {v}: events {np.mean(ms[3:]):.3f} ms, wall {np.mean(wall[3:]):.3f} ms, groups {ng}",
              flush=True)
        outs.setdefault(v, (rec.cpu().numpy(), rep.cpu().numpy(), ng))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]
    lib().sd_cas_set_tuning(b"dedup_variant", 1)
    print("outputs identical")


if __name__ == "__main__":
    main()
