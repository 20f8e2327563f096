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
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    keys = rng.integers(-2**63, 2**63 - 1, a.m, dtype=np.int64)
    dup = rng.choice(a.m, a.m // 10, replace=False)
    keys[dup] = keys[rng.integers(0, a.m, len(dup))]
    src = torch.from_numpy(np.stack([keys, np.arange(a.m, dtype=np.int64)], axis=1)).cuda()
    ctx = sd.Context(0)
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
