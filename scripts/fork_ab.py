"""A/B of "batch_fork" on the bench's library shard (1.25 M files, 40% sampled): the
whole-kind kernels (k_whole_items + 2 x k_whole_merge8) on a side stream beside the
sampled pair (k_cas_sampled_lanes + _merge) vs all on one stream.  One process, the two
variants alternated launch by launch after a warm-up, HIP events on the caller's stream
(the fork joins back into it), outputs asserted identical.
python scripts/fork_ab.py [files] [rounds] -> one JSON line"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = sd.default_context(0)
    sizes, cids, twins = synth.library(0, n, 10_000_000)
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), n, d)
    b = ctx.cas_batch(ext)
    s = torch.cuda.current_stream()
    outs = {v: torch.zeros(n * 32, dtype=torch.uint8, device="cuda") for v in (0, 1)}
    times = {0: [], 1: []}
    for r in range(rounds + 5):
        for v in (0, 1) if r % 2 == 0 else (1, 0):
            sd.set_tuning("batch_fork", v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            b.run(d, outs[v], s)
            e1.record(s)
            e1.synchronize()
            if r >= 5:
                times[v].append(e0.elapsed_time(e1))
    sd.set_tuning("batch_fork", 0)
    same = bool(torch.equal(outs[0], outs[1]))
    res = {"files": n, "sampled": b.n_sampled, "rounds": rounds, "equal": same,
           "one_stream_ms": {"median": float(np.median(times[0])), "min": float(np.min(times[0]))},
           "fork_ms": {"median": float(np.median(times[1])), "min": float(np.min(times[1]))}}
    res["speedup_median"] = res["one_stream_ms"]["median"] / res["fork_ms"]["median"]
    print(json.dumps(res))
    assert same


if __name__ == "__main__":
    main()
