"""configs[1] (k_whole_items + merge8) vs the library's whole-file part: per-launch times
over many back-to-back launches, alone and right after a long sampled-kernel run, to
separate the kernel's steady-state rate from the clock state it starts in (VERDICT r1
item 5).  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402


def stage(ctx, sizes, cids, twins, dev):
    ext, total = sd.stage_plan(sizes)
    d = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                        torch.from_numpy(twins.astype(np.int32)).to(dev), d_ext, len(sizes), d)
    return ext, d


def timed(fn, reps, stream):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        fn()
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]


def summary(ts, comp):
    st = ts[len(ts) // 3:]
    ms = sum(st) / len(st)
    return {"first5_ms": [round(t, 3) for t in ts[:5]], "steady_ms": ms, "min_ms": min(ts),
            "steady_valu_frac": comp * 672 / (ms * 1e-3) / 39.3216e12}


def main():
    dev = torch.device("cuda", 0)
    ctx = sd.Context(0)
    stream = torch.cuda.current_stream()
    s1, c1, t1 = synth.small_library(0, 1_000_000)
    ext1, d1 = stage(ctx, s1, c1, t1, dev)
    b1 = ctx.cas_batch(ext1)
    h1 = torch.empty(len(s1) * 32, dtype=torch.uint8, device=dev)
    n = 1_250_000
    sL, cL, tL = synth.library(0, n, n)
    extL, dL = stage(ctx, sL, cL, tL, dev)
    bL = ctx.cas_batch(extL)
    hL = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    out = {"configs1_compressions": b1.compressions}
    whole_L = bL.compressions - 953 * bL.n_sampled
    # configs[1] alone after an idle gap
    torch.cuda.synchronize()
    import time
    time.sleep(0.5)
    out["configs1_cold"] = summary(timed(lambda: b1.run(d1, h1, stream), 60, stream), b1.compressions)
    # configs[1] right after ~200 ms of the sampled kernel
    timed(lambda: bL.run_part(1, dL, hL, stream), 20, stream)
    out["configs1_after_sampled"] = summary(timed(lambda: b1.run(d1, h1, stream), 60, stream), b1.compressions)
    # the library's whole part: alone (back to back), and interleaved with the sampled kernel
    time.sleep(0.5)
    out["library_whole_alone"] = summary(timed(lambda: bL.run_part(2, dL, hL, stream), 60, stream), whole_L)
    ts = []
    for _ in range(40):
        bL.run_part(1, dL, hL, stream)
        ts += timed(lambda: bL.run_part(2, dL, hL, stream), 1, stream)
    out["library_whole_after_sampled"] = summary(ts, whole_L)
    # configs[1] interleaved with the sampled kernel (as in the library step)
    ts = []
    for _ in range(40):
        bL.run_part(1, dL, hL, stream)
        ts += timed(lambda: b1.run(d1, h1, stream), 1, stream)
    out["configs1_interleaved"] = summary(ts, b1.compressions)
    out["items"] = {"configs1": [b1.full_items, b1.tail_items], "library": [bL.full_items, bL.tail_items]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
