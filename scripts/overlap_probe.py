"""A/B on one box: the library shard's hash phase with the sampled kernel and the
whole-file kernels on ONE stream (in order) vs on TWO streams (each kernel's tail filled by
the other's workgroups).  Alternates A and B `rounds` times, K back-to-back batches each.
python scripts/overlap_probe.py [files] [K] [rounds]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    dev = torch.device("cuda", 0)
    ctx = sd.Context(0)
    sizes, cids, twins = synth.library(0, n, n * 8)
    ext, total = sd.stage_plan(sizes)
    d_staged = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                        torch.from_numpy(twins.astype(np.int32)).to(dev), d_ext, n, d_staged)
    batch = ctx.cas_batch(ext)
    d_hash = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    ev = [torch.cuda.Event() for _ in range(2)]

    def one_stream():
        batch.run_part(1, d_staged, d_hash, s1)
        batch.run_part(2, d_staged, d_hash, s1)

    def two_streams():
        ev[0].record(s1)
        s2.wait_event(ev[0])  # both start after the previous batch on s1
        batch.run_part(1, d_staged, d_hash, s1)
        batch.run_part(2, d_staged, d_hash, s2)
        ev[1].record(s2)
        s1.wait_event(ev[1])

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e3

    for fn in (one_stream, two_streams):  # warm (clock ramp, allocations)
        timed(fn)
    res = {"one_stream_ms": [], "two_streams_ms": []}
    for _ in range(rounds):
        res["one_stream_ms"].append(timed(one_stream))
        res["two_streams_ms"].append(timed(two_streams))
    h1 = d_hash.clone()
    one_stream()
    torch.cuda.synchronize()
    res["equal"] = bool(torch.equal(h1, d_hash))
    res["files"] = n
    res["compressions"] = batch.compressions
    print(json.dumps(res))


if __name__ == "__main__":
    main()
