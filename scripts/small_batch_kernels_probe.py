"""Kernel time vs batch size, latency kernels against throughput kernels, device-resident:
  sampled files: k_cas_sampled_wave (one wave per file) vs k_cas_sampled_lanes + _merge;
  whole files (configs[1] sizes, log-uniform 1..102400): k_whole_wave (one workgroup per
  file) vs the work-list kernels (k_whole_items + 2 x k_whole_merge8).
Per n: median of 20 launches after warm-up, outputs asserted equal.  Sets the
"sampled_wave_max" / "whole_wave_max" thresholds (profiles/r2/r2z_small_batch_kernels.json).
Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402

DEFAULTS = {b"sampled_wave_max": 6144, b"whole_wave_max": 512}


def sweep(ctx, stream, dev, kind, ns):
    key, part = (b"sampled_wave_max", 1) if kind == "sampled" else (b"whole_wave_max", 2)
    rng = np.random.default_rng(11)
    res = {}
    for n in ns:
        if kind == "sampled":
            sizes = (np.arange(n, dtype=np.uint64) * 7919 + 200_000)
        else:
            sizes = np.exp(rng.uniform(0, np.log(102400), n)).astype(np.uint64).clip(1, 102400)
        cids = np.arange(n, dtype=np.uint64) + 5
        ext, total = sd.stage_plan(sizes)
        d = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        d_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
        ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).to(dev), torch.from_numpy(cids.view(np.int64)).to(dev),
                            torch.zeros(n, dtype=torch.int32, device=dev), d_ext, n, d)
        row, outs = {}, []
        for name, thr in (("wave", 1 << 30), ("throughput", 0)):
            check(lib().sd_cas_set_tuning(key, thr))
            b = ctx.cas_batch(ext)
            h = torch.zeros(n * 32, dtype=torch.uint8, device=dev)
            for _ in range(5):
                b.run_part(part, d, h, stream)
            ts = []
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                b.run_part(part, d, h, stream)
                e1.record(stream)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            row[name + "_us"] = ts[len(ts) // 2]
            outs.append(h)
        check(lib().sd_cas_set_tuning(key, DEFAULTS[key]))
        assert torch.equal(outs[0], outs[1]), (kind, n)
        res[str(n)] = row
        del d, d_ext, outs
    return res


def main():
    """--large: the library-scale batches instead (the one-wave-per-file design of the
    north_star sketch against the shipped throughput kernels at 262 144 files, 500 000
    sampled files and configs[1]'s 1 M small files)."""
    dev = torch.device("cuda", 0)
    ctx = sd.Context(0)
    stream = torch.cuda.current_stream()
    if "--large" in sys.argv:
        out = {"sampled": sweep(ctx, stream, dev, "sampled", (262144, 500000)),
               "whole": sweep(ctx, stream, dev, "whole", (262144, 1000000))}
    else:
        out = {"sampled": sweep(ctx, stream, dev, "sampled", (1, 8, 64, 256, 1024, 2048, 4096, 8192, 16384, 65536)),
               "whole": sweep(ctx, stream, dev, "whole", (1, 16, 100, 256, 1024, 2048, 4096, 8192, 16384, 65536))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
