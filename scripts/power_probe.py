"""Board power, shader clock and temperature while one workload loops for a few seconds:
is the hashing kernels' clock under load (2.1-2.2 GHz against 2.38 GHz for the G mix from
registers) set by the power limit?  hwmon sysfs of the visible card, sampled every 20 ms
on a host thread while the GPU runs:

  idle        nothing launched (the board's floor)
  valu_peak   k_valu_peak: the kernels' G block from registers (sd_valu_peak)
  hbm_read    sd_read_probe pattern 0: a coalesced 16 GiB read, no hashing
  hbm_read_lane_1k / _2k   the same bytes read as the hashing kernels do: one lane per 1 KiB
              chunk (2 KiB chunk pair), 16 B loads walking it -- energy per byte by pattern
  sampled     CasBatch.run over 250 000 sampled files (k_cas_sampled_lanes + _merge)
  checksum    ChecksumBatch.run over 4 x 1 GiB (k_ck_leaf + k_ck_reduce)

python scripts/power_probe.py [seconds per mode] -> one JSON line"""
import glob
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402


def hwmon_dirs():
    """The visible device's hwmon first (matched by PCI address: the host's other cards are
    listed in sysfs too), then the rest."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    mine = ""
    if hip.hipDeviceGetPCIBusId(buf, 64, 0) == 0:
        mine = buf.value.decode().lower()
    out = []
    for h in sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*")):
        names = os.listdir(h)
        if any(n.startswith("power1") for n in names) or "freq1_input" in names:
            pci = os.path.basename(os.path.realpath(os.path.join(h, "..", ".."))).lower()
            out.insert(0, h) if mine and pci == mine else out.append(h)
    return out


def read_int(p):
    try:
        with open(p) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


def sample(dirs, stop, rows):
    while not stop.is_set():
        row = {}
        for i, h in enumerate(dirs):
            for key in ("power1_average", "power1_input", "freq1_input", "temp1_input", "temp2_input",
                        "power1_cap"):
                v = read_int(os.path.join(h, key))
                if v is not None:
                    row[f"{i}:{key}"] = v
        rows.append(row)
        time.sleep(0.02)


def summarize(rows):
    keys = sorted({k for r in rows for k in r})
    out = {}
    for k in keys:
        v = np.array([r[k] for r in rows if k in r], dtype=np.float64)
        if len(v):
            out[k] = {"median": float(np.median(v)), "max": float(v.max()), "n": int(len(v))}
    return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    ctx = sd.default_context(0)
    dirs = hwmon_dirs()
    res = {"hwmon": dirs, "hwmon_of_this_device": dirs[0] if dirs else None, "seconds": secs, "modes": {}}
    # inputs
    n = 250_000
    sizes = np.full(n, 1 << 30, np.uint64) + np.arange(n, dtype=np.uint64)
    cids = np.arange(n, dtype=np.uint64)
    ext, total = sd.stage_plan(sizes)
    d_st = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_stage_cas(torch.from_numpy(sizes.view(np.int64)).cuda(), torch.from_numpy(cids.view(np.int64)).cuda(),
                        torch.zeros(n, dtype=torch.int32, device="cuda"),
                        torch.from_numpy(ext.view(np.uint8).copy()).cuda(), n, d_st)
    cas = ctx.cas_batch(ext)
    d_hash = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    GiB = 1 << 30
    ck_len = [GiB] * 4
    ck_off = [i * (GiB + 128) for i in range(4)]
    d_ck = torch.empty(4 * (GiB + 128) + 64, dtype=torch.uint8, device="cuda")
    for i in range(4):
        ctx.synth_fill(40_000 + i, 0, GiB, d_ck[ck_off[i]:])
    ck = ctx.checksum_batch(ck_off, ck_len)
    d_ckh = torch.empty(4 * 32, dtype=torch.uint8, device="cuda")
    d_rd = torch.empty(16 * GiB, dtype=torch.uint8, device="cuda")
    d_rd.fill_(7)
    torch.cuda.synchronize()
    L = lib()
    s = torch.cuda.current_stream().cuda_stream
    modes = {
        "idle": lambda: time.sleep(0.005),
        "valu_peak": lambda: ctx.valu_peak(),
        "hbm_read": lambda: check(L.sd_read_probe(ctx.handle, d_rd.data_ptr(), d_rd.numel(), 0, s)),
        "hbm_read_lane_1k": lambda: check(L.sd_read_probe(ctx.handle, d_rd.data_ptr(), d_rd.numel(), 1, s)),
        "hbm_read_lane_2k": lambda: check(L.sd_read_probe(ctx.handle, d_rd.data_ptr(), d_rd.numel(), 2, s)),
        "sampled": lambda: cas.run(d_st, d_hash),
        "checksum": lambda: ck.run(d_ck, d_ckh),
    }
    for name, fn in modes.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        time.sleep(1.0)  # settle
        rows, stop = [], threading.Event()
        t = threading.Thread(target=sample, args=(dirs, stop, rows), daemon=True)
        launches = 0
        t0 = time.perf_counter()
        t.start()
        while time.perf_counter() - t0 < secs:
            fn()
            launches += 1
            if launches % 4 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        stop.set()
        t.join()
        res["modes"][name] = {"launches": launches, "s_per_launch": dt / launches, "sensors": summarize(rows)}
        print(name, json.dumps(res["modes"][name]), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
