"""Which limit holds the hashing kernels' clock at 2.2-2.3 GHz (round 5)?  power_probe.py
showed the board under its 1400 W cap while the clock drops from 2.39 GHz (the G block from
registers, or a plain HBM read) to 2.2 GHz (the hashing kernels: both at once).  This probe
asks the SMU: amdsmi's violation counters (PPT = package power, socket / VR / HBM thermal,
PROCHOT, "gfx clock below the host limit" split into its power and thermal causes, per XCP)
are read before and after each workload loops for a few seconds, and the GPU metrics table
(per-XCD gfx clocks, socket power, hotspot / memory / VR temperatures, throttle status) is
sampled every 50 ms while it runs.

  idle, valu_peak (k_valu_peak), hbm_read (a coalesced 16 GiB read; _nt: its loads marked
  non-temporal, to compare the energy per byte), sampled (CasBatch.run over
  250 000 sampled files), checksum (ChecksumBatch.run over 4 x 1 GiB)

python scripts/clock_limit_probe.py [seconds per mode=4] -> one JSON line"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spacedrive_amd as sd  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402

METRICS = ("current_socket_power", "temperature_hotspot", "temperature_mem", "temperature_vrgfx",
           "temperature_vrsoc", "temperature_vrmem", "average_gfx_activity", "current_uclk",
           "throttle_status", "indep_throttle_status")
ACC = ("acc_counter", "acc_prochot_thrm", "acc_ppt_pwr", "acc_socket_thrm", "acc_vr_thrm", "acc_hbm_thrm",
       "acc_gfx_clk_below_host_limit")
ACC_XCP = ("acc_gfx_clk_below_host_limit_pwr", "acc_gfx_clk_below_host_limit_thm",
           "acc_gfx_clk_below_host_limit_total", "acc_low_utilization")


def my_handle(amdsmi):
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    mine = buf.value.decode().lower() if hip.hipDeviceGetPCIBusId(buf, 64, 0) == 0 else ""
    for h in amdsmi.amdsmi_get_processor_handles():
        if amdsmi.amdsmi_get_gpu_device_bdf(h).lower() == mine:
            return h, mine
    return None, mine


def nums(v):
    """amdsmi gives ints, "N/A", lists, or per-XCP dicts/lists of them: keep the numbers."""
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, dict):
        return {k: nums(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [nums(x) for x in v]
    return None


def violations(amdsmi, h):
    try:
        v = amdsmi.amdsmi_get_violation_status(h)
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)}
    out = {k: nums(v.get(k)) for k in ACC}
    for k in ACC_XCP:
        out[k] = nums(v.get(k))
    return out


def delta(a, b):
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return b - a
    if isinstance(a, dict) and isinstance(b, dict):
        return {k: delta(a[k], b[k]) for k in a if k in b}
    if isinstance(a, list) and isinstance(b, list):
        return [delta(x, y) for x, y in zip(a, b)]
    return None


def flat_nums(v):
    if isinstance(v, (int, float)):
        return [v]
    if isinstance(v, dict):
        return [x for y in v.values() for x in flat_nums(y)]
    if isinstance(v, list):
        return [x for y in v for x in flat_nums(y)]
    return []


def sample(amdsmi, h, stop, rows):
    while not stop.is_set():
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            row = {k: nums(m.get(k)) for k in METRICS}
            g = [c for c in (nums(m.get("current_gfxclks")) or []) if isinstance(c, int) and 0 < c < 10000]
            row["gfxclk_mean"] = float(np.mean(g)) if g else None
            row["gfxclk_min"] = min(g) if g else None
            rows.append(row)
        except Exception as e:  # noqa: BLE001
            rows.append({"error": repr(e)})
        time.sleep(0.05)


def summarize(rows):
    out = {}
    for k in sorted({k for r in rows for k in r if k != "error"}):
        v = np.array([r[k] for r in rows if isinstance(r.get(k), (int, float))], np.float64)
        if len(v):
            out[k] = {"median": float(np.median(v)), "max": float(v.max()), "min": float(v.min())}
    errs = [r["error"] for r in rows if "error" in r]
    if errs:
        out["errors"] = errs[:3]
    return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    import amdsmi
    ctx = sd.default_context(0)
    amdsmi.amdsmi_init()
    h, bdf = my_handle(amdsmi)
    res = {"bdf": bdf, "found": h is not None, "seconds": secs, "modes": {}}
    if h is None:
        print(json.dumps(res))
        return
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
    ck_off = [i * (GiB + 128) for i in range(4)]
    d_ck = torch.empty(4 * (GiB + 128) + 64, dtype=torch.uint8, device="cuda")
    for i in range(4):
        ctx.synth_fill(40_000 + i, 0, GiB, d_ck[ck_off[i]:])
    ck = ctx.checksum_batch(ck_off, [GiB] * 4)
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
        "hbm_read_nt": lambda: check(L.sd_read_probe(ctx.handle, d_rd.data_ptr(), d_rd.numel(), 3, s)),
        "sampled": lambda: cas.run(d_st, d_hash),
        "checksum": lambda: ck.run(d_ck, d_ckh),
    }
    for name, fn in modes.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        time.sleep(1.0)
        v0 = violations(amdsmi, h)
        rows, stop = [], threading.Event()
        t = threading.Thread(target=sample, args=(amdsmi, h, stop, rows), daemon=True)
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
        v1 = violations(amdsmi, h)
        d = delta(v0, v1) if "error" not in v0 and "error" not in v1 else {"v0": v0, "v1": v1}
        frac = {}
        n_acc = d.get("acc_counter") if isinstance(d, dict) else None
        if isinstance(n_acc, (int, float)) and n_acc > 0:
            for k, x in d.items():
                if k == "acc_counter":
                    continue
                xs = [y for y in flat_nums(x) if isinstance(y, (int, float))]
                if xs:
                    frac[k] = round(max(xs) / n_acc, 4)
        moved = {"hbm_read": d_rd.numel(), "hbm_read_nt": d_rd.numel(), "sampled": total, "checksum": 4 * GiB}.get(name)
        res["modes"][name] = {"launches": launches, "s_per_launch": dt / launches, "metrics": summarize(rows),
                              "TBps": moved / (dt / launches) / 1e12 if moved else None,
                              "violation_delta": d, "violation_frac_of_samples": frac}
        print(name, json.dumps(res["modes"][name]["metrics"]), json.dumps(frac), file=sys.stderr, flush=True)
    amdsmi.amdsmi_shut_down()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
