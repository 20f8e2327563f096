"""gpurun_out/ rocprofv3 output -> committed summaries under profiles/.

    python scripts/summarize_profiles.py TAG

Writes profiles/TAG_kernel_stats.csv (rocprofv3 --stats, verbatim), profiles/TAG_summary.md
(top kernels) and, if PMC passes exist, profiles/pmc_summary.json: per kernel and launch
FETCH_SIZE / WRITE_SIZE (KB), the read-probe calibration factor, and
hbm_bytes_per_launch = FETCH_SIZE * 1024 * factor + WRITE_SIZE * 1024.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
CALIB_BYTES = 4 << 30
CMD = os.environ.get("PROF_CMD", "python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras")
WARMUP = int(os.environ.get("PROF_WARMUP", "3"))
PMC_CMD = os.environ.get("PMC_CMD", "python3 bench.py --steps 1 --warmup 0 --checksum-steps 1 --no-cpu-baseline "
                                    "--no-extras --config-reps 1 --warm-ms 0")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].strip()


def pmc_rows(path):
    """(kernel, grid size in work-items) -> counter -> per-launch values; the launch
    duration under the counter pass goes in as the pseudo-counter "DURATION_NS"."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    seen = set()
    for r in csv.DictReader(open(path)):
        grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        key = (short(r["Kernel_Name"]), grid)
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r.get("Start_Timestamp") and (key, r["Dispatch_Id"]) not in seen:
            seen.add((key, r["Dispatch_Id"]))
            agg[key]["DURATION_NS"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return agg


def trace_shapes(tag):
    """(kernel, grid) -> launch durations in µs from the kernel-trace pass, or {}."""
    shapes = collections.defaultdict(list)
    tr = glob.glob(os.path.join(OUT, f"prof_{tag}", "*kernel_trace.csv"))
    if tr:
        for r in csv.DictReader(open(tr[0])):
            shapes[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return shapes


def steady(v):
    st = v[WARMUP:] if len(v) > WARMUP else v
    return sum(st) / len(st)


# The PMC pass's own launch durations include the counter collection's overhead, and
# GRBM_GUI_ACTIVE counts the GPU's busy cycles around a launch too: for short launches the
# ratio is no clock (round 2 printed 3.4-28.8 GHz).  The clock column therefore divides by
# the same launch shape's steady duration in the kernel-trace pass, and only for launches of
# at least MIN_CLOCK_US, where the overhead is small; others show "-".
MIN_CLOCK_US = 500.0
# ... and only for the compute-bound hashing kernels: a launch that waits (on peers, the
# host, or atomics) spends its trace duration idle, and no ratio of the two passes is a clock
CLOCK_KERNELS = ("k_cas_sampled_lanes", "k_cas_sampled_wave", "k_whole_items", "k_whole_wave", "k_ck_leaf")


def main(tag):
    os.makedirs(PROF, exist_ok=True)
    stats = glob.glob(os.path.join(OUT, f"prof_{tag}", "*kernel_stats.csv"))
    if stats:
        dst = os.path.join(PROF, f"{tag}_kernel_stats.csv")
        shutil.copy(stats[0], dst)
        rows = sorted(csv.DictReader(open(stats[0])), key=lambda r: -float(r["TotalDurationNs"]))
        with open(os.path.join(PROF, f"{tag}_summary.md"), "w") as f:
            f.write(f"# rocprofv3 --kernel-trace --stats ({tag})\n\n")
            f.write(f"Command: `rocprofv3 --kernel-trace --stats --output-format csv -- {CMD}` "
                    "(scripts/profile.sh)\n\n")
            f.write("| kernel | calls | avg µs | total ms | % |\n|---|---|---|---|---|\n")
            for r in rows[:20]:
                f.write(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                        f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |\n")
            shapes = trace_shapes(tag)
            if shapes:  # per launch shape: bench.py's timed launches vs the warm-up ones
                f.write("\nPer launch shape (kernel, grid size in work-items) for the hashing kernels, from "
                        "the kernel trace. `steady avg` drops the first `warmup` launches of the shape "
                        "(clock ramp), i.e. it covers the launches bench.py times.\n\n")
                f.write("| kernel | grid | calls | avg µs | steady avg µs | min µs |\n|---|---|---|---|---|---|\n")
                for (k, g), v in sorted(shapes.items(), key=lambda kv: -sum(kv[1])):
                    if not k.startswith(("k_cas", "k_whole", "k_ck", "k_gb", "k_part", "k_owners")):
                        continue
                    f.write(f"| `{k}` | {g} | {len(v)} | {sum(v) / len(v):.1f} | {steady(v):.1f} | "
                            f"{min(v):.1f} |\n")
        print("wrote", dst)
    pmc = {}
    for d in sorted(glob.glob(os.path.join(OUT, f"pmc_{tag}_*"))):
        f = glob.glob(os.path.join(d, "*counter_collection.csv"))
        if not f:
            continue
        for k, cs in pmc_rows(f[0]).items():
            for c, v in cs.items():
                pmc.setdefault(k, {})[c] = {"launches": len(v), "per_launch": sum(v) / len(v)}
    if not pmc:
        return
    calib = {}
    cf = glob.glob(os.path.join(OUT, f"calib_{tag}", "*counter_collection.csv"))
    if cf:
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(cf[0]))
                if short(r["Kernel_Name"]) == "k_read_probe" and r["Counter_Name"] == "FETCH_SIZE"]
        for pattern, v in zip((0, 1, 2), vals):
            calib[pattern] = CALIB_BYTES / (v * 1024)
    # k_cas_sampled_lanes (8 KiB per lane) / k_whole_items full pairs (2 KiB per lane) read in
    # line pairs (probe pattern 2); the checksum leaf 4 KiB per lane in the same shape
    use = {"k_cas_sampled_lanes": 2, "k_cas_sampled": 2, "k_whole_items": 2, "k_ck_leaf": 2}
    kern = {}
    for (k, grid), cs in sorted(pmc.items()):
        if "FETCH_SIZE" not in cs:
            continue
        fac = calib.get(use.get(k, 0), 2.0)
        fetch = cs["FETCH_SIZE"]["per_launch"] * 1024
        write = cs.get("WRITE_SIZE", {}).get("per_launch", 0.0) * 1024
        kern.setdefault(k, []).append({
            "grid": grid, "launches": cs["FETCH_SIZE"]["launches"],
            "FETCH_SIZE_KB": cs["FETCH_SIZE"]["per_launch"],
            "WRITE_SIZE_KB": cs.get("WRITE_SIZE", {}).get("per_launch"),
            "fetch_factor": fac, "hbm_bytes_per_launch": fetch * fac + write,
            "counters": {c: v["per_launch"] for c, v in cs.items()}})
    out = {"tag": tag, "calibration_fetch_factor_by_pattern": calib,
           "command": PMC_CMD,
           "note": "per kernel and launch shape (grid = work-items); hbm_bytes = FETCH_SIZE*1024*factor + "
                   "WRITE_SIZE*1024; factor from read probes of a known 4 GiB byte count (scripts/pmc_calib.py), "
                   "2.0 (MI355X_MICROARCH.md gfx950 rule) if absent.  bench.py emits roofline.traffic only for a "
                   "launch whose grid matches an entry here",
           "kernels": kern}
    json.dump(out, open(os.path.join(PROF, "pmc_summary.json"), "w"), indent=1)
    print("wrote profiles/pmc_summary.json")
    # the hashing and dedup kernels: HBM bytes, clock and VALU issue per launch shape
    with open(os.path.join(PROF, f"{tag}_pmc.md"), "w") as f:
        f.write(f"# rocprofv3 PMC per launch shape ({tag})\n\nCommand of every pass: `rocprofv3 --pmc <group> -- "
                f"{PMC_CMD}` (scripts/profile.sh); one counter group per pass.  HBM bytes = FETCH_SIZE x 1024 x "
                "calibrated factor + WRITE_SIZE x 1024 (factor from `scripts/pmc_calib.py`'s 4 GiB read probes: "
                f"{ {k: round(v, 4) for k, v in calib.items()} }).  MHz = GRBM_GUI_ACTIVE / 8 XCDs / the same launch "
                f"shape's steady duration in the kernel-trace pass (`{tag}_summary.md`), shown only for launches of "
                f"at least {MIN_CLOCK_US:.0f} µs of the compute-bound hashing kernels (GRBM_GUI_ACTIVE also counts the "
                "busy cycles around a launch, so short launches give no clock, and a launch that waits -- RCCL, the "
                "grouping's atomics -- is idle for part of its trace duration); lane-ops/clk/CU = SQ_INSTS_VALU x 64 lanes / (GUI cycles / 8 x 256 "
                "CUs), same rule: 64 is the measured issue ceiling of BLAKE3's G mix (scripts/valu_probe7.hip), "
                "128 the SIMD-32 full rate.\n\n")
        f.write("| kernel | grid | HBM GB/launch | VALU wave-insts | GUI cycles | trace µs | MHz | lane-ops/clk/CU |\n"
                "|---|---|---|---|---|---|---|---|\n")
        shapes = trace_shapes(tag)
        for k, lst in sorted(kern.items()):
            if not k.startswith(("k_cas", "k_whole", "k_ck", "k_gb", "k_part", "k_owners", "rccl")):
                continue
            for e in lst:
                c = e["counters"]
                gui, valu = c.get("GRBM_GUI_ACTIVE"), c.get("SQ_INSTS_VALU")
                tr_us = steady(shapes[(k, e["grid"])]) if shapes.get((k, e["grid"])) else None
                long_enough = tr_us is not None and tr_us >= MIN_CLOCK_US and k in CLOCK_KERNELS
                mhz = gui / 8 / tr_us if gui and long_enough else None
                ipc = valu * 64 / (gui / 8 * 256) if gui and valu and long_enough else None
                f.write(f"| `{k}` | {e['grid']} | {e['hbm_bytes_per_launch'] / 1e9:.4g} | "
                        f"{'%.4g' % valu if valu is not None else '-'} | {'%.4g' % gui if gui is not None else '-'} | "
                        f"{'%.1f' % tr_us if tr_us else '-'} | "
                        f"{'%.0f' % mhz if mhz else '-'} | {'%.1f' % ipc if ipc else '-'} |\n")
    print(f"wrote profiles/{tag}_pmc.md")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r1")
