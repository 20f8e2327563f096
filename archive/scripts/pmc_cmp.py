"""Summarise rocprofv3 --pmc output dirs: per kernel (short name) the counters averaged per
dispatch, plus VALU busy = SQ_INSTS_VALU * 4 / (SIMDs * GRBM_GUI_ACTIVE / XCDs) and
wave-instructions per compression where the caller gives compressions per dispatch.

    python scripts/pmc_cmp.py DIR [DIR ...]
"""
import collections
import csv
import glob
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].strip()


for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            agg[short(r["Kernel_Name"])][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    print(f"== {d}")
    for k, cs in agg.items():
        per = collections.defaultdict(list)
        for (c, disp), v in cs.items():
            per[c].append(sum(v))
        avg = {c: sum(v) / len(v) for c, v in per.items()}
        line = ", ".join(f"{c}={v:.4g}" for c, v in sorted(avg.items()))
        if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
            busy = avg["SQ_INSTS_VALU"] * 4 / (1024 * avg["GRBM_GUI_ACTIVE"] / 8)
            line += f", VALU_busy={busy:.3f}"
        print(f"  {k}: n={len(next(iter(per.values())))} {line}")
