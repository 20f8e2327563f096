"""Print the interesting numbers of a bench.py JSON line (last line of the file)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
SKIP = ("note", "peak_basis", "workload", "sample", "per_unit", "traffic_source")


def show(k, v, ind=0):
    if isinstance(v, dict):
        print(" " * ind + k + ":")
        for kk, vv in v.items():
            if kk not in SKIP:
                show(kk, vv, ind + 2)
    elif isinstance(v, float):
        print(" " * ind + f"{k}: {v:.4g}")
    else:
        print(" " * ind + f"{k}: {v}")


for k in (sys.argv[2:] or ["value", "ms_per_step", "roofline", "kernels", "dedup", "with_h2d", "file_backed",
                           "file_backed_checksum", "latency", "checksum", "configs", "cpu_baseline"]):
    show(k, d.get(k))
