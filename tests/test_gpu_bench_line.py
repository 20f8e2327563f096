"""bench.py end to end on the GPU at reduced sizes: the run exits 0, stdout carries exactly
one JSON line inside the driver's budget with the contract keys first, every leg's oracle
check reports zero mismatches, and the full record lands in the file the line names.  The
driver's own bench runs the default sizes; this guards the emitter and every leg's plumbing
in the driver-run GPU tests."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

SMALL = ["--steps", "3", "--warmup", "1", "--files-per-gpu", "60000", "--checksum-gib", "1", "--checksum-steps", "2",
         "--split-gib", "1", "--config-files", "20000", "--config-reps", "3", "--warm-ms", "20",
         "--file-backed-files", "20000", "--identifier-files", "10000", "--host-staged-files", "20000",
         "--host-checksum-gib", "1", "--file-checksum-mib", "1024", "--latency-calls", "40", "--cpu-seconds", "0.3"]


def test_bench_small_run_emits_one_compact_line(tmp_path):
    full = str(tmp_path / "full.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--full-out", full], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    line = lines[0]
    assert len(line) <= bench.LINE_TARGET
    d = json.loads(line)
    assert list(d)[:len(bench.STD_KEYS)] == list(bench.STD_KEYS)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    assert list(d)[len(bench.STD_KEYS):len(bench.STD_KEYS) + 2] == ["roofline", "cpu_baseline"]
    assert 0 < d["roofline"]["frac"] < 1.2 and d["roofline"]["kernel_ms"] > 0
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1
    # every leg's oracle check: [files, mismatches] with zero mismatches
    assert d["parity"]["sample"][1] == 0 and d["parity"]["full"] == [60000, 0]
    for k, v in d["legs"].items():
        for pk in ("parity", "parity_full", "mixed_parity"):
            if pk in v:
                assert v[pk][1] == 0 and v[pk][0] > 0, (k, pk, v[pk])
    assert d["legs"]["configs_small"]["parity_full"] == [20000, 0]
    assert d["legs"]["configs_sampled"]["parity_full"] == [20000, 0]
    assert d["dedup"]["parity"] is True and d["dedup"]["records_per_rank"] == [d["dedup"]["records"]]
    assert d["full_record"] == full
    with open(full) as f:
        rec = json.load(f)
    assert abs(rec["value"] / d["value"] - 1) < 1e-3 and "note" in rec["steps_serial"]
