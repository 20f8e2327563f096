"""bench.py's stdout line: the driver lost round 5's 24.4 KB line, so
the line is now a compact record, the standard keys complete and first, then `roofline`,
then `cpu_baseline`, then one short record per leg; the full record goes to a file.  Fed here
with recorded full results: the N = 1 default run (r5zt) and the 8-rank rehearsal (r5zr), the
latter also reshaped as an 8-GPU RCCL line (rccl_libs present, 8 ranks of records)."""
import copy
import io
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

R5 = os.path.join(ROOT, "profiles", "r5")


def _load(name):
    with open(os.path.join(R5, name)) as f:
        return json.load(f)


def _n8_rccl():
    """the 8-rank rehearsal record as the 8-GPU node's line would carry it over RCCL"""
    d = _load("r5zr_rehearse8.json")
    d["distributed"] = dict(d["distributed"], backend="nccl", dedup_transport="rccl",
                            rccl_libs=_load("r5zt_bench.json")["distributed"]["rccl_libs"])
    d["dedup"] = dict(d["dedup"], transport="rccl", records_per_rank=[1250000 + 37 * r for r in range(8)],
                      phases_ms_max_over_ranks={"partition": 0.04, "allgather_rows": 0.05, "host_turnaround": 0.02,
                                                "sendrecv": 0.9, "group_owners": 0.25})
    d["launch"] = dict(d["launch"], share_gpu=False, devices_used=8)
    return d


RECORDS = {"n1_default": lambda: _load("r5zt_bench.json"), "n8_rehearsal": lambda: _load("r5zr_rehearse8.json"),
           "n8_rccl": _n8_rccl}


@pytest.mark.parametrize("which", sorted(RECORDS))
def test_line_fits_and_parses(which, tmp_path):
    out = RECORDS[which]()
    s = io.StringIO()
    full = str(tmp_path / "full.json")
    line = bench.emit(out, s, full)
    assert s.getvalue() == line + "\n" and "\n" not in line
    assert len(line) <= bench.LINE_BUDGET
    assert len(line) <= bench.LINE_TARGET  # fits the driver's 8.4 KB stdout tail whole
    d = json.loads(line)
    # the standard keys, complete and first, in the contract's order
    assert list(d)[:len(bench.STD_KEYS)] == list(bench.STD_KEYS)
    for k in bench.STD_KEYS:
        assert k in d
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["n_gpus"] == out["n_gpus"]
    assert d["steps"] == out["steps"] and d["warmup"] == out["warmup"]
    assert d["value"] == out["value"] and d["ms_per_step"] == out["ms_per_step"]  # full precision
    assert list(d)[len(bench.STD_KEYS)] == "roofline"
    for k in ("frac", "frac_full_rate", "achieved", "peak", "kernel_ms", "bound", "unit"):
        assert k in d["roofline"], k
    # the full record is on disk, unchanged
    with open(full) as f:
        assert json.load(f) == out
    assert d["full_record"] == full


def test_n1_line_carries_cpu_baseline_and_legs():
    d = json.loads(bench.emit(_load("r5zt_bench.json"), io.StringIO()))
    assert list(d)[len(bench.STD_KEYS) + 1] == "cpu_baseline"
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample", "single_thread", "all_cores", "host_cpu", "end_to_end"):
        assert k in cb, k
    for k in ("with_h2d_cas", "with_h2d_checksum", "file_backed_cas", "file_backed_checksum"):
        assert {"ratio", "host_share"} <= set(cb["end_to_end"][k]), k
    legs = d["legs"]
    for k in ("configs_small", "configs_sampled"):
        assert legs[k]["parity_full"] == [1_000_000, 0] and legs[k]["valu_frac"] > 0
    assert legs["checksum"]["parity"] == [2, 0]
    assert d["roofline"]["traffic"] and d["roofline"]["issue_rate_pmc_frac"] and d["roofline"]["sclk_mhz_median"]


def test_n8_line_keeps_balance_and_rccl():
    d = json.loads(bench.emit(_n8_rccl(), io.StringIO()))
    assert d["n_gpus"] == 8 and d["distributed"]["world"] == 8
    assert d["distributed"]["rccl_libs"]["one_rccl"] is True
    assert len(d["dedup"]["records_per_rank"]) == 8
    assert d["parity"]["full"] == [2_400_000, 0] and d["parity"]["ranks"] == 8
    # the with-H2D leg runs on every rank at once: the line keeps the aggregate
    assert d["legs"]["with_h2d_cas"]["aggregate_files_per_s"] > d["legs"]["with_h2d_cas"]["end_to_end"]


def test_overlong_line_fails_loudly():
    out = _load("r5zt_bench.json")
    out = copy.deepcopy(out)
    out["config"]["workload"] = "x" * (bench.LINE_BUDGET + 1)
    with pytest.raises(SystemExit):
        bench.emit(out, io.StringIO())


def test_sig_rounds_floats_only():
    assert bench._sig({"a": 1.23456789, "b": [2.0004999, 7], "c": "1.23456"}) == {"a": 1.235, "b": [2.0, 7],
                                                                                   "c": "1.23456"}
