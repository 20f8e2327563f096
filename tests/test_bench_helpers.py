"""bench.py's own checking machinery, on the CPU: every leg's oracle check goes through
`parity` (a mismatch must fail the run), the even-stride `sample_idx`, and `oracle_hashes`
(the oracle's full hashes of a sample of synthetic files, built from the generator the
device kernels use).  The sampled rows must be the rows of the whole set: the same cas_ids
as the oracle's own synthetic cas path over all files, and as the library's CPU path over
the oracle-staged messages."""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd._native import check, lib  # noqa: E402
from spacedrive_amd.device import stage_plan  # noqa: E402


def test_parity_fails_on_a_mismatch():
    ok = bench.parity(10, 0, "x", extra=1)
    assert ok == {"files": 10, "mismatches": 0, "oracle": "x", "extra": 1}
    with pytest.raises(AssertionError):
        bench.parity(10, 1, "x")


@pytest.mark.parametrize("n", [1, 10, 33, 5000, 1_250_000])
def test_sample_idx(n):
    idx = bench.sample_idx(n)
    assert idx.dtype == np.int64 and (np.diff(idx) > 0).all()
    assert idx[0] == 0 and idx[-1] == n - 1 and idx.max() < n
    assert set(range(min(32, n))) <= set(idx.tolist())
    assert len(idx) <= min(n, 4096 + 32)


def test_oracle_hashes_are_the_sampled_rows(oracle_native):
    n = 3000
    sizes, cids, twins = synth.library(0, n, 10_000_000)
    idx = bench.sample_idx(n, k=257, head=32)
    got = bench.oracle_hashes(sizes, cids, twins, idx)
    assert got.shape == (len(idx), 32)
    whole = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=4)
    assert np.array_equal(got[:, :8], whole[idx])
    # the library's CPU path over the oracle-staged messages of the whole set
    ext, total = stage_plan(sizes)
    buf = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    out = ctypes.create_string_buffer(17 * n)
    check(lib().sd_cpu_cas_ids(buf.ctypes.data, total + 64, np.ascontiguousarray(ext).ctypes.data, n, out, None, 4))
    raw = out.raw
    assert [raw[17 * i:17 * i + 16].decode() for i in idx] == [r[:8].tobytes().hex() for r in got]


def test_effective_cpus_within_the_affinity_mask_and_quota():
    n = bench.effective_cpus()
    assert bench.all_cores() == len(os.sched_getaffinity(0))
    assert 1 <= n <= bench.all_cores()
    q = bench.host_cpu()["cgroup_cpu_quota"]
    if q:
        assert n <= int(np.ceil(q))


# ------------------------------------------------------------------ --gpus N launcher
def test_launch_mode_rules():
    """--gpus N without WORLD_SIZE starts N ranks; under a launcher the
    rank count must equal --gpus; --gpus 1 stays in-process."""
    assert bench.launch_mode(1, {}) == "inprocess"
    assert bench.launch_mode(2, {}) == "spawn"
    assert bench.launch_mode(8, {}) == "spawn"
    assert bench.launch_mode(8, {"WORLD_SIZE": "8"}) == "rank"
    assert bench.launch_mode(1, {"WORLD_SIZE": "1"}) == "rank"
    for gpus, ws in ((8, "1"), (1, "8"), (2, "4")):
        with pytest.raises(SystemExit) as e:
            bench.launch_mode(gpus, {"WORLD_SIZE": ws})
        assert "WORLD_SIZE" in str(e.value) and f"--gpus {gpus}" in str(e.value)
    with pytest.raises(SystemExit):
        bench.launch_mode(0, {})


def test_launcher_cmd_is_the_drivers_command():
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[-5] == os.path.join(ROOT, "bench.py") and cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def test_bench_refuses_a_world_size_mismatch():
    """The real entry point: WORLD_SIZE=2 with --gpus 8 exits non-zero before any GPU work."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_spawn_relays_rank0_line_and_exit_code(tmp_path):
    """spawn_ranks runs the launcher as a child, relays its JSON line to stdout (other stdout
    to stderr) and returns its exit code; a child that exits 0 without a line is a failure.
    A stand-in launcher prints what rank 0 would."""
    import subprocess
    script = tmp_path / "fake_launcher.py"
    script.write_text("import sys\nprint('banner')\nprint('{\"metric\": \"m\", \"n_gpus\": 2}')\n"
                      "sys.exit(int(sys.argv[1]))\n")
    for rc in (0, 3):
        r = subprocess.run([sys.executable, "-c",
                            "import sys; sys.path.insert(0, %r); import bench\n"
                            "bench.launcher_cmd = lambda g, a, p: [sys.executable, %r, a[0]]\n"
                            "sys.exit(bench.spawn_ranks(2, [%r]))" % (ROOT, str(script), str(rc))],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == rc
        assert r.stdout.strip() == '{"metric": "m", "n_gpus": 2}'
        assert "banner" in r.stderr and "banner" not in r.stdout
    script.write_text("print('no line')\n")
    r = subprocess.run([sys.executable, "-c",
                        "import sys; sys.path.insert(0, %r); import bench\n"
                        "bench.launcher_cmd = lambda g, a, p: [sys.executable, %r]\n"
                        "sys.exit(bench.spawn_ranks(2, []))" % (ROOT, str(script))],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and r.stdout == ""


# ------------------------------------------------------------------ multi-GiB goldens
def test_bench_goldens_cover_every_rank_of_the_default_run():
    g = bench.golden_checksums()
    flen = (64 << 30) // 16
    for r in range(8):
        start = r * 1_250_000
        for i in (0, 15):
            assert f"{10_000 + start + i}:{flen}" in g["synth"]
        m = g["mixed"][f"{start}:{16 * flen}"]
        offs, lens = bench.mixed_layout(start, 16 * flen)
        mi = min(range(len(lens)), key=lambda k: lens[k])
        assert (m["index"], m["offset"], m["len"]) == (mi, offs[mi], lens[mi])
    assert f"20000:{(32 << 30) + 12345}" in g["synth"]


@pytest.mark.parametrize("which", ["configs3", "mixed"])
def test_bench_goldens_equal_the_oracle(oracle_native, which):
    """Re-derives goldens with the oracle: rank 1's configs[3] file 15 (4 GiB), and rank 0's
    shortest mixed file (2.2 GiB spanning two generated files).  The rest were made by the
    same code (make_bench_golden.py); the split file's 32 GiB hash equals round 4's GPU run
    (profiles/r4/r4y_bench.json checksum_one_file.hash)."""
    g = bench.golden_checksums()
    flen = (64 << 30) // 16
    nt = min(8, os.cpu_count() or 1)
    if which == "configs3":
        cid = 10_000 + 1_250_000 + 15
        assert oracle_native.checksum_synth_mt(flen, cid, 0, nthreads=nt).hex() == g["synth"][f"{cid}:{flen}"]
        want, src = bench.synth_checksum_expected(cid, flen, live=False)
        assert src == "golden" and want == g["synth"][f"{cid}:{flen}"]
    else:
        m = g["mixed"][f"0:{16 * flen}"]
        assert bench.mixed_host_checksum(0, m["offset"], m["len"], flen, nt).hex() == m["hash"]


def test_bench_golden_lookup_falls_back_to_the_oracle(oracle_native):
    """A file the goldens do not hold (a non-default size) is hashed by the oracle live."""
    want, src = bench.synth_checksum_expected(10_000, 3 << 20, live=False)
    assert src == "oracle (live)"
    assert want == oracle_native.checksum_synth_mt(3 << 20, 10_000, 0, nthreads=2).hex()


def test_timing_laps_add_up():
    tm = bench.Timing()
    tm.lap("a")
    tm.lap("b")
    tm.lap("a")
    assert set(tm) == {"a", "b"} and all(v >= 0 for v in tm.values())


# ------------------------------------------------------------------ full-output parity
def test_full_parity_digest_and_live(oracle_native, monkeypatch):
    """full_parity checks every cas_id: against the committed digest when it holds the
    workload, else (or to locate a mismatch) against the oracle's cas_ids computed live."""
    import torch
    n = 3000
    sizes, cids, twins = synth.library(0, n, 10 * n)
    ids = oracle_native.cas_ids_synth_simd(sizes, cids, twins, nthreads=4)
    h = np.zeros((n, 32), np.uint8)
    h[:, :8] = ids
    h[:, 8:] = 7  # bytes past the cas_id are not part of it
    d = torch.from_numpy(h.reshape(-1).copy())
    gen = lambda: (sizes, cids, twins)  # noqa: E731
    live = bench.full_parity(d, n, "test:none", gen, live=False)
    assert live["mismatches"] == 0 and live["expected_from"] == "oracle (live)" and not live["digest_mismatch"]
    g = dict(bench.golden_checksums())
    g["cas_digest"] = dict(g.get("cas_digest", {}), **{"test:key": bench.cas_digest(ids)})
    monkeypatch.setattr(bench, "_golden", g)
    ok = bench.full_parity(d, n, "test:key", gen, live=False)
    assert ok["mismatches"] == 0 and ok["expected_from"] == "golden"
    h[1234, 3] ^= 1
    bad = bench.full_parity(torch.from_numpy(h.reshape(-1).copy()), n, "test:key", gen, live=False)
    assert bad["mismatches"] == 1 and bad["first_bad_index"] == 1234 and bad["digest_mismatch"]


def test_library_digests_cover_every_rank_of_1_2_4_8():
    g = bench.golden_checksums()["cas_digest"]
    for world in (1, 2, 4, 8):
        for r in range(world):
            assert bench.library_digest_key(r * 1_250_000, 1_250_000, world * 1_250_000) in g
    assert bench.config_digest_key("small", 1_000_000) in g and bench.config_digest_key("sampled", 1_000_000) in g


def test_library_digest_equals_the_oracle_for_one_shard(oracle_native):
    """Re-derives one committed shard digest (rank 1 of 2) with the oracle."""
    s, c, t = synth.library(1_250_000, 1_250_000, 2_500_000)
    ids = oracle_native.cas_ids_synth_simd(s, c, t, nthreads=min(8, os.cpu_count() or 1))
    assert bench.cas_digest(ids) == bench.golden_checksums()["cas_digest"][
        bench.library_digest_key(1_250_000, 1_250_000, 2_500_000)]


def test_pmc_lookups_cover_the_default_launch_shapes():
    """The committed PMC summary holds the default run's dominant launch shapes: the sampled
    pair of a 1.25 M-file shard and configs[3]'s 16 x 4 GiB leaf launch -- HBM bytes per launch
    (`traffic`) and the per-clock issue rate (`issue_rate_pmc`), the latter at the G mix's
    ceiling within 5 %."""
    from spacedrive_amd import synth
    sizes, _, _ = synth.library(0, 1_250_000, 1_250_000)  # the default shard (--files-per-gpu)
    n_sampled = int((sizes > 102400).sum())
    grids = bench.sampled_grids(n_sampled)
    tr = bench.pmc_traffic_sum(bench.SAMPLED_KERNELS, grids)
    assert tr is not None and 0.99 < tr["bytes"] / (n_sampled * (57352 + 32)) < 1.02
    r = bench.pmc_issue_rate(bench.SAMPLED_KERNELS[0], grids[0])
    assert r is not None and 0.95 < r["frac"] <= 1.02, r
    ck = bench.pmc_issue_rate("k_ck_leaf", bench.ck_leaf_grid(16 * 4096))
    assert ck is not None and 0.95 < ck["frac"] <= 1.02, ck
    assert bench.pmc_issue_rate("k_cas_sampled_lanes", 12345) is None
