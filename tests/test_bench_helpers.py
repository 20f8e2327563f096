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
