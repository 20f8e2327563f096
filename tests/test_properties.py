"""Property tests (hypothesis, CPU only) of the library's host code against the oracle:
random inputs drawn around the BLAKE3 block (64 B), chunk (1 KiB), cas-threshold
(102 400 B) and leaf-block (1 MiB) boundaries.

* the CPU hash of any byte string equals the C oracle's (blake3 crate 1.4.1 restated);
* the output does not depend on how the input is split across ranks (sd_cpu_split_*: the
  leaves of any rank count merge into the one-piece checksum, BLAKE3's update-split
  independence);
* the stage plan lays out every message as cas.rs:25-58 builds it (8-byte header, whole
  content up to 102 400 B, 57 352 B otherwise), 16-B aligned, non-overlapping, in order;
* cas_ids over a staged batch of random sizes equal the oracle's, file by file;
* the shard plan covers [0, n) with contiguous, ordered, cost-balanced ranges."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import cas_spec as cs
from spacedrive_amd import cpu, split
from spacedrive_amd.dedup import shard_plan
from spacedrive_amd.device import stage_plan

KIB, MIB = 1024, 1 << 20
SETTINGS = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def near(points, spread=2):
    """lengths at and just around each boundary point"""
    return st.sampled_from(points).flatmap(lambda p: st.integers(max(0, p - spread), p + spread))


LENGTHS = st.one_of(
    st.integers(0, 4 * KIB),
    near([64, 1024, 2048, 16 * KIB, 57352, 102400, 102408, MIB, 2 * MIB, 3 * MIB]),
    st.integers(0, 3 * MIB + 5000),
)


def rand_bytes(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@SETTINGS
@given(n=LENGTHS, seed=st.integers(0, 2**32 - 1))
def test_cpu_blake3_equals_oracle(oracle_native, n, seed):
    d = rand_bytes(seed, n)
    assert cpu.blake3(d) == oracle_native.blake3(d)


@SETTINGS
@given(n=st.one_of(near([MIB, 2 * MIB, 3 * MIB, 5 * MIB], 3), st.integers(0, 6 * MIB)),
       ranks=st.integers(1, 7), seed=st.integers(0, 2**32 - 1))
def test_split_leaves_merge_to_the_checksum(oracle_native, n, ranks, seed):
    data = np.zeros(n + 64, np.uint8)
    data[:n] = np.frombuffer(rand_bytes(seed, n), np.uint8)
    cvs, end = None, 0
    for r in range(ranks):
        off, ln, cv_bytes = split.split_range(n, ranks, r)
        assert off == end  # contiguous, in rank order
        end = off + ln
        mine = split.cpu_leaves(data[off:off + ln], n, ranks, r, nthreads=2)
        q = cv_bytes // (32 * ranks)
        if cvs is None:
            cvs = np.zeros(cv_bytes, np.uint8)
        cvs[r * q * 32:(r + 1) * q * 32] = mine[r * q * 32:(r + 1) * q * 32]
    assert end == n
    assert split.cpu_root(cvs, n) == oracle_native.blake3(data[:n].tobytes())


SIZES = st.lists(st.one_of(st.integers(0, 3 * KIB), near([1016, 1017, 102400, 102401]),
                           st.integers(102401, 1 << 40)), min_size=1, max_size=40)


@SETTINGS
@given(sizes=SIZES)
def test_stage_plan_layout_matches_cas_rs(sizes):
    sz = np.array(sizes, np.uint64)
    ext, total = stage_plan(sz)
    end = 0
    for s, e in zip(sizes, ext):
        want_len = 8 + s if s <= cs.MINIMUM_FILE_SIZE else 57352
        assert int(e["msg_len"]) == want_len
        assert int(e["size"]) == s
        off = int(e["msg_offset"])
        assert off % 16 == 0 and off >= end
        end = off + want_len
    assert total >= end


@SETTINGS
@given(sizes=st.lists(st.one_of(st.integers(1, 3 * KIB), near([102400, 102401]),
                                st.integers(102401, 1 << 34)), min_size=1, max_size=24),
       seed=st.integers(0, 2**31))
def test_cpu_cas_ids_staged_equal_oracle(oracle_native, sizes, seed):
    sz = np.array(sizes, np.uint64)
    cids = np.arange(seed, seed + len(sizes), dtype=np.uint64)
    twins = np.zeros(len(sizes), np.uint32)
    ext, total = stage_plan(sz)
    buf = oracle_native.stage_synth(sz, cids, twins, ext["msg_offset"], total)
    want = [bytes(r).hex() for r in oracle_native.cas_ids_synth(sz, cids, twins)]
    assert cpu.cas_ids_staged(buf, ext) == want


def msg_compressions(size):
    """compressions of a file's cas message (SURVEY.md §8(d) algorithmic units)"""
    m = 8 + size if size <= cs.MINIMUM_FILE_SIZE else 57352
    chunks = max(1, -(-m // 1024))
    blocks = sum(max(1, -(-min(1024, m - 1024 * c) // 64)) for c in range(chunks))
    return blocks + chunks - 1


@SETTINGS
@given(sizes=st.lists(st.one_of(st.integers(0, 102400), st.integers(102401, 1 << 33)), min_size=0, max_size=300),
       ranks=st.integers(1, 9))
def test_shard_plan_is_a_balanced_ordered_cover(sizes, ranks):
    bounds = [int(b) for b in shard_plan(np.array(sizes, np.uint64), ranks)]
    assert bounds[0] == 0 and bounds[-1] == len(sizes)
    assert all(a <= b for a, b in zip(bounds, bounds[1:]))
    cost = [msg_compressions(s) for s in sizes]
    total, worst = sum(cost), max(cost, default=0)
    for r in range(ranks):  # each rank within one file of its even share
        assert sum(cost[bounds[r]:bounds[r + 1]]) <= total / ranks + worst + 1


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
