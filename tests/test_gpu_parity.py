"""Parity of the HIP path (through the C ABI) with the oracle -- run on an MI355X: -m gpu.

Bit-exact on every byte: the full 32-byte BLAKE3 of every staged message, the 16-hex
cas_id, the 64-hex checksum, and the dedup grouping.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cas_spec as cs  # noqa: E402
from spacedrive_amd import synth  # noqa: E402
from spacedrive_amd.dedup import group_host, keys_from_hashes, partition_host  # noqa: E402

NT = 16  # oracle threads: the GPU box's host share per GPU


@pytest.fixture(scope="module")
def ctx():
    import spacedrive_amd
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    c = spacedrive_amd.default_context(0)
    # the product library must be the in-tree HIP build
    maps = open("/proc/self/maps").read()
    assert "spacedrive_amd/libsdcas.so" in maps
    return c


@pytest.fixture(scope="module", autouse=True)
def _gpu_route_for_batches():
    """sd_cas_ids_files hashes calls of up to "batch_cpu_max" files on the CPU path, and
    sd_file_checksums calls of up to "checksum_cpu_max" (by default all), and the learned
    routes ("checksum_split_adapt") may send large calls to the CPU path; the parity tests
    below exercise the GPU routes, so the module turns these policies off (the policies have
    their own tests) and restores the library defaults after."""
    import spacedrive_amd as sd
    keep = {k: sd.get_tuning(k) for k in ("batch_cpu_max", "checksum_cpu_max", "checksum_split_adapt")}
    sd.set_tuning("batch_cpu_max", 0)
    sd.set_tuning("checksum_cpu_max", 0)  # sd_file_checksums: its GPU route (the default is the CPU path)
    # sd_checksums' co-hashed calls and sd_file_checksums' split always take the GPU side
    # (the learned routes have their own tests)
    sd.set_tuning("checksum_split_adapt", 0)
    yield
    for k, v in keep.items():
        sd.set_tuning(k, v)


@pytest.fixture(scope="module", autouse=True)
def _rccl_background(ctx):
    """The one single-rank RCCL communicator (sd_comm_create) the RCCL tests share, created
    on a background thread as the module starts: RCCL's initialisation takes seconds, its
    collectives microseconds, and the other tests need not wait for it."""
    import threading
    from spacedrive_amd import dedup
    box = {}

    def make():
        try:
            box["comm"] = dedup.make_comm(ctx)
        except BaseException as e:  # noqa: BLE001 -- re-raised in the tests that need it
            box["err"] = e

    t = threading.Thread(target=make, daemon=True)
    t.start()
    yield t, box
    t.join()
    if "comm" in box:
        box["comm"].close()


@pytest.fixture
def rccl_comm(_rccl_background):
    t, box = _rccl_background
    t.join()
    if "err" in box:
        raise box["err"]
    return box["comm"]


def stage_synth(ctx, sizes, cids, twins):
    from spacedrive_amd.device import stage_plan
    n = len(sizes)
    ext, total = stage_plan(sizes)
    d_staged = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    d_ext = torch.from_numpy(ext.view(np.uint8).copy()).cuda()
    ctx.synth_stage_cas(torch.from_numpy(sizes.astype(np.uint64).view(np.int64)).cuda(),
                        torch.from_numpy(cids.astype(np.uint64).view(np.int64)).cuda(),
                        torch.from_numpy(twins.astype(np.int32)).cuda(), d_ext, n, d_staged)
    return ext, total, d_staged


def gpu_cas(ctx, sizes, cids, twins, return_staged=False):
    ext, total, d_staged = stage_synth(ctx, sizes, cids, twins)
    b = ctx.cas_batch(ext)
    out = torch.zeros(max(len(sizes), 1) * 32, dtype=torch.uint8, device="cuda")
    b.run(d_staged, out)
    torch.cuda.synchronize()
    h = out.cpu().numpy()[:len(sizes) * 32].reshape(-1, 32)
    if return_staged:
        return h, ext, d_staged.cpu().numpy()
    return h


def test_synth_stage_matches_oracle_messages(ctx, oracle_native):
    sizes = np.array([0, 1, 7, 8, 9, 1015, 1016, 1017, 102400, 102401, 555555, (1 << 32) + 1], np.uint64)
    cids = np.arange(100, 100 + len(sizes), dtype=np.uint64)
    twins = np.zeros(len(sizes), np.uint32)
    twins[-2] = 9
    _, ext, staged = gpu_cas(ctx, sizes, cids, twins, return_staged=True)
    for i in range(len(sizes)):
        o, L = int(ext["msg_offset"][i]), int(ext["msg_len"][i])
        want = oracle_native.cas_message(int(cids[i]), int(twins[i]), int(sizes[i]))
        assert staged[o:o + L].tobytes() == want, i
        pad = (o + L + 63) // 64 * 64
        assert not staged[o + L:pad].any()


def test_cas_goldens(ctx, golden):
    files = golden["cas_synth"]["files"]
    sizes = np.array([f["size"] for f in files], np.uint64)
    cids = np.array([f["content_id"] for f in files], np.uint64)
    twins = np.array([f["twin"] for f in files], np.uint32)
    h = gpu_cas(ctx, sizes, cids, twins)
    for f, row in zip(files, h):
        assert row[:8].tobytes().hex() == f["cas_id"], f


def test_cas_pattern_goldens_host_staged(ctx, golden):
    # host-staged pattern content through the drop-in sd_cas_ids entry point
    import ctypes
    from spacedrive_amd._native import check, lib
    from spacedrive_amd.device import stage_plan
    cp = golden["cas_pattern"]["cas_id"]
    sizes = np.array([int(s) for s in cp], np.uint64)
    ext, total = stage_plan(sizes)
    staged = np.zeros(total, np.uint8)
    reader = lambda o, n: bytes((o + k) % 251 for k in range(n))  # noqa: E731
    for i, s in enumerate(sizes):
        msg = cs.cas_message(reader, int(s))
        o = int(ext["msg_offset"][i])
        staged[o:o + len(msg)] = np.frombuffer(msg, np.uint8)
    out = ctypes.create_string_buffer(17 * len(sizes))
    check(lib().sd_cas_ids(ctx.handle, staged.ctypes.data, total, ext.ctypes.data, len(sizes), out, None))
    raw = out.raw  # one copy of the buffer
    for i, s in enumerate(cp):
        assert raw[17 * i:17 * i + 16].decode() == cp[s], s


@pytest.mark.parametrize("cohash", [0, 15])
def test_sd_cas_ids_pipelined_windows(ctx, cohash):
    # the drop-in host entry point over several 512 MiB windows (two alternating streams),
    # with entries pre-marked failed that must be skipped and left untouched -- the GPU
    # alone, and with 15 host threads hashing from the end of the list beside it
    # ("host_cohash_threads"): both sides must have hashed files, every result equal
    import ctypes
    import spacedrive_amd as sd
    from spacedrive_amd._native import check, lib
    n = 40000
    sizes, cids, twins = synth.library(0, n, n, small_frac=0.3)
    h, ext, staged = gpu_cas(ctx, sizes, cids, twins, return_staged=True)
    assert ext["msg_offset"][-1] > (1 << 30)  # more than two windows
    host = torch.from_numpy(staged).pin_memory()
    status = np.zeros(n, np.int32)
    status[::1001] = 2  # staging failed upstream
    out = ctypes.create_string_buffer(b"#" * (17 * n), 17 * n)
    keep = sd.get_tuning("host_cohash_threads")
    before = np.zeros(2, np.uint64)
    after = np.zeros(2, np.uint64)
    check(lib().sd_cas_ids_stats(ctx.handle, before.ctypes.data))
    sd.set_tuning("host_cohash_threads", cohash)
    try:
        check(lib().sd_cas_ids(ctx.handle, host.data_ptr(), len(staged), ext.ctypes.data, n, out,
                               status.ctypes.data))
    finally:
        sd.set_tuning("host_cohash_threads", keep)
    check(lib().sd_cas_ids_stats(ctx.handle, after.ctypes.data))
    gpu_files, host_files = (int(x) for x in after - before)
    assert gpu_files + host_files == n - len(range(0, n, 1001))
    assert (host_files > 0 and gpu_files > 0) if cohash else host_files == 0
    raw = out.raw
    for i in range(n):
        if i % 1001 == 0:
            assert status[i] == 2 and raw[17 * i:17 * i + 16] == b"#" * 16
        else:
            assert status[i] == 0 and raw[17 * i:17 * i + 16].decode() == h[i, :8].tobytes().hex(), i


@pytest.mark.parametrize("mode", ["latency", "throughput"])
def test_cas_latency_and_throughput_kernels(ctx, oracle_native, mode):
    # the same batch through the latency kernels (k_cas_sampled_wave, k_whole_wave: one
    # wave / workgroup per file) and the throughput kernels (lanes + merge, work lists),
    # forced by the "sampled_wave_max" / "whole_wave_max" thresholds: full 32-byte hashes
    # of every message length 0..2100, around the whole-file limit, and sampled files
    from spacedrive_amd._native import lib
    big = 1 << 30
    thr = big if mode == "latency" else 0
    assert lib().sd_cas_set_tuning(b"sampled_wave_max", thr) == 0
    assert lib().sd_cas_set_tuning(b"whole_wave_max", thr) == 0
    try:
        sizes = np.concatenate([np.arange(0, 2100), np.arange(102300, 102401),
                                np.arange(102401, 102401 + 300 * 4099, 4099)]).astype(np.uint64)
        np.random.default_rng(9).shuffle(sizes)
        cids = np.arange(len(sizes), dtype=np.uint64) + 31
        twins = np.zeros(len(sizes), np.uint32)
        h, ext, staged = gpu_cas(ctx, sizes, cids, twins, return_staged=True)
        full = oracle_native.checksums(staged, ext["msg_offset"], ext["msg_len"].astype(np.uint64), nthreads=NT)
        mism = np.nonzero((h != full).any(axis=1))[0]
        assert len(mism) == 0, [(int(sizes[i])) for i in mism[:10]]
    finally:
        lib().sd_cas_set_tuning(b"sampled_wave_max", 6144)  # the defaults
        lib().sd_cas_set_tuning(b"whole_wave_max", 512)


def test_cas_exhaustive_small_sizes(ctx, oracle_native):
    # every message length across the first three chunks and the whole-file threshold
    sizes = np.concatenate([np.arange(0, 3200), np.arange(101000, 102500), np.arange(20000, 22000, 7)]).astype(np.uint64)
    np.random.default_rng(5).shuffle(sizes)  # work-list planning must not depend on input order
    cids = np.arange(len(sizes), dtype=np.uint64) + 7
    twins = np.zeros(len(sizes), np.uint32)
    h, ext, staged = gpu_cas(ctx, sizes, cids, twins, return_staged=True)
    full = oracle_native.checksums(staged, ext["msg_offset"], ext["msg_len"].astype(np.uint64), nthreads=NT)
    mism = np.nonzero((h != full).any(axis=1))[0]
    assert len(mism) == 0, [(int(sizes[i])) for i in mism[:10]]


def test_cas_mixture_full_hash_vs_oracle(ctx, oracle_native):
    # configs[0]-style mixture incl. dups, twins and every edge size; full 32-byte hashes
    n = 30000
    sizes, cids, twins = synth.library(0, n, n)
    h, ext, staged = gpu_cas(ctx, sizes, cids, twins, return_staged=True)
    full = oracle_native.checksums(staged, ext["msg_offset"], ext["msg_len"].astype(np.uint64), nthreads=NT)
    assert np.array_equal(h, full)
    # and the message bytes are the reference's (oracle builds them from the generator)
    ids = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=NT)
    assert np.array_equal(h[:, :8], ids)


def test_cas_configs0_full_size_and_idempotent(ctx, oracle_native):
    # configs[0]: 100k mixed files -- full size, bit-exact vs the oracle, twice
    n = 100_000
    sizes, cids, twins = synth.library(0, n, n)
    h1 = gpu_cas(ctx, sizes, cids, twins)
    h2 = gpu_cas(ctx, sizes, cids, twins)
    assert np.array_equal(h1, h2)
    ids = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=NT)
    assert np.array_equal(h1[:, :8], ids)


def _cas_digest(h):
    """SHA-256 of n cas_ids in file order (bench.py cas_digest: equal to the oracle's digest
    only if every one of the n cas_ids is)"""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(h[:, :8]).tobytes()).hexdigest()


@pytest.mark.parametrize("key", ["configs:small:1000000", "configs:sampled:1000000", "library:0:1250000:1250000"])
def test_cas_baseline_sizes_vs_committed_oracle_digest(ctx, golden, key):
    """BASELINE.json's full sizes, bit-exact, independent of bench.py's line (VERDICT r5 item
    3): configs[1] (1 M whole-content files), configs[2] (1 M sampled files, 57 GB of staged
    messages) and the headline 1.25 M-file mixture shard, staged on the device by
    sd_synth_stage_cas and hashed through sd_cas_batch_run; the SHA-256 of all cas_ids
    against the C oracle's, committed in tests/golden/bench_checksums.json
    (make_bench_golden.py)."""
    kind, *rest = key.split(":")
    if kind == "configs":
        n = int(rest[1])
        gen = synth.small_library if rest[0] == "small" else synth.sampled_library
        sizes, cids, twins = gen(0, n)
    else:
        start, n, n_total = (int(x) for x in rest)
        sizes, cids, twins = synth.library(start, n, n_total)
    h = gpu_cas(ctx, sizes, cids, twins)
    torch.cuda.empty_cache()
    assert h.shape == (n, 32)
    assert _cas_digest(h) == golden["bench_checksums"]["cas_digest"][key]


def test_checksum_configs3_batch_vs_committed_oracle(ctx, golden):
    """configs[3] at its full size: 16 files x 4 GiB (64 GiB) in one sd_checksum_batch_run
    launch set, as bench.py hashes them; files 0 and 15 against the C oracle's committed
    checksums, and the whole batch twice (deterministic)."""
    nf, flen = 16, 4 << 30
    d = torch.empty(nf * flen + 128, dtype=torch.uint8, device="cuda")
    offs = [i * flen for i in range(nf)]
    for i in range(nf):
        ctx.synth_fill(10_000 + i, 0, flen, d[offs[i]:])
    b = ctx.checksum_batch(offs, [flen] * nf)
    s1 = torch.zeros(nf * 32, dtype=torch.uint8, device="cuda")
    s2 = torch.zeros_like(s1)
    b.run(d, s1)
    b.run(d, s2)
    torch.cuda.synchronize()
    del d
    torch.cuda.empty_cache()
    assert torch.equal(s1, s2)
    sums = s1.cpu().numpy().reshape(nf, 32)
    want = golden["bench_checksums"]["synth"]
    for i in (0, nf - 1):
        assert sums[i].tobytes().hex() == want[f"{10_000 + i}:{flen}"], i
    assert len({r.tobytes() for r in sums}) == nf  # 16 different contents


@pytest.mark.parametrize("wave_max", [0, 6144])
def test_cas_sampled_batch_shapes(ctx, oracle_native, wave_max):
    # throughput path (sampled_wave_max 0): k_cas_sampled_lanes, 7 lanes per file in 256-lane
    # workgroups (files straddle them), and k_cas_sampled_merge, one lane per file; latency
    # path (the default threshold): one wave per file -- partial last workgroups bit-exact
    from spacedrive_amd._native import lib
    assert lib().sd_cas_set_tuning(b"sampled_wave_max", wave_max) == 0
    try:
        for n in (1, 7, 15, 16, 17, 31, 32, 33, 36, 37, 65, 255, 256, 257, 1000):
            sizes = np.full(n, 200001, np.uint64) + np.arange(n, dtype=np.uint64) * 4099
            cids = np.arange(n, dtype=np.uint64) + 22
            h = gpu_cas(ctx, sizes, cids, np.zeros(n, np.uint32))
            assert np.array_equal(h[:, :8], oracle_native.cas_ids_synth(sizes, cids, nthreads=NT)), n
    finally:
        lib().sd_cas_set_tuning(b"sampled_wave_max", 6144)


def test_cas_huge_sampled_sizes(ctx, oracle_native):
    """Sampled files far past 4 GiB, up to u64's maximum size: the device stager's sample
    offsets (8192 + k * ((size - 16384) / 4), cas.rs:41-51), its footer at size - 8192 and the
    le64 header in 64-bit arithmetic, then the sampled kernels -- bit-exact with the C
    oracle, which tests/test_oracle.py pins to the Python spec at the same sizes."""
    from tests.test_oracle import HUGE_SAMPLED
    sizes = np.array(HUGE_SAMPLED * 40, np.uint64)  # 280 files: the throughput kernels' batch shape too
    cids = np.arange(700, 700 + len(sizes), dtype=np.uint64) % np.uint64(len(HUGE_SAMPLED)) + np.uint64(700)
    twins = np.zeros(len(sizes), np.uint32)
    h = gpu_cas(ctx, sizes, cids, twins)
    want = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=NT)
    assert np.array_equal(h[:, :8], want)


def test_sample_twins_and_duplicates(ctx):
    sizes = np.array([5 << 20, 5 << 20, 5 << 20, 3000, 3000], np.uint64)
    cids = np.array([1, 1, 1, 2, 2], np.uint64)
    twins = np.array([0, 0, 4, 0, 0], np.uint32)
    h = gpu_cas(ctx, sizes, cids, twins)
    assert h[0, :8].tobytes() == h[1, :8].tobytes() == h[2, :8].tobytes()  # twin: same cas_id
    assert h[3].tobytes() == h[4].tobytes()


# ------------------------------------------------------------------------ checksums
def gpu_checksums(ctx, lens, cids, twins):
    offs, off = [], 0
    for L in lens:
        offs.append(off)
        off = (off + int(L) + 64 + 63) // 64 * 64
    d = torch.zeros(off + 64, dtype=torch.uint8, device="cuda")
    for L, o, c, t in zip(lens, offs, cids, twins):
        if L:
            ctx.synth_fill(int(c), int(t), int(L), d[o:])
    b = ctx.checksum_batch(offs, lens)
    out = torch.zeros(max(len(lens), 1) * 32, dtype=torch.uint8, device="cuda")
    b.run(d, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()[:len(lens) * 32].reshape(-1, 32)


def test_checksum_goldens(ctx, golden):
    files = golden["checksum_synth"]["files"]
    lens = [f["size"] for f in files]
    h = gpu_checksums(ctx, lens, [f["content_id"] for f in files], [f["twin"] for f in files])
    for f, row in zip(files, h):
        assert row.tobytes().hex() == f["checksum"], f


def test_checksum_sizes_vs_oracle(ctx, oracle_native):
    MiB = 1 << 20
    lens = [0, 1, 1024, 1025, 4096, 4097, 5 * 1024, MiB - 1, MiB, MiB + 1, 4 * MiB + 3, 7 * MiB,
            256 * MiB, 256 * MiB + 1, 300 * MiB + 17, 3 * 1024 + 1, 1020 * 1024 + 5]
    cids = list(range(500, 500 + len(lens)))
    twins = [i % 3 for i in range(len(lens))]
    h = gpu_checksums(ctx, lens, cids, twins)
    want = oracle_native.checksums_synth(np.array(lens, np.uint64), np.array(cids, np.uint64),
                                         np.array(twins, np.uint32), nthreads=NT)
    bad = [lens[i] for i in range(len(lens)) if h[i].tobytes() != want[i].tobytes()]
    assert not bad, bad


def test_checksum_multi_gib_vs_oracle(ctx, oracle_native):
    """configs[3] sizes: a 4 GiB file exactly as bench.py hashes it (content id 10000),
    the SURVEY.md 8(d) edge size 2^32 + 1, and an odd 5 GiB + 12345 twin -- byte offsets
    past 2^32 and multi-level reduce passes -- against the chunk-parallel C oracle."""
    lens = [4 << 30, (1 << 32) + 1, (5 << 30) + 12345]
    cids, twins = [10_000, 77, 78], [0, 0, 9]
    h = gpu_checksums(ctx, lens, cids, twins)
    torch.cuda.empty_cache()
    for i, L in enumerate(lens):
        want = oracle_native.checksum_synth_mt(L, cids[i], twins[i], nthreads=NT)
        assert h[i].tobytes() == want, L


def test_file_api_on_disk(ctx, tmp_path, golden):
    import spacedrive_amd as sd
    sizes = [0, 1, 1017, 102400, 102401, 2 << 20, 300 * (1 << 20) + 5]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"f{i}.bin"
        with open(p, "wb") as f:
            pos = 0
            while pos < s:
                n = min(64 << 20, s - pos)
                f.write(cs.synth_bytes(60 + i, 0, pos, n))
                pos += n
        paths.append(str(p))
    ids = sd.generate_cas_ids(paths, sizes)
    for i, s in enumerate(sizes):
        assert ids[i] == cs.generate_cas_id(cs.synth_reader(60 + i), s), s
    sums = sd.file_checksums(paths)
    from oracle import native
    want = native.checksums_synth(np.array(sizes, np.uint64), np.arange(60, 60 + len(sizes), dtype=np.uint64),
                                  nthreads=NT)
    for i in range(len(sizes)):
        assert sums[i] == want[i].tobytes().hex(), sizes[i]
    assert sd.file_checksum(paths[2]) == sums[2]
    assert sd.generate_cas_id(paths[4], sizes[4]) == ids[4]
    # FileMetadata: empty file -> cas_id None (file_identifier/mod.rs:80-88)
    md = sd.FileMetadata.batch(paths[:3])
    assert md[0].cas_id is None and md[1].cas_id == ids[1]
    # a missing file; a file shorter than its planned size whose samples still fit (the
    # tail comes from the real end, cas.rs:54: the reference returns an id); one whose
    # last sample runs past EOF (read_exact's UnexpectedEof)
    r = sd.generate_cas_ids([str(tmp_path / "missing"), paths[5], paths[5]], [10, (2 << 20) + 100, 3 << 20])
    assert isinstance(r[0], FileNotFoundError) or (isinstance(r[0], OSError) and r[0].errno == 2)
    content = open(paths[5], "rb").read()
    assert r[1] == cs.generate_cas_id_file(content, (2 << 20) + 100)
    assert isinstance(r[2], sd.UnexpectedEofError)
    with pytest.raises(OSError):
        sd.file_checksum(str(tmp_path / "missing"))


# ---------------------------------------------------------------------------- dedup
@pytest.fixture(params=[0, 1])
def dedup_variant(request):
    """sd_dedup_group: 0 = rocPRIM radix sort, 1 = LDS buckets (the default)."""
    from spacedrive_amd._native import lib
    assert lib().sd_cas_set_tuning(b"dedup_variant", request.param) == 0
    yield request.param
    lib().sd_cas_set_tuning(b"dedup_variant", 1)  # the default


def _group_check(ctx, recs: np.ndarray, index_sorted: bool = False):
    gr, grep, gng = group_host(recs)
    sub = torch.from_numpy(recs.copy()).cuda()
    rep = torch.zeros(max(len(recs), 1), dtype=torch.int64, device="cuda")
    ng = ctx.dedup_group(sub, len(recs), rep, index_sorted=index_sorted)
    assert ng == gng
    assert np.array_equal(sub.cpu().numpy(), gr)
    assert np.array_equal(rep.cpu().numpy()[:len(recs)], grep)


def test_dedup_group_edge_sizes(ctx, dedup_variant):
    rng = np.random.default_rng(7)
    for m in (0, 1, 2, 3, 47, 48, 49, 97, 1000, 4099):
        keys = rng.integers(0, 2**63, m, dtype=np.int64) * 2 + rng.integers(0, 2, m)  # full 64-bit range
        if m > 4:
            keys[m // 2:m // 2 + 3] = keys[0]  # a group of 4
        recs = np.stack([keys, rng.permutation(m).astype(np.int64) * 3 + 5], axis=1)
        _group_check(ctx, recs)
    # all keys equal (span 0), and a narrow key range (one cas_id prefix bucket of a rank)
    _group_check(ctx, np.stack([np.full(300, 12345, np.int64), np.arange(300, dtype=np.int64)[::-1].copy()], axis=1))
    narrow = (np.int64(0x1234) << np.int64(48)) + rng.integers(0, 2**40, 20000, dtype=np.int64)
    _group_check(ctx, np.stack([narrow, np.arange(20000, dtype=np.int64)], axis=1), index_sorted=True)


def test_dedup_group_large_groups(ctx, dedup_variant):
    """Duplicate groups larger than a wave's LDS bucket (512): 3000 files and 40 groups of
    600..1500 go to the workgroup sort (k_gb_sort_big); 5000 exceed it (radix fallback)."""
    rng = np.random.default_rng(8)
    m = 200000
    keys = rng.integers(-2**63, 2**63 - 1, m, dtype=np.int64)
    perm = rng.permutation(m)
    keys[perm[:3000]] = keys[perm[0]]
    at = 3000
    for g in range(40):
        sz = 600 + 23 * g
        keys[perm[at:at + sz]] = keys[perm[at]]
        at += sz
    recs = np.stack([keys, np.arange(m, dtype=np.int64)], axis=1)
    _group_check(ctx, recs, index_sorted=True)
    _group_check(ctx, recs[::-1].copy())
    keys[perm[at:at + 5000]] = keys[perm[at]]
    recs = np.stack([keys, np.arange(m, dtype=np.int64)], axis=1)
    _group_check(ctx, recs, index_sorted=True)
    _group_check(ctx, recs[::-1].copy())


def test_dedup_group_matches_host(ctx, dedup_variant):
    n = 50000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    h = gpu_cas(ctx, sizes, cids, twins)
    d_hash = torch.from_numpy(h.copy()).cuda()
    valid = (sizes != 0).astype(np.uint8)
    d_valid = torch.from_numpy(valid).cuda()
    keys = keys_from_hashes(h)
    idx = np.arange(n, dtype=np.int64)
    for nparts in (1, 2, 8):
        counts = torch.zeros(nparts, dtype=torch.int64, device="cuda")
        recs = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
        nv = ctx.dedup_partition(d_hash, d_valid, n, 0, nparts, counts, recs)
        assert nv == int(valid.sum())
        hrecs, hcounts = partition_host(keys[valid == 1], idx[valid == 1], nparts)
        assert counts.cpu().numpy().tolist() == hcounts.tolist()
        r = recs[:nv].cpu().numpy()
        assert np.array_equal(r, hrecs)  # stable: by destination, input order within one
        start = 0
        for d in range(nparts):
            seg = r[start:start + hcounts[d]]
            start += hcounts[d]
            gr, grep, gng = group_host(seg)
            for sorted_flag, src in ((True, seg), (False, seg[::-1].copy())):  # fast path; general path
                sub = torch.from_numpy(src.copy()).cuda()
                rep = torch.zeros(max(len(seg), 1), dtype=torch.int64, device="cuda")
                ng = ctx.dedup_group(sub, len(seg), rep, index_sorted=sorted_flag)
                assert ng == gng
                assert np.array_equal(sub.cpu().numpy(), gr)
                assert np.array_equal(rep.cpu().numpy()[:len(seg)], grep)


def test_valu_peak_plausible(ctx):
    v = ctx.valu_peak()
    assert 5e12 < v < 2e14, v


def test_file_checksums_packing_and_streaming(ctx, tmp_path):
    # many small files packed per window, files larger than half the 256 MiB window streamed
    # between them (their hashes arrive asynchronously, at later syncs of their slot), an
    # unreadable path in the middle: results in input order
    import spacedrive_amd as sd
    from oracle import native
    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(0, 3 << 20, 150)]
    sizes[40] = (300 << 20) + 7
    sizes[41] = 256 << 20  # exactly one window + nothing: packed? no -> streamed (len + 128 > W)
    sizes[42] = 0
    sizes[43] = (129 << 20) + 1  # a third streamed file in a row: the two message plans alternate
    sizes[100] = 128 << 20  # streamed between packs
    paths = []
    for i, sz in enumerate(sizes):
        p = tmp_path / f"c{i}"
        with open(p, "wb") as f:
            pos = 0
            while pos < sz:
                k = min(64 << 20, sz - pos)
                f.write(cs.synth_bytes(3000 + i, 0, pos, k))
                pos += k
        paths.append(str(p))
    paths.insert(77, str(tmp_path / "nope"))
    got = sd.file_checksums(paths)
    assert isinstance(got[77], OSError)
    del got[77]
    big = [i for i, sz in enumerate(sizes) if sz > (64 << 20)]  # chunk-parallel checker for these
    small = [i for i in range(len(sizes)) if i not in big]
    want = {}
    w = native.checksums_synth(np.array([sizes[i] for i in small], np.uint64), np.array([3000 + i for i in small],
                                                                                       np.uint64), nthreads=NT)
    for j, i in enumerate(small):
        want[i] = w[j].tobytes().hex()
    for i in big:
        want[i] = native.checksum_synth_mt(sizes[i], 3000 + i, 0, nthreads=NT).hex()
    for i in range(len(sizes)):
        assert got[i] == want[i], (i, sizes[i])


@pytest.mark.parametrize("mode,budget", [("blocks", 0), ("blocks", 3), ("files", 0)])
def test_file_checksums_hybrid_split(ctx, tmp_path, mode, budget):
    """sd_file_checksums' split policy ("checksum_hybrid_threads", default 6): a call whose regular
    files of >= 8 MiB total >= 512 MiB runs the GPU route and the CPU path at once -- by
    blocks (round 5's default: the GPU's slots take runs of 1 MiB blocks while free, the host
    threads single blocks, roots merged from both sides' CVs) or by whole files (round 4,
    "checksum_split_blocks" 0) -- the small ones and a FIFO to the CPU path.  Every result
    equals the oracle's read schedule (hash.rs:10-24), an unreadable path keeps its error,
    the call is counted as split and both sides hashed bytes, also under a 3-thread host
    budget; below the threshold the CPU path alone runs."""
    import threading
    import spacedrive_amd as sd
    from oracle import native
    MiB = 1 << 20
    sizes = [40 * MiB + 3, 8 * MiB, 3000, 0, 96 * MiB + 1, 64 * MiB, 12345, 130 * MiB + 77, 16 * MiB - 1,
             72 * MiB, 5 * MiB, 100 * MiB + 5, 33 * MiB]
    paths = []
    for i, sz in enumerate(sizes):
        p = tmp_path / f"h{i}"
        with open(p, "wb") as f:
            pos = 0
            while pos < sz:
                k = min(32 << 20, sz - pos)
                f.write(cs.synth_bytes(5000 + i, 0, pos, k))
                pos += k
        paths.append(str(p))
    fifo = str(tmp_path / "fifo")
    os.mkfifo(fifo)
    fifo_data = cs.synth_bytes(6000, 0, 0, 4000)  # one write: hash.rs's first read returns it

    def feed():
        with open(fifo, "wb", buffering=0) as f:
            f.write(fifo_data)
    paths.insert(5, fifo)
    paths.insert(9, str(tmp_path / "missing"))
    want_h, want_st = native.file_checksums([p for p in paths if p != fifo], nthreads=NT)
    want = dict(zip([p for p in paths if p != fifo], zip(want_h, want_st)))
    from spacedrive_amd._native import check, lib
    keep = {k: sd.get_tuning(k) for k in ("checksum_cpu_max", "checksum_hybrid_threads", "checksum_split_blocks",
                                          "host_cpu_budget", "checksum_split_adapt")}
    sd.set_tuning("checksum_cpu_max", 2147483647)  # the library default (the module sets 0)
    sd.set_tuning("checksum_split_adapt", 0)  # always the split (the learned route has its own test)
    sd.set_tuning("checksum_hybrid_threads", 6)  # the library default
    sd.set_tuning("checksum_split_blocks", 1 if mode == "blocks" else 0)
    sd.set_tuning("host_cpu_budget", budget)
    by0 = np.zeros(2, np.uint64)
    check(lib().sd_file_checksums_bytes(sd.default_context().handle, by0.ctypes.data))
    try:
        before = sd.file_checksums_stats()
        t = threading.Thread(target=feed)
        t.start()
        got = sd.file_checksums(paths)
        t.join()
        after = sd.file_checksums_stats()
        assert after["hybrid"] == before["hybrid"] + 1 and after["cpu"] == before["cpu"]
        by1 = np.zeros(2, np.uint64)
        check(lib().sd_file_checksums_bytes(sd.default_context().handle, by1.ctypes.data))
        assert by1[0] > by0[0] and by1[1] > by0[1], (by0, by1)  # both sides hashed
        assert got[5] == native.blake3(fifo_data).hex()
        for p, g in zip(paths, got):
            if p == fifo:
                continue
            h, st = want[p]
            if st != 0:
                assert isinstance(g, OSError), p
            else:
                assert g == h.tobytes().hex(), p
        # under 512 MiB of large files: the CPU path alone
        small_call = [p for p, sz in zip(paths[:4], sizes[:4])]
        sd.file_checksums(small_call)
        assert sd.file_checksums_stats()["cpu"] == after["cpu"] + 1
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)


@pytest.mark.parametrize("slots", [1, 15])
def test_file_checksums_split_block_edges(ctx, tmp_path, oracle_native, slots):
    """The block split (round 5) around its own boundaries: files of k MiB and k MiB +- 1 /
    1023 / 1024 / 1025 bytes (a last block of 1 byte up to a full one, and one-byte-short
    blocks), a file of 32 MiB (one GPU run exactly) and 33 MiB + 1, with the GPU given 1 slot
    (the host threads take most blocks, edge blocks included) or 15 (the GPU takes most):
    every root merged from the two sides' CVs equals the oracle's file_checksum."""
    import spacedrive_amd as sd
    MiB = 1 << 20
    sizes = [8 * MiB - 1, 8 * MiB, 8 * MiB + 1, 9 * MiB + 1023, 9 * MiB + 1024, 9 * MiB + 1025, 10 * MiB - 1024,
             32 * MiB, 33 * MiB + 1, 47 * MiB + 77, 64 * MiB - 1, 64 * MiB + 1, 100 * MiB + 3, 128 * MiB + 513,
             130 * MiB - 1]
    assert sum(sizes) >= 512 * MiB
    paths = []
    for i, L in enumerate(sizes):
        p = tmp_path / f"e{i}"
        with open(p, "wb") as f:
            pos = 0
            while pos < L:
                k = min(32 * MiB, L - pos)
                f.write(oracle_native.synth_bytes(9000 + i, 0, pos, k))
                pos += k
        paths.append(str(p))
    want = [w.tobytes().hex() for w in oracle_native.file_checksums(paths, nthreads=NT)[0]]
    locked = None
    if os.geteuid() != 0:  # a large file the call stats but cannot open: its error, the rest hashed
        locked = tmp_path / "locked"
        with open(locked, "wb") as f:
            f.truncate(24 * MiB)
        os.chmod(locked, 0)
        paths.insert(4, str(locked))
    keep = {k: sd.get_tuning(k) for k in ("checksum_cpu_max", "checksum_hybrid_threads", "checksum_split_blocks",
                                          "checksum_split_adapt")}
    sd.set_tuning("checksum_cpu_max", 2147483647)  # the library default (the module sets 0)
    sd.set_tuning("checksum_split_adapt", 0)  # always the split
    sd.set_tuning("checksum_hybrid_threads", slots)
    sd.set_tuning("checksum_split_blocks", 1)
    try:
        before = sd.file_checksums_stats()["hybrid"]
        for _ in range(2):  # the sides' shares differ run to run
            got = sd.file_checksums(paths)
            if locked is not None:
                assert isinstance(got.pop(4), PermissionError)
            assert got == want
        assert sd.file_checksums_stats()["hybrid"] == before + 2
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)


def test_file_checksums_learned_route(ctx, tmp_path, oracle_native):
    """"checksum_split_adapt" k (round 5, default 8): a call the split applies to takes the
    split or the CPU path alone by this context's recent GB/s of each -- each once, then the
    faster, the other every k-th call.  With k = 2 over six calls both routes run, each
    result equals the oracle's, and every call is counted on the route it took."""
    import spacedrive_amd as sd
    MiB = 1 << 20
    sizes = [64 * MiB + 5 * i for i in range(9)]
    paths = []
    for i, L in enumerate(sizes):
        p = tmp_path / f"r{i}"
        with open(p, "wb") as f:
            pos = 0
            while pos < L:
                k = min(32 * MiB, L - pos)
                f.write(oracle_native.synth_bytes(9500 + i, 0, pos, k))
                pos += k
        paths.append(str(p))
    want = [w.tobytes().hex() for w in oracle_native.file_checksums(paths, nthreads=NT)[0]]
    keep = {k: sd.get_tuning(k) for k in ("checksum_cpu_max", "checksum_split_adapt")}
    sd.set_tuning("checksum_cpu_max", 2147483647)  # the library default (the module sets 0)
    sd.set_tuning("checksum_split_adapt", 2)
    try:
        before = sd.file_checksums_stats()
        for _ in range(6):
            assert sd.file_checksums(paths) == want
        after = sd.file_checksums_stats()
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)
    took_split, took_cpu = after["hybrid"] - before["hybrid"], after["cpu"] - before["cpu"]
    assert took_split + took_cpu == 6 and after["gpu"] == before["gpu"]
    assert took_split >= 2 and took_cpu >= 2, (took_split, took_cpu)  # k = 2: the loser every 2nd call
    learned = sd.file_checksums_learned()  # each route counted once its warm-up call is past
    assert learned["split_calls"] >= 1 and learned["cpu_calls"] >= 1, learned
    assert learned["split_GBps"] > 0 and learned["cpu_GBps"] > 0, learned


def test_concurrent_callers_share_a_context(ctx, tmp_path):
    # the C ABI is thread-safe and re-entrant: 6 host threads, one context
    import threading
    import spacedrive_amd as sd
    paths, sizes = [], []
    for i in range(60):
        sz = [10, 5000, 102400, 300000][i % 4] + i
        p = tmp_path / f"t{i}"
        p.write_bytes(cs.synth_bytes(500 + i, 0, 0, sz))
        paths.append(str(p))
        sizes.append(sz)
    want = [cs.generate_cas_id(cs.synth_reader(500 + i), sizes[i]) for i in range(60)]
    errors = []

    def worker(k):
        try:
            for _ in range(5):
                sl = slice(k * 10, k * 10 + 10)
                got = sd.generate_cas_ids(paths[sl], sizes[sl])
                assert got == want[sl]
                sums = sd.file_checksums(paths[sl])
                assert all(isinstance(x, str) and len(x) == 64 for x in sums)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_concurrent_split_checksum_calls(ctx, tmp_path, oracle_native):
    """Two host threads, one context, each a split sd_file_checksums call (>= 512 MiB of
    files >= 8 MiB: the block split, round 5) at once, three times over: the calls share the
    context's pools and slots, and every checksum equals the oracle's."""
    import threading
    import spacedrive_amd as sd
    MiB = 1 << 20
    sets = [[40 * MiB + 7 * i for i in range(12)] + [3000, 77 * MiB], [64 * MiB + 11 * i for i in range(9)]]
    paths = []
    for s, lens in enumerate(sets):
        ps = []
        for i, L in enumerate(lens):
            p = tmp_path / f"s{s}_{i}"
            with open(p, "wb") as f:
                pos = 0
                while pos < L:
                    k = min(32 * MiB, L - pos)
                    f.write(oracle_native.synth_bytes(7000 + 100 * s + i, 0, pos, k))
                    pos += k
            ps.append(str(p))
        paths.append(ps)
    want = [[w.tobytes().hex() for w in oracle_native.file_checksums(ps, nthreads=NT)[0]] for ps in paths]
    keep = {k: sd.get_tuning(k) for k in ("checksum_cpu_max", "checksum_hybrid_threads", "checksum_split_adapt")}
    sd.set_tuning("checksum_cpu_max", 2147483647)  # the library default (the module sets 0)
    sd.set_tuning("checksum_split_adapt", 0)  # always the split
    sd.set_tuning("checksum_hybrid_threads", 6)
    errors = []
    before = sd.file_checksums_stats()["hybrid"]

    def worker(s):
        try:
            for _ in range(3):
                assert sd.file_checksums(paths[s]) == want[s]
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    try:
        th = [threading.Thread(target=worker, args=(s,)) for s in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=300)
        assert not any(x.is_alive() for x in th)
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)
    assert not errors, errors
    assert sd.file_checksums_stats()["hybrid"] == before + 6


@pytest.mark.parametrize("ring,hot", [(4, 0), (2, 0), (16, 1)])
def test_cas_ids_files_pipelined_windows(ctx, tmp_path, oracle_native, ring, hot):
    """sd_cas_ids_files over many 1 MiB windows (the readers run ahead through a ring of
    `ring` pinned windows while earlier windows are copied and hashed), with I/O errors and
    short files interleaved, equals the reference read schedule on the CPU -- with the
    readers writing the windows directly and through their cache-resident buffer
    ("files_stage_hot")."""
    import spacedrive_amd as sd
    from spacedrive_amd import synth
    from spacedrive_amd._native import lib
    from spacedrive_amd.device import stage_plan
    n = 400
    sizes, cids, twins = synth.library(0, n, n)
    sizes = np.minimum(sizes, np.uint64(1 << 34))
    ext, total = stage_plan(sizes)
    buf = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    paths = synth.write_files(str(tmp_path), sizes, buf, ext)
    plan = [int(x) for x in sizes]
    paths[7] = str(tmp_path / "missing")  # IO_ERROR(ENOENT)
    bigs = [i for i in range(n) if sizes[i] > 102400 and i != 7]
    big, fits = bigs[0], bigs[1]
    plan[big] = 2 * int(sizes[big]) + (10 << 20)  # planned far past EOF: the last sample hits EOF
    plan[fits] = int(sizes[fits]) + 1000  # planned a little past EOF: samples fit, tail at the real end
    small = [i for i in range(n) if 100 < sizes[i] <= 102400 and i != 7]
    plan[small[0]] = int(sizes[small[0]]) + 50  # whole kind, the file is shorter than planned
    plan[small[1]] = int(sizes[small[1]]) - 50  # whole kind, the file is longer than planned
    want, wst = oracle_native.cas_ids_files(paths, np.array(plan, np.uint64), nthreads=4)
    keep = {k: sd.get_tuning(k) for k in ("files_window_mb", "files_ring", "files_stage_hot")}
    sd.set_tuning("files_window_mb", 1)
    sd.set_tuning("files_ring", ring)
    sd.set_tuning("files_stage_hot", hot)
    try:
        got = sd.generate_cas_ids(paths, plan)
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)
    for i in range(n):
        if wst[i] == 0:
            assert got[i] == want[i].tobytes().hex(), i
        elif wst[i] == 3:
            assert isinstance(got[i], sd.UnexpectedEofError), i
        else:
            assert isinstance(got[i], FileNotFoundError), i
    assert wst[7] != 0 and wst[big] == 3 and wst[fits] == 0 and wst[small[0]] == 0 and wst[small[1]] == 0


def test_latency_path_coalesces_concurrent_single_file_calls(ctx, tmp_path):
    """Watcher / non_indexed callers (watcher/utils.rs:235,393,438-446, non_indexed.rs:164-187)
    hash one file per call from many tasks: sd_cas_id_path / sd_file_checksum_path must
    return exactly what the batch path returns, with errors per call, while the library
    folds the concurrent calls into fewer GPU batches."""
    import threading
    import spacedrive_amd as sd
    from oracle import native
    sizes = [1, 1017, 5000, 102400, 102401, 700_000, 3 << 20] * 6
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"w{i}.bin"
        p.write_bytes(native.synth_bytes(300 + i, 0, 0, s))
        paths.append(str(p))
    want_ids = sd.generate_cas_ids(paths, sizes)
    want_sums = sd.file_checksums(paths)
    sd.set_tuning("latency_cpu_max", 0)  # every single-file call goes to the GPU coalescer
    before = sd.coalescer_stats()
    got_ids, got_sums, errs = [None] * len(paths), [None] * len(paths), []
    barrier = threading.Barrier(len(paths))

    def worker(i):
        barrier.wait()
        got_ids[i] = sd.generate_cas_id(paths[i], sizes[i])
        got_sums[i] = sd.file_checksum(paths[i])
        try:
            sd.generate_cas_id(str(tmp_path / f"missing{i}"), 10)
        except FileNotFoundError:
            errs.append(i)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(paths))]
    try:
        for t in th:
            t.start()
        for t in th:
            t.join()
        after = sd.coalescer_stats()
        # a 700 000-B file planned as 900 000: the last sample ends at 681 144 and the tail
        # is read at the real end (SeekFrom::End, cas.rs:54) -- the reference returns an id
        content = open(paths[5], "rb").read()
        assert sd.generate_cas_id(paths[5], 900_000) == cs.generate_cas_id_file(content, 900_000)
        with pytest.raises(sd.UnexpectedEofError):  # planned 1.6 MB: a sample runs past EOF
            sd.generate_cas_id(paths[5], 1_600_000)
    finally:
        sd.set_tuning("latency_cpu_max", 16)
    assert got_ids == want_ids and got_sums == want_sums
    assert sorted(errs) == list(range(len(paths)))
    calls = after["requests"] - before["requests"]
    batches = after["batches"] - before["batches"]
    assert calls == 3 * len(paths) and after["cpu"] == before["cpu"]
    assert batches < calls and after["max_batch"] > 1, after


def test_pipeline_object_owners_vs_reference_replay(ctx, oracle_native):
    # hash (GPU) -> partition -> group -> owners == identifier_job_step replay on oracle cas_ids
    from oracle.identifier_spec import identifier_replay
    from spacedrive_amd.dedup import dedup_shard
    n = 20000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    h = gpu_cas(ctx, sizes, cids, twins)
    d_hash = torch.from_numpy(h.copy()).cuda()
    d_valid = torch.from_numpy((sizes != 0).astype(np.uint8)).cuda()
    recs, rep, ng, owner = dedup_shard(ctx, d_hash, d_valid, n, 0)
    got = np.arange(n)
    got[recs[:, 1].cpu().numpy()] = owner.cpu().numpy()
    ids = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=NT)
    cas = [None if sizes[i] == 0 else ids[i].tobytes().hex() for i in range(n)]
    want, _ = identifier_replay(cas)
    assert got.tolist() == want


def test_library_pipeline_parity_sharded(ctx):
    """scripts/parity_full.py at a reduced size: 4 shards of the library, cas_ids vs the
    oracle, and the 4-rank dedup exchange emulated with device partitions + device
    grouping vs the host grouping of the oracle's ids.  (The committed full-size run,
    10 M files over 8 shards + configs[3], is profiles/r1d_parity_full.json.)"""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "parity_full", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                                    "parity_full.py"))
    pf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pf)
    r = pf.cas_library(ctx, 400_000, 4, NT)
    assert r["cas_id_mismatches"] == 0, r["first_mismatches"]
    assert r["dedup"]["bucket_record_mismatches"] == 0 and r["dedup"]["bucket_rep_mismatches"] == 0
    assert r["dedup"]["duplicate_files"] > 0 and r["empty_files"] > 0


def test_file_api_past_4gib_sparse(ctx, tmp_path, oracle_native):
    """Files larger than 2^32 through the path-based entry points: the sample windows and
    the tail sit past 4 GiB (64-bit pread offsets in the stager).  The files are sparse,
    with the generator's bytes written only where generate_cas_id reads (cas.rs:31-58),
    so their cas_id equals that of the fully generated file; the checksum covers the
    holes too and is checked against the oracle over the file's bytes."""
    import spacedrive_amd as sd
    sizes = [(1 << 32) + 1, (5 << 30) + 12345]
    paths = []
    for i, s in enumerate(sizes):
        p = str(tmp_path / f"big{i}.bin")
        with open(p, "wb") as f:
            f.truncate(s)
            for off, ln in synth.sample_windows(s):
                f.seek(off)
                f.write(cs.synth_bytes(70 + i, 0, off, ln))
        paths.append(p)
    ids = sd.generate_cas_ids(paths, sizes)
    for i, s in enumerate(sizes):
        assert ids[i] == cs.generate_cas_id(cs.synth_reader(70 + i), s), s
    assert sd.generate_cas_id(paths[1], sizes[1]) == ids[1]  # the coalesced single-file path
    got, st = oracle_native.cas_ids_files(paths, sizes, nthreads=2)  # the reference's read schedule
    assert not st.any() and [g.tobytes().hex() for g in got] == ids
    sums = sd.file_checksums(paths[:1])
    data = np.memmap(paths[0], dtype=np.uint8, mode="r")
    want = oracle_native.checksum_mt(data, sizes[0], nthreads=NT).hex()
    assert sums[0] == want


def test_file_api_past_a_tebibyte_sparse(ctx, tmp_path, oracle_native):
    """Sampled files of 1-8 TiB (sparse) through the GPU route of sd_cas_ids_files and the
    latency path: the stager's 64-bit reads up to the footer, then the kernels -- equal to
    the Python spec (tests/test_cpu_path.py runs the CPU path and sd_cas_stage_files on the
    same files)."""
    import spacedrive_amd as sd
    from tests.test_cpu_path import _sparse_sampled
    sizes = [(1 << 40) + 12345, (1 << 42) + 3, (1 << 43) - 1]
    made = [(s, _sparse_sampled(tmp_path, f"tb{i}", s, 990 + i), 990 + i) for i, s in enumerate(sizes)]
    made = [m for m in made if m[1]]
    if not made:
        pytest.skip("the filesystem refuses files of 1 TiB")
    paths, szs = [p for _, p, _ in made], [s for s, _, _ in made]
    want = [cs.generate_cas_id(cs.synth_reader(c), s) for s, _, c in made]
    assert sd.generate_cas_ids(paths, szs) == want  # the module sets batch_cpu_max 0: the GPU route
    assert sd.generate_cas_id(paths[-1], szs[-1]) == want[-1]


def test_dedup_owners_matches_torch_rule(ctx):
    """sd_dedup_owners (one kernel) == identifier.object_owners (the torch statement)."""
    from spacedrive_amd.identifier import object_owners
    rng = np.random.default_rng(11)
    for m, chunk in ((0, 100), (1, 100), (100000, 100), (4099, 7)):
        idx = np.sort(rng.choice(10 * max(m, 1), m, replace=False)).astype(np.int64)
        rep = np.minimum(idx, idx[rng.integers(0, max(m, 1), m)] if m else idx)
        recs = torch.from_numpy(np.stack([rng.integers(0, 2**62, m), idx], axis=1).astype(np.int64)).cuda()
        d_rep = torch.from_numpy(rep).cuda()
        out = torch.full((max(m, 1),), -1, dtype=torch.int64, device="cuda")
        ctx.dedup_owners(recs, m, d_rep, out, chunk_size=chunk)
        torch.cuda.synchronize()
        want = object_owners(torch.from_numpy(idx), torch.from_numpy(rep), chunk_size=chunk).numpy()
        assert np.array_equal(out.cpu().numpy()[:m], want)


# ------------------------------------------------- file length != size (cas.rs read semantics)
def _mismatch_files(tmp_path, cases, base):
    paths, sizes = [], []
    for i, (flen, size) in enumerate(cases):
        p = tmp_path / f"mm{base}_{i}"
        with open(p, "wb") as f:
            pos = 0
            while pos < flen:
                k = min(64 << 20, flen - pos)
                f.write(cs.synth_bytes(base + i, 0, pos, k))
                pos += k
        paths.append(str(p))
        sizes.append(size)
    return paths, sizes


@pytest.mark.parametrize("route", ["batch", "single-gpu", "single-policy"])
def test_length_differs_from_size(ctx, tmp_path, oracle_native, route):
    """generate_cas_id on files whose length differs from the size the
    caller planned (a stale directory-walk metadata.len(), non_indexed.rs:168; a file that
    grows while it is scanned), through sd_cas_ids_files ("batch") and sd_cas_id_path
    (forced onto the GPU coalescer, and under the default CPU/GPU latency policy), equals
    the oracle's reference read schedule: fs::read to EOF for the whole kind (cas.rs:29),
    read_exact + seek(End(-8192)) for the sampled kind (cas.rs:31-58)."""
    import threading
    import spacedrive_amd as sd
    from tests.test_oracle import LENGTH_MISMATCH_CASES
    cases = LENGTH_MISMATCH_CASES + [
        (102_400 + 4096, 102_400),   # whole kind, 4 KiB longer than the largest whole size
        (64 * 1024, 65 * 1024),      # whole kind, 1 KiB short: a shorter message in the batch
        ((300 << 20) + 5, 100),      # whole kind, 300 MiB: the overflow streams over two windows
        (5 << 20, 300_000),          # sampled, far longer than size
    ]
    paths, sizes = _mismatch_files(tmp_path, cases, 4000)
    want, wst = oracle_native.cas_ids_files(paths, np.array(sizes, np.uint64), nthreads=4)
    if route == "batch":
        got = sd.generate_cas_ids(paths, sizes)
    else:
        got = [None] * len(paths)
        if route == "single-gpu":
            sd.set_tuning("latency_cpu_max", 0)
        try:
            def one(i):
                try:
                    got[i] = sd.generate_cas_id(paths[i], sizes[i])
                except OSError as e:  # noqa: PERF203
                    got[i] = e
            th = [threading.Thread(target=one, args=(i,)) for i in range(len(paths))]
            for t in th:
                t.start()
            for t in th:
                t.join()
        finally:
            sd.set_tuning("latency_cpu_max", 16)
    for i in range(len(paths)):
        if wst[i] == 0:
            assert got[i] == want[i].tobytes().hex(), (i, cases[i])
        else:
            assert wst[i] == 3 and isinstance(got[i], sd.UnexpectedEofError), (i, cases[i], got[i])


def test_long_whole_messages_staged(ctx, oracle_native):
    """Whole-kind messages longer than 8 + 102400 B (a file larger than the size it was
    staged with) through the staged entry points: sd_cas_ids and a device batch route them
    to the chunk-parallel kernels and scatter their hashes in order among normal ones."""
    import ctypes
    from spacedrive_amd._native import check, lib
    from spacedrive_amd.device import EXTENT_DTYPE
    rng = np.random.default_rng(12)
    lens = [102_409, 131_072, 131_073, 1 << 20, (1 << 20) + 8, 3 * (1 << 20) + 77, 9, 1000, 57352, 102_408]
    sizes = [5, 100, 102_400, 0, 77, 1, 1, 992, 200_000, 102_400]  # kinds follow size; lens are the messages
    ext = np.zeros(len(lens), EXTENT_DTYPE)
    off = 0
    for i, (L, s) in enumerate(zip(lens, sizes)):
        ext[i] = (s, off, L, 1 if s <= 102400 else 2)
        off = (off + L + 127) // 128 * 128
    staged = np.zeros(off + 64, np.uint8)
    for i, L in enumerate(lens):
        o = int(ext["msg_offset"][i])
        staged[o:o + L] = rng.integers(0, 256, L, dtype=np.uint8)
    want = oracle_native.checksums(staged, ext["msg_offset"], ext["msg_len"].astype(np.uint64), nthreads=NT)
    out = ctypes.create_string_buffer(17 * len(lens))
    check(lib().sd_cas_ids(ctx.handle, staged.ctypes.data, len(staged), ext.ctypes.data, len(lens), out, None))
    raw = out.raw  # one copy of the buffer
    for i in range(len(lens)):
        assert raw[17 * i:17 * i + 16].decode() == want[i, :8].tobytes().hex(), (i, lens[i])
    b = ctx.cas_batch(ext)
    d_st = torch.from_numpy(staged).cuda()
    h = torch.zeros(len(lens) * 32, dtype=torch.uint8, device="cuda")
    b.run(d_st, h)
    torch.cuda.synchronize()
    assert np.array_equal(h.cpu().numpy().reshape(-1, 32), want)


def test_checksum_reads_like_hash_rs(ctx, tmp_path):
    """sd_file_checksums reads 1 MiB calls until a short one (hash.rs:14-20): a FIFO
    (st_size 0) hashes what its first read returns, between ordinary packed files."""
    import threading
    import spacedrive_amd as sd
    from oracle import blake3_spec as b3
    fifo = str(tmp_path / "fifo")
    os.mkfifo(fifo)
    payload = cs.synth_bytes(97, 0, 0, 4000)
    a = tmp_path / "a"
    a.write_bytes(cs.synth_bytes(1, 0, 0, 5000))
    t = threading.Thread(target=lambda: open(fifo, "wb", buffering=0).write(payload))
    t.start()
    got = sd.file_checksums([str(a), fifo, str(a)])
    t.join()
    assert got[1] == b3.blake3(payload).hex()
    assert got[0] == got[2] == b3.blake3(cs.synth_bytes(1, 0, 0, 5000)).hex()


def test_latency_policy_routes_and_agrees(ctx, tmp_path):
    """few concurrent single-file calls are hashed on the CPU path
    (counted in coalescer_stats()["cpu"]), and give exactly what the GPU batch gives."""
    import spacedrive_amd as sd
    sizes = [10, 5000, 102400, 300000, 5 << 20]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"lp{i}"
        p.write_bytes(cs.synth_bytes(600 + i, 0, 0, s))
        paths.append(str(p))
    want = sd.generate_cas_ids(paths, sizes)
    want_sums = sd.file_checksums(paths)
    before = sd.coalescer_stats()
    got = [sd.generate_cas_id(p, s) for p, s in zip(paths, sizes)]
    sums = [sd.file_checksum(p) for p in paths]
    after = sd.coalescer_stats()
    assert got == want and sums == want_sums
    assert after["cpu"] - before["cpu"] == 2 * len(paths) and after["batches"] == before["batches"]


def test_batch_policy_routes_small_calls_to_the_cpu_path(ctx, tmp_path):
    """SURVEY.md §8(f) rank 4 for batch calls: a generate_cas_ids (sd_cas_ids_files) call of
    at most "batch_cpu_max" files is hashed on the CPU path (counted in
    cas_ids_files_stats()["cpu"]) and returns exactly the GPU route's ids and statuses,
    including a file shorter than its size and a missing path."""
    import spacedrive_amd as sd
    sizes = [0, 1, 1016, 102400, 102401, 300000, 5 << 20, 4000, 200000]
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"bp{i}"
        p.write_bytes(cs.synth_bytes(700 + i, 0, 0, s if i < 7 else s // 2))  # the last two shrank
        paths.append(str(p))
    paths.append(str(tmp_path / "missing"))
    sizes.append(5000)

    def ids():  # an id, or the error's type and errno
        return [r if isinstance(r, str) else (type(r).__name__, r.errno) for r in sd.generate_cas_ids(paths, sizes)]

    want = ids()
    assert sum(isinstance(r, str) for r in want) == len(paths) - 2, want  # the shrunk sampled file, the missing one
    s0 = sd.cas_ids_files_stats()
    sd.set_tuning("batch_cpu_max", len(paths))
    try:
        got = ids()
    finally:
        sd.set_tuning("batch_cpu_max", 0)
    s1 = sd.cas_ids_files_stats()
    assert got == want
    assert s1["cpu"] - s0["cpu"] == 1 and s1["gpu"] - s0["gpu"] == 0
    sd.set_tuning("batch_cpu_max", len(paths) - 1)  # one file more than the threshold: the GPU
    try:
        assert ids() == want
    finally:
        sd.set_tuning("batch_cpu_max", 0)
    s2 = sd.cas_ids_files_stats()
    assert s2["gpu"] - s1["gpu"] == 1 and s2["cpu"] == s1["cpu"]


def test_directory_paths_fail_like_the_reference(ctx, tmp_path, oracle_native):
    """Directories among the files of a GPU-route call: File::open succeeds on Linux and the
    first read fails with EISDIR (cas.rs:29,36; hash.rs:16), so each directory gets
    OSError(EISDIR) -- with a whole-kind and a sampled-kind size, and in a checksum call
    beside packed small files and a streamed large one -- while every regular file's result
    equals the oracle's."""
    import errno
    import spacedrive_amd as sd
    (tmp_path / "d1").mkdir()
    (tmp_path / "d2").mkdir()
    sizes = [3000, 150_000, 9 << 20, 1]
    files = []
    for i, n in enumerate(sizes):
        p = tmp_path / f"r{i}"
        p.write_bytes(cs.synth_bytes(900 + i, 0, 0, n))
        files.append(str(p))
    paths = [str(tmp_path / "d1"), files[0], str(tmp_path / "d2"), files[1], files[2], str(tmp_path / "d1"), files[3]]
    cas_sizes = [4096, 3000, 200_000, 150_000, 9 << 20, 102_400, 1]
    got = sd.generate_cas_ids(paths, cas_sizes)
    got_ck = sd.file_checksums(paths)
    for j, p in enumerate(paths):
        if p in files:
            content = open(p, "rb").read()
            assert got[j] == cs.generate_cas_id_file(content, cas_sizes[j]), j
            assert got_ck[j] == oracle_native.blake3(content).hex(), j
        else:
            for r in (got[j], got_ck[j]):
                assert isinstance(r, OSError) and r.errno == errno.EISDIR, (j, r)


def test_symlinks_and_unreadable_files(ctx, tmp_path, oracle_native):
    """File::open follows symlinks: a link to a regular file hashes as the file, a dangling
    link fails with ENOENT; a file without read permission fails with EACCES (checked only
    when not running as root, who may read it anyway).  GPU routes, one call each."""
    import errno
    import spacedrive_amd as sd
    content = cs.synth_bytes(950, 0, 0, 250_000)
    real = tmp_path / "real"
    real.write_bytes(content)
    (tmp_path / "link").symlink_to(real)
    (tmp_path / "dangling").symlink_to(tmp_path / "nowhere")
    locked = tmp_path / "locked"
    locked.write_bytes(content)
    locked.chmod(0)
    paths = [str(tmp_path / "link"), str(tmp_path / "dangling"), str(locked), str(real)]
    try:
        ids = sd.generate_cas_ids(paths, [250_000] * 4)
        cks = sd.file_checksums(paths)
    finally:
        locked.chmod(0o644)
    want_id, want_ck = cs.generate_cas_id_file(content, 250_000), oracle_native.blake3(content).hex()
    for r in (ids, cks):
        w = want_id if r is ids else want_ck
        assert r[0] == w and r[3] == w
        assert isinstance(r[1], OSError) and r[1].errno == errno.ENOENT
        if os.geteuid() != 0:
            assert isinstance(r[2], OSError) and r[2].errno == errno.EACCES
        else:
            assert r[2] == w


def test_dedup_mgpu_through_rccl_single_rank(ctx, rccl_comm):
    """sd_cas_dedup_mgpu through a real RCCL communicator (1 rank: the
    all-gather and the grouped send/recv to self run; no world == 1 short-circuit) equals
    the host grouping; an undersized output fails with SD_ERR_CAPACITY before the exchange
    and the retrying runner recovers."""
    from spacedrive_amd import dedup
    from spacedrive_amd._native import SD_ERR_CAPACITY, SdCasError
    from spacedrive_amd.identifier import object_owners
    n = 60000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    h = gpu_cas(ctx, sizes, cids, twins)
    d_hash = torch.from_numpy(h.copy()).cuda()
    valid = (sizes != 0)
    d_valid = torch.from_numpy(valid.astype(np.uint8)).cuda()
    comm = rccl_comm
    base = 7_000_000  # a shard of a larger library
    recs_h = np.stack([keys_from_hashes(h)[valid].view(np.int64), np.arange(base, base + n)[valid]], axis=1)
    gr, grep, gng = group_host(recs_h)
    small = torch.empty((10, 2), dtype=torch.int64, device="cuda")
    with pytest.raises(SdCasError) as e:
        ctx.dedup_mgpu(comm, d_hash, d_valid, n, base, small, small[:, 0].clone(), small[:, 0].clone(), 10)
    assert e.value.rc == SD_ERR_CAPACITY and e.value.needed == int(valid.sum())
    runner = dedup.RcclDedup(ctx, comm, d_hash.device, capacity=100)  # regrows once
    for _ in range(2):  # and reuses its buffers
        recs, rep, ng, owner = runner(d_hash, d_valid, n, base)
        torch.cuda.synchronize()
        assert ng == gng
        assert np.array_equal(recs.cpu().numpy(), gr)
        assert np.array_equal(rep.cpu().numpy(), grep)
        want_owner = object_owners(torch.from_numpy(gr[:, 1].copy()), torch.from_numpy(grep), 100).numpy()
        assert np.array_equal(owner.cpu().numpy(), want_owner)
    # the torch.distributed exchange path gives the same outputs
    r2, rep2, ng2, own2 = dedup.dedup_shard(ctx, d_hash, d_valid, n, base)
    assert ng2 == gng and np.array_equal(r2.cpu().numpy(), gr) and np.array_equal(own2.cpu().numpy(), want_owner)


def test_dedup_mgpu_bounded_wait_breaks_the_comm(ctx):
    """"comm_timeout_ms" (round 6): over RCCL every wait of sd_cas_dedup_mgpu for its peers
    is bounded.  A host function that holds the call's stream stands in for a peer that never
    arrives (no spinning kernel, no abort -- safe on a shared box): the call returns
    SD_ERR_COMM naming the step within the bound, the communicator refuses every later call,
    and once the stream is released its queued work drains and sd_comm_destroy returns."""
    import threading
    import time
    import spacedrive_amd as sd
    from spacedrive_amd import dedup
    from spacedrive_amd._native import SdCasError
    comm = dedup.make_comm(ctx)  # its own: the fixture's communicator stays usable
    n = 5000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    d_hash = torch.from_numpy(gpu_cas(ctx, sizes, cids, twins).copy()).cuda()
    d_valid = torch.from_numpy((sizes != 0).astype(np.uint8)).cuda()
    recs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    rep = torch.empty(n, dtype=torch.int64, device="cuda")
    own = torch.empty(n, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    m, ng = ctx.dedup_mgpu(comm, d_hash, d_valid, n, 0, recs, rep, own, n, stream=s)  # a normal call
    assert m == int((sizes != 0).sum()) and ng > 0
    s.synchronize()
    gate = threading.Event()
    hold = ctypes.CFUNCTYPE(None, ctypes.c_void_p)(lambda _: gate.wait(60))
    hip = ctypes.CDLL("libamdhip64.so")
    keep = sd.get_tuning("comm_timeout_ms")
    sd.set_tuning("comm_timeout_ms", 300)
    try:
        assert hip.hipLaunchHostFunc(ctypes.c_void_p(s.cuda_stream), hold, None) == 0
        t0 = time.monotonic()
        with pytest.raises(SdCasError) as e:
            ctx.dedup_mgpu(comm, d_hash, d_valid, n, 0, recs, rep, own, n, stream=s)
        waited = time.monotonic() - t0
        assert e.value.rc == -5 and "all-gather of the count rows" in str(e.value), str(e.value)
        assert "comm_timeout_ms = 300" in str(e.value) and 0.25 < waited < 20, waited
    finally:
        gate.set()
        sd.set_tuning("comm_timeout_ms", keep)
    s.synchronize()  # the call's queued partition and all-gather drain (one rank: RCCL to self)
    with pytest.raises(SdCasError) as e2:
        ctx.dedup_mgpu(comm, d_hash, d_valid, n, 0, recs, rep, own, n, stream=s)
    assert e2.value.rc == -5 and "broken" in str(e2.value)
    comm.close()  # a broken communicator releases nothing, and does not wait
    assert keep == 300000


def test_dedup_of_one_batch_beside_the_next_batchs_hashing(ctx, rccl_comm):
    """The pipelined scan (bench.py steps_pipelined): batch k's
    sd_cas_dedup_mgpu on one stream while batch k+1 hashes on another, two hash buffers
    alternating.  Every batch's grouping equals the host grouping of its own hashes."""
    from spacedrive_amd import dedup
    from spacedrive_amd.identifier import object_owners
    n, B = 40000, 4
    libs = [synth.library(k * n, n, B * n, dup_frac=0.2) for k in range(B)]
    staged = [stage_synth(ctx, *lib) for lib in libs]
    batches = [ctx.cas_batch(ext) for ext, _, _ in staged]
    torch.cuda.synchronize()  # staged before the other streams read it
    valid = [torch.from_numpy((lib[0] != 0).astype(np.uint8)).cuda() for lib in libs]
    hs, ds = torch.cuda.Stream(), torch.cuda.Stream()
    bufs = [torch.zeros(n * 32, dtype=torch.uint8, device="cuda") for _ in range(2)]
    e_hash = [torch.cuda.Event() for _ in range(2)]
    e_ded = [torch.cuda.Event() for _ in range(2)]
    runner = dedup.RcclDedup(ctx, rccl_comm, bufs[0].device, capacity=n + 1024)
    got, hashes = [], []

    def hash_into(k):
        b = k & 1
        if k >= 2:
            hs.wait_event(e_ded[b])
        batches[k].run(staged[k][2], bufs[b], hs)
        e_hash[b].record(hs)

    hash_into(0)
    for k in range(B):
        b = k & 1
        if k + 1 < B:
            hash_into(k + 1)
        ds.wait_event(e_hash[b])
        recs, rep, ng, owner = runner(bufs[b].view(n, 32), valid[k], n, k * n, stream=ds)
        ds.synchronize()
        got.append((recs.cpu().numpy(), rep.cpu().numpy(), ng, owner.cpu().numpy()))
        hashes.append(bufs[b].cpu().numpy().reshape(n, 32))  # still batch k's: batch k+2 waits for e_ded
        e_ded[b].record(ds)
    torch.cuda.synchronize()
    for k in range(B):
        h = hashes[k]
        assert np.array_equal(h, gpu_cas(ctx, *libs[k]))
        ok = libs[k][0] != 0
        gr, grep, gng = group_host(np.stack([keys_from_hashes(h)[ok].view(np.int64),
                                             np.arange(k * n, (k + 1) * n)[ok]], axis=1))
        recs, rep, ng, owner = got[k]
        assert ng == gng and np.array_equal(recs, gr) and np.array_equal(rep, grep)
        want_owner = object_owners(torch.from_numpy(gr[:, 1].copy()), torch.from_numpy(grep), 100).numpy()
        assert np.array_equal(owner, want_owner)


def test_checksums_from_host_memory(ctx, oracle_native):
    """sd_checksums: ranges of a host buffer (pinned) -> hex, packed windows and a range
    larger than a window (streamed with a known length), against the oracle."""
    import ctypes
    from spacedrive_amd._native import check, lib
    MiB = 1 << 20
    lens = [0, 1, 1025, MiB + 3, 5 * MiB, (300 << 20) + 5, 77, 2 * MiB - 1]
    offs, off = [], 0
    for L in lens:
        offs.append(off)
        off = (off + L + 64 + 63) // 64 * 64
    host = torch.empty(off + 64, dtype=torch.uint8, pin_memory=True)
    d = torch.zeros(off + 64, dtype=torch.uint8, device="cuda")
    for i, (L, o) in enumerate(zip(lens, offs)):
        if L:
            ctx.synth_fill(800 + i, 0, L, d[o:])
    torch.cuda.synchronize()
    host.copy_(d.cpu())
    del d
    arr_o = np.array(offs, np.uint64)
    arr_l = np.array(lens, np.uint64)
    out = ctypes.create_string_buffer(65 * len(lens))
    check(lib().sd_checksums(ctx.handle, host.data_ptr(), arr_o.ctypes.data, arr_l.ctypes.data, len(lens), out))
    want = oracle_native.checksums_simd(host.numpy(), arr_o, arr_l, nthreads=NT)
    raw = out.raw  # one copy of the buffer
    for i in range(len(lens)):
        assert raw[65 * i:65 * i + 64].decode() == want[i].tobytes().hex(), lens[i]


@pytest.mark.parametrize("cohash", [0, 15])
def test_checksums_from_host_memory_cohashed(ctx, oracle_native, cohash):
    """sd_checksums over > 1 GiB of host ranges (large ranges streamed, runs of small ones
    packed) with host threads co-hashing from the end ("host_cohash_threads" 15: large
    ranges block-parallel on the CPU path, small ones in batches) and without: every hash
    equals the oracle's, whichever side took its range."""
    import ctypes
    import spacedrive_amd as sd
    from spacedrive_amd._native import check, lib
    MiB = 1 << 20
    rng = np.random.default_rng(41)
    lens = [(300 << 20) + 5, 0, 77, (150 << 20) + 1] + [int(x) for x in rng.integers(1, 3 * MiB, 180)] + \
        [(260 << 20) + 3, 9 * MiB, 1025, (200 << 20) + 64, 5]
    offs, off = [], 0
    for L in lens:
        offs.append(off)
        off = (off + L + 128 + 127) // 128 * 128
    assert off > (1 << 30)
    d = torch.randint(0, 256, (off + 64,), dtype=torch.uint8, device="cuda")
    host = torch.empty(off + 64, dtype=torch.uint8, pin_memory=True)
    host.copy_(d)
    del d
    arr_o = np.array(offs, np.uint64)
    arr_l = np.array(lens, np.uint64)
    out = ctypes.create_string_buffer(65 * len(lens))
    keep = sd.get_tuning("host_cohash_threads")
    sd.set_tuning("host_cohash_threads", cohash)
    st0, st1 = np.zeros(2, np.uint64), np.zeros(2, np.uint64)
    try:
        check(lib().sd_checksums_stats(ctx.handle, st0.ctypes.data))
        check(lib().sd_checksums(ctx.handle, host.data_ptr(), arr_o.ctypes.data, arr_l.ctypes.data, len(lens), out))
        check(lib().sd_checksums_stats(ctx.handle, st1.ctypes.data))
    finally:
        sd.set_tuning("host_cohash_threads", keep)
    want = oracle_native.checksums_simd(host.numpy(), arr_o, arr_l, nthreads=NT)
    raw = out.raw
    for i in range(len(lens)):
        assert raw[65 * i:65 * i + 64].decode() == want[i].tobytes().hex(), (i, lens[i])
    # sd_checksums_stats: every byte counted once, on the side that hashed it
    d_gpu, d_host = (int(x) for x in (st1 - st0))
    assert d_gpu + d_host == sum(lens)
    assert (d_host > 0 and d_gpu > 0) if cohash else d_host == 0


def test_checksums_learned_route(ctx, oracle_native):
    """"checksum_split_adapt" k for sd_checksums (round 6): a co-hash-eligible call (>= 1 GiB)
    runs co-hashed (the GPU + host threads) or on the CPU path alone, each once as a warm-up
    and once counted, then the faster by its learned GB/s and the other every k-th call.
    Every call's hashes equal the oracle's, whichever route ran; a CPU-route call hashes
    every byte on the host (sd_checksums_stats), a co-hashed one gives the GPU a share."""
    import spacedrive_amd as sd
    from spacedrive_amd._native import check, lib
    lens = [(300 << 20) + 5, 77, (400 << 20) + 1, 3 << 20, (360 << 20) + 3]
    offs, off = [], 0
    for L in lens:
        offs.append(off)
        off = (off + L + 128 + 127) // 128 * 128
    assert sum(lens) >= 1 << 30
    d = torch.randint(0, 256, (off + 64,), dtype=torch.uint8, device="cuda")
    host = torch.empty(off + 64, dtype=torch.uint8, pin_memory=True)
    host.copy_(d)
    del d
    arr_o, arr_l = np.array(offs, np.uint64), np.array(lens, np.uint64)
    want = [w.tobytes().hex() for w in oracle_native.checksums_simd(host.numpy(), arr_o, arr_l, nthreads=NT)]
    out = ctypes.create_string_buffer(65 * len(lens))
    keep = {k: sd.get_tuning(k) for k in ("checksum_split_adapt", "host_cohash_threads")}
    sd.set_tuning("host_cohash_threads", 14)  # a change of a key the rates depend on:
    sd.set_tuning("host_cohash_threads", 15)  # the context learns afresh
    sd.set_tuning("checksum_split_adapt", 2)
    routes = []
    try:
        for _ in range(8):
            st0, st1 = np.zeros(2, np.uint64), np.zeros(2, np.uint64)
            check(lib().sd_checksums_stats(ctx.handle, st0.ctypes.data))
            ctypes.memset(out, 0, 65 * len(lens))
            check(lib().sd_checksums(ctx.handle, host.data_ptr(), arr_o.ctypes.data, arr_l.ctypes.data, len(lens),
                                     out))
            check(lib().sd_checksums_stats(ctx.handle, st1.ctypes.data))
            raw = out.raw
            assert [raw[65 * i:65 * i + 64].decode() for i in range(len(lens))] == want
            d_gpu, d_host = (int(x) for x in (st1 - st0))
            assert d_gpu + d_host == sum(lens)
            routes.append("cpu" if d_gpu == 0 else "cohash")
        learned = sd.checksums_learned()
    finally:
        for k, v in keep.items():
            sd.set_tuning(k, v)
    assert routes[:2] == ["cohash", "cohash"] and routes[2:4] == ["cpu", "cpu"], routes
    assert learned["cohash_calls"] >= 1 and learned["cpu_calls"] >= 1 and learned["cohash_GBps"] > 0, learned
    faster = "cohash" if learned["cohash_GBps"] >= learned["cpu_GBps"] else "cpu"
    assert faster in routes[4:] and len(set(routes[4:])) == 2, routes  # k = 2: the other every 2nd call


@pytest.mark.parametrize("cohash", [0, 15])
def test_checksums_one_huge_range_shared(ctx, oracle_native, cohash):
    """sd_checksums with ranges of >= 256 MiB: with host co-hashing the one nearest the
    predicted meeting point has its 1 MiB blocks shared -- the GPU takes windows from the
    front, the host 64-block claims from the back, the host's chaining values are uploaded
    beside the GPU's and one reduce gives the hash; the other ranges are claimed whole.
    Cases: one huge range alone; huge ranges among small ones before and after; six 300 MiB
    ranges (the shared one in the middle); and a 2 GiB range first, then four of 64 MiB
    (the shared range is the GPU's first, the host reaches it last).  Every hash equals
    the oracle's."""
    import ctypes
    import spacedrive_amd as sd
    from spacedrive_amd._native import check, lib
    MiB = 1 << 20
    cases = [[(1 << 30) + 12345],
             [3000, 5 * MiB + 1, (2 << 30) + 777, 64, (1 << 30) + (1 << 20), 1025],
             [300 * MiB + 17 * i for i in range(6)],
             [(2 << 30) + 3] + [64 * MiB] * 4]
    for lens in cases:
        offs, off = [], 0
        for L in lens:
            offs.append(off)
            off = (off + L + 127) // 128 * 128
        d = torch.randint(0, 256, (off + 64,), dtype=torch.uint8, device="cuda")
        host = torch.empty(off + 64, dtype=torch.uint8, pin_memory=True)
        host.copy_(d)
        del d
        arr_o = np.array(offs, np.uint64)
        arr_l = np.array(lens, np.uint64)
        out = ctypes.create_string_buffer(65 * len(lens))
        keep = sd.get_tuning("host_cohash_threads")
        sd.set_tuning("host_cohash_threads", cohash)
        try:
            check(lib().sd_checksums(ctx.handle, host.data_ptr(), arr_o.ctypes.data, arr_l.ctypes.data, len(lens),
                                     out))
        finally:
            sd.set_tuning("host_cohash_threads", keep)
        hn = host.numpy()
        raw = out.raw
        for i, (o, L) in enumerate(zip(offs, lens)):
            want = oracle_native.checksum_mt(hn[o:o + L], L, nthreads=NT).hex()
            assert raw[65 * i:65 * i + 64].decode() == want, (lens, i, L)
        del host


def test_checksums_host_ranges_any_layout(ctx, oracle_native):
    """sd_checksums over host ranges laid out every way a caller may: 16-byte starts (leaf-
    sized ranges then start a new copy run on a 128-B device line), gaps,
    a range hashed twice (overlap), one that lies before the previous one, small ranges
    between big ones, and more than one 256 MiB window -- against the oracle."""
    import ctypes
    from spacedrive_amd._native import check, lib
    MiB = 1 << 20
    rng = np.random.default_rng(355)
    span = 300 * MiB
    host = torch.empty(span + 128, dtype=torch.uint8, pin_memory=True)
    host.numpy()[:] = rng.integers(0, 256, span + 128, dtype=np.uint8)
    offs, lens, off = [], [], 16
    for L in [MiB + 16, 7, 3 * MiB + 5, 2 * MiB, 100, 5 * MiB + 1, 64 * MiB + 48, 1025, 130 * MiB + 3,
              90 * MiB + 16, 2 * MiB + 1]:
        offs.append(off)
        lens.append(L)
        off = (off + L + 16 * int(rng.integers(0, 9)) + 15) // 16 * 16  # gaps of 0..128 bytes
    assert off <= span
    offs += [offs[2], offs[1], 48]              # hashed again; before the previous range
    lens += [lens[2], lens[1], 4 * MiB + 9]
    arr_o = np.array(offs, np.uint64)
    arr_l = np.array(lens, np.uint64)
    out = ctypes.create_string_buffer(65 * len(lens))
    check(lib().sd_checksums(ctx.handle, host.data_ptr(), arr_o.ctypes.data, arr_l.ctypes.data, len(lens), out))
    want = oracle_native.checksums_simd(host.numpy(), arr_o, arr_l, nthreads=NT)
    raw = out.raw
    for i in range(len(lens)):
        assert raw[65 * i:65 * i + 64].decode() == want[i].tobytes().hex(), (i, offs[i], lens[i])


def test_checksums_host_ranges_end_at_a_guard_page(ctx, oracle_native):
    """sd_checksums reads no byte past a range: pageable buffers whose last range ends at
    an unreadable (PROT_NONE) page, through the packed window and the streamed (> 256 MiB)
    route.  The last range starts 16-byte aligned and ends 16 bytes past a 64-byte boundary,
    so reading up to the next 64-byte boundary (the old window copy) would fault."""
    import ctypes
    import mmap
    from spacedrive_amd._native import check, lib
    page = mmap.PAGESIZE
    # the third set: leaf-sized ranges at mid-line starts, each copied as its own run (§3.2b)
    for lens in ([3, 1000, 4096 + 16], [(300 << 20) + 16], [5, (1 << 20) + 16, 3 * (1 << 20) + 7, (2 << 20) + 16]):
        offs, off = [], 0
        for L in lens:
            off = (off + 15) // 16 * 16
            offs.append(off)
            off += L
        span = off
        npages = (span + page - 1) // page
        m = mmap.mmap(-1, (npages + 1) * page)  # the data, then the guard page
        whole = np.frombuffer(m, dtype=np.uint8)
        base = whole.ctypes.data
        start = base + npages * page - span     # the last range ends at the guard page
        assert start % 16 == 0
        data = whole[npages * page - span:npages * page]
        rng = np.random.default_rng(len(lens))
        data[:] = rng.integers(0, 256, span, dtype=np.uint8)
        padded = np.concatenate([data, np.zeros(128, np.uint8)])  # the oracle's own copy
        libc = ctypes.CDLL(None, use_errno=True)
        assert libc.mprotect(ctypes.c_void_p(base + npages * page), page, 0) == 0  # PROT_NONE
        arr_o = np.array(offs, np.uint64)
        arr_l = np.array(lens, np.uint64)
        out = ctypes.create_string_buffer(65 * len(lens))
        check(lib().sd_checksums(ctx.handle, start, arr_o.ctypes.data, arr_l.ctypes.data, len(lens), out))
        want = oracle_native.checksums_simd(padded, arr_o, arr_l, nthreads=NT)
        raw = out.raw
        for i in range(len(lens)):
            assert raw[65 * i:65 * i + 64].decode() == want[i].tobytes().hex(), lens[i]
        assert libc.mprotect(ctypes.c_void_p(base + npages * page), page, 3) == 0  # back to RW
        del data, whole
        m.close()


def test_checksums_host_ranges_around_a_guard_page(ctx, oracle_native):
    """ranges on both sides of an unreadable page inside one window -- small
    ranges (which share a run with their neighbours) included -- are hashed without reading
    the hole: a gap that holds a whole page no range touches starts a new H2D run."""
    import ctypes
    import mmap
    from spacedrive_amd._native import check, lib
    page = mmap.PAGESIZE
    m = mmap.mmap(-1, 6 * page)
    whole = np.frombuffer(m, dtype=np.uint8)
    rng = np.random.default_rng(5)
    whole[:] = rng.integers(0, 256, whole.size, dtype=np.uint8)
    base = whole.ctypes.data
    libc = ctypes.CDLL(None, use_errno=True)
    hole = 3 * page  # pages [3, 4) unreadable
    # before the hole: two small ranges sharing page 2; after it: small ranges on page 4, 5
    offs = [2 * page + 16, 2 * page + 1024, 3 * page - 48, hole + page, hole + page + 80, 5 * page + 16]
    lens = [100, 2000, 48, 64, 1000, page - 32]
    assert libc.mprotect(ctypes.c_void_p(base + hole), page, 0) == 0
    try:
        arr_o = np.array(offs, np.uint64)
        arr_l = np.array(lens, np.uint64)
        out = ctypes.create_string_buffer(65 * len(lens))
        check(lib().sd_checksums(ctx.handle, base, arr_o.ctypes.data, arr_l.ctypes.data, len(lens), out))
    finally:
        assert libc.mprotect(ctypes.c_void_p(base + hole), page, 3) == 0
    padded = np.concatenate([whole, np.zeros(128, np.uint8)])
    want = oracle_native.checksums_simd(padded, arr_o, arr_l, nthreads=NT)
    raw = out.raw
    for i in range(len(lens)):
        assert raw[65 * i:65 * i + 64].decode() == want[i].tobytes().hex(), i
    del whole
    m.close()


def test_coalesced_batches_take_the_batch_policies(ctx, tmp_path):
    """beyond "latency_cpu_max" calls in flight, single-file calls are coalesced
    and the dispatcher hands each batch to sd_cas_ids_files / sd_file_checksums, whose batch
    policies then route it: with the defaults a coalesced batch (at most "coalesce_max" =
    4096 files) is hashed on the CPU path, with the policies off on the GPU.  Same results."""
    import threading
    import spacedrive_amd as sd
    from oracle import native
    sizes = [1, 1017, 102400, 102401, 700_000] * 8
    paths = []
    for i, s in enumerate(sizes):
        p = tmp_path / f"c{i}.bin"
        p.write_bytes(native.synth_bytes(500 + i, 0, 0, s))
        paths.append(str(p))
    want_ids = sd.generate_cas_ids(paths, sizes)
    want_sums = sd.file_checksums(paths)

    def burst():
        ids, sums = [None] * len(paths), [None] * len(paths)
        barrier = threading.Barrier(len(paths))

        def worker(i):
            barrier.wait()
            ids[i] = sd.generate_cas_id(paths[i], sizes[i])
            sums[i] = sd.file_checksum(paths[i])
        th = [threading.Thread(target=worker, args=(i,)) for i in range(len(paths))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return ids, sums

    keep = {k: sd.get_tuning(k) for k in ("batch_cpu_max", "checksum_cpu_max")}
    sd.set_tuning("latency_cpu_max", 0)  # every single-file call is coalesced
    try:
        for policy in ("default", "off"):
            sd.set_tuning("batch_cpu_max", 4096 if policy == "default" else 0)
            sd.set_tuning("checksum_cpu_max", 2147483647 if policy == "default" else 0)
            c0, k0 = sd.cas_ids_files_stats(), sd.file_checksums_stats()
            ids, sums = burst()
            c1, k1 = sd.cas_ids_files_stats(), sd.file_checksums_stats()
            assert ids == want_ids and sums == want_sums, policy
            route = "cpu" if policy == "default" else "gpu"
            other = "gpu" if route == "cpu" else "cpu"
            assert c1[route] > c0[route] and c1[other] == c0[other], (policy, c0, c1)
            assert k1[route] > k0[route] and k1[other] == k0[other], (policy, k0, k1)
    finally:
        sd.set_tuning("latency_cpu_max", 16)
        for k, v in keep.items():
            sd.set_tuning(k, v)


def test_split_checksum_ranks_on_one_gpu(ctx, oracle_native):
    """One file over R ranks (sd_split_checksum_leaves / _root), the ranks emulated on one
    device: each rank's leaves read only its own slice (a view at its byte range) and write
    only its own CV slots, so one shared CV buffer stands for the gathered one.  Bit-exact
    vs the oracle's BLAKE3 of the whole file, up to 4 GiB + 12345 (block CVs past 2^32)."""
    from spacedrive_amd.device import SplitChecksum
    MiB = 1 << 20
    cases = [(0, (1, 2)), (1, (1, 3)), (MiB, (1, 2)), (MiB + 1, (1, 2, 3)), (5 * MiB + 3, (1, 2, 4, 7)),
             (300 * MiB + 77, (3, 8)), ((4 << 30) + 12345, (1, 3, 8))]
    for total, ranks in cases:
        d = torch.zeros(total + 128, dtype=torch.uint8, device="cuda")
        if total:
            ctx.synth_fill(900, 0, total, d)
        want = oracle_native.checksum_synth_mt(total, 900, 0, nthreads=NT).hex()
        for R in ranks:
            cvs = None
            splits = [SplitChecksum(ctx, total, R, r) for r in range(R)]
            for sc in splits:
                if cvs is None:
                    cvs = torch.zeros(sc.cv_bytes, dtype=torch.uint8, device="cuda")
                sc.leaves(d[sc.offset:], cvs)
            out = torch.zeros(32, dtype=torch.uint8, device="cuda")
            splits[0].root(cvs, out)
            torch.cuda.synchronize()
            assert bytes(out.cpu().numpy()).hex() == want, (total, R)
            for sc in splits:
                sc.close()
        del d


def test_split_checksum_mgpu_through_rccl_single_rank(ctx, oracle_native, rccl_comm):
    """sd_split_checksum_mgpu over a real (single-rank) RCCL communicator, and the
    torch.distributed statement (checksum_split) on the device, against the oracle."""
    from spacedrive_amd._native import SdCasError
    from spacedrive_amd.device import SplitChecksum
    from spacedrive_amd.split import checksum_split
    total = (37 << 20) + 5
    d = torch.zeros(total + 128, dtype=torch.uint8, device="cuda")
    ctx.synth_fill(901, 0, total, d)
    want = oracle_native.checksum_synth_mt(total, 901, 0, nthreads=NT).hex()
    comm = rccl_comm
    sc = SplitChecksum(ctx, total, 1, 0)
    cvs = torch.zeros(sc.cv_bytes, dtype=torch.uint8, device="cuda")
    out = torch.zeros(32, dtype=torch.uint8, device="cuda")
    sc.mgpu(comm, d, cvs, out)
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()).hex() == want
    bad = SplitChecksum(ctx, total, 2, 0)  # a split for another world size
    with pytest.raises(SdCasError):
        bad.mgpu(comm, d, torch.zeros(bad.cv_bytes, dtype=torch.uint8, device="cuda"), out)
    assert checksum_split(d[:total + 64], total, ctx=ctx) == want


def _run_ranks(R, fn):
    """fn(rank) on R threads (ctypes releases the GIL inside the library); results by rank,
    the first exception re-raised."""
    import threading
    out, errs = [None] * R, []

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(R)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=180)
    assert not any(t.is_alive() for t in ts), "a rank thread did not finish"
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("R", [2, 3, 5, 8])
def test_dedup_mgpu_in_process_ranks(ctx, R):
    """sd_cas_dedup_mgpu with R > 1 ranks (configs[4]'s exchange): RCCL
    refuses two ranks on one GPU, so the ranks are threads of this process on the in-process
    transport (sd_comm_create_local) -- the same partition, gathered count matrix, capacity
    check, per-peer offsets, grouping and Object rule as over RCCL.  Uneven shards; each
    rank's output == the host grouping of the records whose cas_id prefix it owns, with the
    chunk-of-100 owners; an undersized rank makes every rank return SD_ERR_CAPACITY, and a
    second round of calls on the same communicators (buffers reused) agrees."""
    from spacedrive_amd import dedup
    from spacedrive_amd._native import SD_ERR_CAPACITY, SdCasError
    from spacedrive_amd.dedup import dest_of
    from spacedrive_amd.device import Comm, CommGroup, Context
    from spacedrive_amd.identifier import object_owners
    n = 90000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    h = gpu_cas(ctx, sizes, cids, twins)
    valid = sizes != 0
    keys = keys_from_hashes(h)
    cuts = [0] + [int(c) for c in np.cumsum(np.random.default_rng(R).dirichlet(np.ones(R)) * n)[:-1]] + [n]
    group = CommGroup(R)
    ctxs = [Context(0) for _ in range(R)]
    comms = [Comm(ctxs[r], None, R, r, group=group) for r in range(R)]
    d_hash = torch.from_numpy(h.reshape(-1).copy()).cuda()  # flat: a shard is a byte offset
    d_valid = torch.from_numpy(valid.astype(np.uint8)).cuda()
    torch.cuda.synchronize()
    all_recs = np.stack([keys[valid].view(np.int64), np.arange(n)[valid]], axis=1)
    dst = dest_of(all_recs[:, 0].view(np.uint64), R)

    def rank_call(r, capacity):
        lo, hi = cuts[r], cuts[r + 1]
        st = torch.cuda.Stream()
        if capacity is not None:
            buf = torch.empty((max(capacity, 1), 2), dtype=torch.int64, device="cuda")
            try:
                ctxs[r].dedup_mgpu(comms[r], d_hash[lo * 32:], d_valid[lo:], hi - lo, lo, buf, buf[:, 0].clone(),
                                   buf[:, 1].clone(), capacity, stream=st)
            except SdCasError as e:
                return e.rc, e.needed
            return 0, None
        runner = dedup.RcclDedup(ctxs[r], comms[r], d_hash.device, capacity=hi - lo + 1024)
        res = []
        for _ in range(2):
            recs, rep, ng, own = runner(d_hash[lo * 32:], d_valid[lo:], hi - lo, lo, stream=st)
            st.synchronize()
            res.append((recs.cpu().numpy(), rep.cpu().numpy(), ng, own.cpu().numpy()))
        return res

    try:
        # rank 1 undersized: every rank stops before the exchange, each told its own need
        caps = [n] * R
        caps[1] = 3
        got = _run_ranks(R, lambda r: rank_call(r, caps[r]))
        for r in range(R):
            assert got[r] == (SD_ERR_CAPACITY, int((dst == r).sum())), (r, got[r])
        got = _run_ranks(R, lambda r: rank_call(r, None))
        assert sum(len(g[0][0]) for g in got) == int(valid.sum())
        for r in range(R):
            gr, grep, gng = group_host(all_recs[dst == r])
            want_owner = object_owners(torch.from_numpy(gr[:, 1].copy()), torch.from_numpy(grep), 100).numpy()
            for recs, rep, ng, own in got[r]:
                assert ng == gng, (r, ng, gng)
                assert np.array_equal(recs, gr) and np.array_equal(rep, grep)
                assert np.array_equal(own, want_owner)
    finally:
        for c in comms:
            c.close()
        group.close()
        for c in ctxs:
            c.close()


def test_split_checksum_mgpu_in_process_ranks(ctx, oracle_native):
    """sd_split_checksum_mgpu over R = 3 and 4 in-process ranks: each rank hashes its own
    blocks into its own CV buffer, the in-place all-gather fills the others' slots, and
    every rank's root equals the oracle's BLAKE3 of the whole file."""
    from spacedrive_amd.device import Comm, CommGroup, Context, SplitChecksum
    total = (45 << 20) + 77
    d = torch.zeros(total + 128, dtype=torch.uint8, device="cuda")
    ctx.synth_fill(902, 0, total, d)
    torch.cuda.synchronize()
    want = oracle_native.checksum_synth_mt(total, 902, 0, nthreads=NT).hex()
    for R in (3, 4):
        group = CommGroup(R)
        ctxs = [Context(0) for _ in range(R)]
        comms = [Comm(ctxs[r], None, R, r, group=group) for r in range(R)]

        def rank(r):
            sc = SplitChecksum(ctxs[r], total, R, r)
            cvs = torch.zeros(sc.cv_bytes, dtype=torch.uint8, device="cuda")
            out = torch.zeros(32, dtype=torch.uint8, device="cuda")
            st = torch.cuda.Stream()
            sc.mgpu(comms[r], d[sc.offset:], cvs, out, stream=st)
            st.synchronize()
            sc.close()
            return bytes(out.cpu().numpy()).hex()

        try:
            assert _run_ranks(R, rank) == [want] * R
        finally:
            for c in comms:
                c.close()
            group.close()
            for c in ctxs:
                c.close()


def _need_devices(k):
    if torch.cuda.device_count() < k:
        pytest.skip(f"needs {k} visible GPUs (the pool's boxes have one): the in-process communicator's "
                    "cross-device copies are untested there")


@pytest.mark.parametrize("R", [2, 4])
def test_dedup_mgpu_in_process_ranks_across_devices(R):
    """The in-process communicator with its ranks on DIFFERENT devices of one process
    (README: several GPUs from one process): each rank's shard, context,
    stream and output on device r % ndev, the exchange's peer copies (hipMemcpyDefault)
    crossing devices.  Each rank's groups, representatives and Object owners == the host
    grouping.  Skipped where fewer than two GPUs are visible."""
    _need_devices(2)
    from spacedrive_amd import dedup
    from spacedrive_amd.dedup import dest_of
    from spacedrive_amd.device import Comm, CommGroup, Context
    from spacedrive_amd.identifier import object_owners
    ndev = torch.cuda.device_count()
    n = 60000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    c0 = Context(0)
    try:
        h = gpu_cas(c0, sizes, cids, twins)
    finally:
        c0.close()
    valid = sizes != 0
    keys = keys_from_hashes(h)
    cuts = [0] + [int(c) for c in np.cumsum(np.random.default_rng(R).dirichlet(np.ones(R)) * n)[:-1]] + [n]
    group = CommGroup(R)
    ctxs = [Context(r % ndev) for r in range(R)]
    comms = [Comm(ctxs[r], None, R, r, group=group) for r in range(R)]
    all_recs = np.stack([keys[valid].view(np.int64), np.arange(n)[valid]], axis=1)
    dst = dest_of(all_recs[:, 0].view(np.uint64), R)

    def rank_call(r):
        lo, hi = cuts[r], cuts[r + 1]
        dev = torch.device("cuda", r % ndev)
        with torch.cuda.device(dev):
            d_hash = torch.from_numpy(h[lo:hi].reshape(-1).copy()).to(dev)
            d_valid = torch.from_numpy(valid[lo:hi].astype(np.uint8)).to(dev)
            st = torch.cuda.Stream(device=dev)
            runner = dedup.RcclDedup(ctxs[r], comms[r], dev, capacity=n)
            recs, rep, ng, own = runner(d_hash, d_valid, hi - lo, lo, stream=st)
            st.synchronize()
            assert recs.device == dev
            return recs.cpu().numpy(), rep.cpu().numpy(), ng, own.cpu().numpy()

    try:
        got = _run_ranks(R, rank_call)
        assert sum(len(g[0]) for g in got) == int(valid.sum())
        for r in range(R):
            gr, grep, gng = group_host(all_recs[dst == r])
            want_owner = object_owners(torch.from_numpy(gr[:, 1].copy()), torch.from_numpy(grep), 100).numpy()
            recs, rep, ng, own = got[r]
            assert ng == gng and np.array_equal(recs, gr) and np.array_equal(rep, grep)
            assert np.array_equal(own, want_owner)
    finally:
        for c in comms:
            c.close()
        group.close()
        for c in ctxs:
            c.close()


def test_split_checksum_mgpu_in_process_ranks_across_devices(oracle_native):
    """sd_split_checksum_mgpu over in-process ranks on different devices: each rank's slice
    and CV buffer on its own device, the in-place all-gather copying CV slots across
    devices; every rank's root == the oracle.  Skipped where fewer than two GPUs are
    visible."""
    _need_devices(2)
    from spacedrive_amd.device import Comm, CommGroup, Context, SplitChecksum
    ndev = torch.cuda.device_count()
    R = max(2, min(4, ndev))
    total = (37 << 20) + 501
    want = oracle_native.checksum_synth_mt(total, 903, 0, nthreads=NT).hex()
    group = CommGroup(R)
    ctxs = [Context(r % ndev) for r in range(R)]
    comms = [Comm(ctxs[r], None, R, r, group=group) for r in range(R)]

    def rank(r):
        dev = torch.device("cuda", r % ndev)
        with torch.cuda.device(dev):
            sc = SplitChecksum(ctxs[r], total, R, r)
            d = torch.zeros(sc.len + 128, dtype=torch.uint8, device=dev)
            if sc.len:
                ctxs[r].synth_fill(903, 0, sc.len, d, offset=sc.offset)
            cvs = torch.zeros(sc.cv_bytes, dtype=torch.uint8, device=dev)
            out = torch.zeros(32, dtype=torch.uint8, device=dev)
            st = torch.cuda.Stream(device=dev)
            torch.cuda.synchronize(dev)
            sc.mgpu(comms[r], d, cvs, out, stream=st)
            st.synchronize()
            sc.close()
            return bytes(out.cpu().numpy()).hex()

    try:
        assert _run_ranks(R, rank) == [want] * R
    finally:
        for c in comms:
            c.close()
        group.close()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("route", ["batch", "single-gpu"])
def test_pipe_whole_kind_reads_every_byte(ctx, tmp_path, oracle_native, route):
    """generate_cas_id on a pipe (a metadata length of 0, as non_indexed passes for one):
    fs::read takes every byte the writer gives until it closes (cas.rs:29).  A pipe cannot
    be read twice, so the stager keeps its bytes and hashes le64(0) || them from memory."""
    import threading
    import spacedrive_amd as sd
    from spacedrive_amd._native import lib
    data = cs.synth_bytes(77, 0, 0, 150000)
    fifo = str(tmp_path / "pipe")
    os.mkfifo(fifo)
    plain = tmp_path / "plain"
    plain.write_bytes(b"x" * 5000)

    def writer():
        with open(fifo, "wb") as f:
            for o in range(0, len(data), 4000):
                f.write(data[o:o + 4000])

    t = threading.Thread(target=writer)
    t.start()
    try:
        if route == "batch":
            got = sd.generate_cas_ids([str(plain), fifo], [5000, 0])
        else:
            assert lib().sd_cas_set_tuning(b"latency_cpu_max", 0) == 0  # the GPU-coalesced route
            try:
                got = [sd.generate_cas_id(str(plain), 5000), sd.generate_cas_id(fifo, 0)]
            finally:
                lib().sd_cas_set_tuning(b"latency_cpu_max", 16)
    finally:
        t.join()
    le64 = lambda v: int(v).to_bytes(8, "little")  # noqa: E731  (cas.rs:25)
    assert got[0] == oracle_native.blake3(le64(5000) + b"x" * 5000)[:8].hex()
    assert got[1] == oracle_native.blake3(le64(0) + data)[:8].hex()


def test_file_checksum_split_on_device(ctx, tmp_path, oracle_native):
    """split.file_checksum_split: the rank's byte range of a file read from disk and hashed
    by the device's split leaves + root (one rank here) == the oracle's BLAKE3 of the file."""
    from spacedrive_amd.split import file_checksum_split
    n = (9 << 20) + 4321
    data = cs.synth_bytes(902, 0, 0, n)
    p = tmp_path / "big.bin"
    p.write_bytes(data)
    assert file_checksum_split(str(p), ctx=ctx) == oracle_native.blake3(data).hex()


def test_hashes_files_to_device_then_rccl_dedup(ctx, tmp_path, oracle_native, rccl_comm):
    """sd_cas_hashes_files -> sd_cas_dedup_mgpu: a rank's library scan from files with the
    hashes left on the device.  Rows equal the oracle's full hashes of the reference's
    messages (including a whole file that outgrew its size and an empty file), d_valid
    marks hashed non-empty files, and the RCCL dedup over those rows equals the host
    grouping of the oracle's cas_ids."""
    import spacedrive_amd as sd  # noqa: F401
    from spacedrive_amd import synth
    n = 3000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    sizes = np.minimum(sizes, np.uint64(1 << 30))
    ext, total = sd.stage_plan(sizes)
    buf = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    paths = synth.write_files(str(tmp_path), sizes, buf, ext)
    plan = sizes.copy()
    small = [i for i in range(n) if 100 < sizes[i] <= 102400]
    plan[small[0]] = sizes[small[0]] - 60  # the file is longer than its metadata said: re-read
    paths[5] = str(tmp_path / "missing")
    want, wst = oracle_native.cas_ids_files(paths, plan, nthreads=NT)
    d_hash = torch.zeros((n, 32), dtype=torch.uint8, device="cuda")
    d_valid = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = ctx.hashes_files(paths, plan, d_hash, d_valid)
    assert np.array_equal(st != 0, wst != 0) and st[5] != 0
    h = d_hash.cpu().numpy()
    ok = st == 0
    assert np.array_equal(h[ok, :8], want[ok])
    assert np.array_equal(d_valid.cpu().numpy().astype(bool), ok & (plan != 0))
    # the rank's dedup over the device rows, as a multi-GPU scan would run it
    base = 40_000
    cap = n + 16
    recs = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    rep = torch.empty(cap, dtype=torch.int64, device="cuda")
    own = torch.empty(cap, dtype=torch.int64, device="cuda")
    m, ng = ctx.dedup_mgpu(rccl_comm, d_hash, d_valid, n, base, recs, rep, own, cap)
    torch.cuda.synchronize()
    valid = ok & (plan != 0)
    recs_h = np.stack([keys_from_hashes(h)[valid].view(np.int64), np.arange(base, base + n)[valid]], axis=1)
    gr, grep, gng = group_host(recs_h)
    assert m == len(gr) and ng == gng
    assert np.array_equal(recs[:m].cpu().numpy(), gr) and np.array_equal(rep[:m].cpu().numpy(), grep)


def test_scan_library_from_files(ctx, tmp_path, oracle_native, rccl_comm):
    """library.scan_library: shard plan -> files hashed into device rows -> RCCL dedup ->
    Object owners, one rank; equal to the oracle's cas_ids (the reference's reads) and to
    the host grouping and chunk-of-100 rule over them; the torch.distributed exchange gives
    the same result."""
    from spacedrive_amd import synth
    from spacedrive_amd.identifier import object_owners
    from spacedrive_amd.library import scan_library
    n = 2500
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.3)
    sizes = np.minimum(sizes, np.uint64(1 << 30))
    from spacedrive_amd.device import stage_plan
    ext, total = stage_plan(sizes)
    buf = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    paths = synth.write_files(str(tmp_path), sizes, buf, ext)
    paths[11] = str(tmp_path / "missing")
    want, wst = oracle_native.cas_ids_files(paths, sizes, nthreads=NT)
    r = scan_library(ctx, paths, sizes, comm=rccl_comm)
    assert r["shard"] == (0, n)
    for i in range(n):
        if wst[i] == 0:
            assert r["cas_ids"][i] == want[i].tobytes().hex(), i
        else:
            assert isinstance(r["cas_ids"][i], OSError), i
    valid = (wst == 0) & (sizes != 0)
    keys = want.copy().view(">u8").reshape(-1).astype(np.uint64)
    gr, grep, gng = group_host(np.stack([keys[valid].view(np.int64), np.arange(n)[valid]], axis=1))
    assert r["n_groups"] == gng
    assert np.array_equal(r["records"].cpu().numpy(), gr) and np.array_equal(r["rep"].cpu().numpy(), grep)
    own = object_owners(torch.from_numpy(gr[:, 1].copy()), torch.from_numpy(grep), 100).numpy()
    assert np.array_equal(r["owner"].cpu().numpy(), own)
    t = scan_library(ctx, paths, sizes)  # the torch.distributed statement of the exchange
    assert t["n_groups"] == gng and np.array_equal(t["records"].cpu().numpy(), gr)


def test_wrappers_order_side_streams_after_the_current_stream(ctx, oracle_native, rccl_comm):
    """The Python wrappers that take a `stream` (CasBatch.run, RcclDedup, SplitChecksum.mgpu)
    order it after the work queued on the current stream: each input below is produced by
    a kernel just queued on the current stream, and the wrapper is called on a fresh side
    stream with no manual wait_stream -- its outputs equal the serial ones."""
    from spacedrive_amd import dedup
    from spacedrive_amd.device import SplitChecksum
    n = 200_000
    sizes, cids, twins = synth.library(0, n, n, dup_frac=0.2)
    want = gpu_cas(ctx, sizes, cids, twins)  # serial, synchronised
    # (1) CasBatch.run: the staged messages are still being generated on the current stream
    ext, _, d_staged = stage_synth(ctx, sizes, cids, twins)
    b = ctx.cas_batch(ext)
    side = torch.cuda.Stream()
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")  # a fill queued on the current stream
    b.run(d_staged, out, side)
    side.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(n, 32), want)
    # (2) RcclDedup: the hashes are being recomputed on the current stream
    d_hash = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    b.run(d_staged, d_hash)
    valid = (sizes != 0)
    d_valid = torch.from_numpy(valid.astype(np.uint8)).cuda()
    runner = dedup.RcclDedup(ctx, rccl_comm, d_hash.device, capacity=n + 1024)
    recs, rep, ng, owner = runner(d_hash.view(n, 32), d_valid, n, 0, stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    keys = keys_from_hashes(want)
    gr, grep, gng = group_host(np.stack([keys.view(np.int64), np.arange(n, dtype=np.int64)], 1)[valid])
    assert ng == gng and np.array_equal(recs.cpu().numpy(), gr) and np.array_equal(rep.cpu().numpy(), grep)
    # (3) SplitChecksum.mgpu: 1 GiB of file bytes still being generated on the current stream
    total = (1 << 30) + 333
    d = torch.empty(total + 128, dtype=torch.uint8, device="cuda")
    ctx.synth_fill(903, 0, total, d)
    sc = SplitChecksum(ctx, total, 1, 0)
    cvs = torch.zeros(sc.cv_bytes, dtype=torch.uint8, device="cuda")
    h = torch.zeros(32, dtype=torch.uint8, device="cuda")
    side2 = torch.cuda.Stream()
    sc.mgpu(rccl_comm, d, cvs, h, stream=side2)
    side2.synchronize()
    assert bytes(h.cpu().numpy()).hex() == oracle_native.checksum_synth_mt(total, 903, 0, nthreads=NT).hex()
    sc.close()
    b.close()
