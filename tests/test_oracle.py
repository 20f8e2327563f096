"""The oracle itself: pinned to the reference's KAT and the official BLAKE3 vectors,
and the C restatement cross-checked against the Python spec and the goldens."""
import numpy as np
import pytest

from oracle import blake3_spec as b3
from oracle import cas_spec as cs


def pat(n):
    return bytes(i % 251 for i in range(n))


def test_kat_derive_b3(golden):
    # crates/crypto/src/keys/hashing.rs:210-213,323-328 via blake3::derive_key
    k = golden["kat_derive_b3"]
    got = b3.derive_key(k["context"], bytes.fromhex(k["key_hex"] + k["salt_hex"]))
    assert list(got) == k["expected"]


def test_official_vectors(golden):
    for n, h in golden["blake3_official"]["hash"].items():
        assert b3.blake3(pat(int(n))).hex() == h, n


def _stack_shape(n):
    # spec CV-stack tree (Hasher.update/finalize) on symbolic leaves
    stack, cur = [], None
    for c in range(n):
        if cur is not None:
            total = c
            node = cur
            while total & 1 == 0:
                node = (stack.pop(), node)
                total >>= 1
            stack.append(node)
        cur = c
    out = cur
    for left in reversed(stack):
        out = (left, out)
    return out


def _level_shape(n):
    level = list(range(n))
    while len(level) > 1:
        nxt = [(level[i], level[i + 1]) for i in range(0, len(level) - 1, 2)]
        if len(level) & 1:
            nxt.append(level[-1])
        level = nxt
    return level[0]


def _blocked_shape(n, group):
    # kernels: aligned power-of-two groups merged level-wise, then level-wise on top
    groups = [_level_shape_range(s, min(s + group, n)) for s in range(0, n, group)]
    while len(groups) > 1:
        nxt = [(groups[i], groups[i + 1]) for i in range(0, len(groups) - 1, 2)]
        if len(groups) & 1:
            nxt.append(groups[-1])
        groups = nxt
    return groups[0]


def _level_shape_range(a, b):
    level = list(range(a, b))
    while len(level) > 1:
        nxt = [(level[i], level[i + 1]) for i in range(0, len(level) - 1, 2)]
        if len(level) & 1:
            nxt.append(level[-1])
        level = nxt
    return level[0]


def test_tree_shapes_equal():
    # SURVEY.md §7 "hard parts": level-wise merge with odd carry == spec tree, 1..600 chunks;
    # and the kernels' blocked form (4- or 16-chunk lanes, 1024-chunk blocks, 256-way groups)
    for n in range(1, 601):
        s = _stack_shape(n)
        assert _level_shape(n) == s, n
        assert _blocked_shape(n, 4) == s, n
        assert _blocked_shape(n, 16) == s, n
        assert _blocked_shape(n, 64) == s, n
    for n in (1023, 1024, 1025, 4097, 70000):
        assert _blocked_shape(n, 1024) == _level_shape(n), n


def _eager_fold(nodes, tail=None):
    # k_cas_sampled_merge / k_whole_merge8 (cas_kernels.hip): each node merges into a CV
    # stack as it arrives (while (i + 1) is even), the last node stays out of the stack
    # unless a tail follows, then the stack folds onto it from the top
    st, cur = [], None
    for i, nd in enumerate(nodes):
        cur, t = nd, i + 1
        while t % 2 == 0:
            cur, t = (st.pop(), cur), t // 2
        if tail is not None or i + 1 < len(nodes):
            st.append(cur)
    if tail is not None:
        cur = tail
    while st:
        cur = (st.pop(), cur)
    return cur


def test_kernel_stack_merges_equal_spec_tree():
    # the sampled pair: 56 full chunks in groups of U (lanes kernel, level-wise in-lane),
    # then the merge kernel folds the 56/U group CVs and the tail chunk 56
    for u in (2, 4, 8):
        groups = [_level_shape_range(s, s + u) for s in range(0, 56, u)]
        assert _eager_fold(groups, tail=56) == _stack_shape(57), u
    # whole-file messages of 1..128 chunks: pair nodes, merge8 pass A over aligned groups
    # of <= 8 pairs, pass B over <= 8 of those
    for n in range(1, 129):
        pairs = [_level_shape_range(s, min(s + 2, n)) for s in range(0, n, 2)]
        a = [_eager_fold(pairs[s:s + 8]) for s in range(0, len(pairs), 8)]
        assert _eager_fold(a) == _stack_shape(n), n


def test_levelwise_hash_matches_spec():
    for n in (0, 1, 64, 65, 1024, 1025, 3 * 1024 + 7, 8 * 1024, 9 * 1024 + 1):
        assert b3.levelwise_hash(pat(n)) == b3.blake3(pat(n)), n


def test_cas_goldens_python(golden):
    cp = golden["cas_pattern"]["cas_id"]
    for s in ("0", "1", "1016", "1017", "102400", "102401", "4294967297"):
        reader = lambda o, n: bytes((o + k) % 251 for k in range(n))
        assert cs.generate_cas_id(reader, int(s)) == cp[s]


def test_sample_windows_reference_trace():
    # cas.rs:35-58: samples at 8192 + k*seek_jump, k = 0..3, footer at size - 8192
    for size in (102401, 131072, 1 << 20, (1 << 32) + 1):
        w = cs.sample_windows(size)
        j = (size - 16384) // 4
        assert w == [(0, 8192)] + [(8192 + k * j, 10240) for k in range(4)] + [(size - 8192, 8192)]
    assert sum(n for _, n in cs.sample_windows(102401)) + 8 == cs.SAMPLED_MSG_LEN == 57352


def test_threshold_is_inclusive():
    # cas.rs:27: size <= 102400 hashes the whole file (SURVEY.md spec discrepancy note)
    assert len(cs.cas_message(lambda o, n: bytes(n), 102400)) == 8 + 102400
    assert len(cs.cas_message(lambda o, n: bytes(n), 102401)) == 57352


def test_c_oracle_blake3_vs_spec(oracle_native):
    rng = np.random.default_rng(1)
    for n in [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 4096, 5000, 16385, 66000]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle_native.blake3(data) == b3.blake3(data), n


def test_c_oracle_cas_goldens(oracle_native, golden):
    files = golden["cas_synth"]["files"]
    sizes = np.array([f["size"] for f in files], np.uint64)
    cids = np.array([f["content_id"] for f in files], np.uint64)
    twins = np.array([f["twin"] for f in files], np.uint32)
    for nt in (1, 4):
        out = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=nt)
        for f, h in zip(files, out):
            assert h.tobytes().hex() == f["cas_id"], f


def test_c_oracle_checksum_goldens(oracle_native, golden):
    files = golden["checksum_synth"]["files"]
    sizes = np.array([f["size"] for f in files], np.uint64)
    cids = np.array([f["content_id"] for f in files], np.uint64)
    twins = np.array([f["twin"] for f in files], np.uint32)
    out = oracle_native.checksums_synth(sizes, cids, twins, nthreads=3)
    for f, h in zip(files, out):
        assert h.tobytes().hex() == f["checksum"], f
    cp = golden["checksum_pattern"]["checksum"]
    for s, h in cp.items():
        data = np.frombuffer(pat(int(s)) + bytes(64), np.uint8)
        got = oracle_native.checksums(data, [0], [int(s)])[0].tobytes().hex()
        assert got == h, s


def test_twins_share_cas_not_checksum(oracle_native):
    size = 3 << 20
    a = oracle_native.cas_ids_synth(np.array([size, size], np.uint64), np.array([9, 9], np.uint64),
                                    np.array([0, 7], np.uint32))
    assert a[0].tobytes() == a[1].tobytes()
    c = oracle_native.checksums_synth(np.array([size, size], np.uint64), np.array([9, 9], np.uint64),
                                      np.array([0, 7], np.uint32))
    assert c[0].tobytes() != c[1].tobytes()


def test_synth_generator_c_vs_python(oracle_native, golden):
    for cid, hexs in golden["cas_synth"]["synth_prefix40"].items():
        assert oracle_native.synth_bytes(int(cid), 0, 0, 40).hex() == hexs
    rng = np.random.default_rng(5)
    for _ in range(50):
        cid, off, ln = int(rng.integers(0, 1 << 62)), int(rng.integers(0, 1 << 33)), int(rng.integers(0, 300))
        tw = int(rng.integers(0, 3))
        assert oracle_native.synth_bytes(cid, tw, off, ln) == cs.synth_bytes(cid, tw, off, ln)
    assert oracle_native.synth_bytes(3, 5, 18430, 4) == cs.synth_bytes(3, 5, 18430, 4)


HUGE_SAMPLED = [(1 << 32) - 1, (1 << 32) + 1, (1 << 33) + 7, (1 << 40) + 12345, (1 << 50) - 1, (1 << 62) + 3,
                (1 << 64) - 1]


def test_c_oracle_huge_sampled_sizes_vs_spec(oracle_native):
    """Sampled files far past 4 GiB -- a 1 TiB video, sizes up to u64's maximum: the sample
    offsets 8192 + k * ((size - 16384) / 4) (cas.rs:41-51), the footer at size - 8192
    (cas.rs:54-57) and the le64 header all need 64-bit arithmetic.  The C oracle's cas
    messages and cas_ids equal the Python spec's over the same synthetic content."""
    sizes = np.array(HUGE_SAMPLED, np.uint64)
    cids = np.arange(700, 700 + len(sizes), dtype=np.uint64)
    ids = oracle_native.cas_ids_synth(sizes, cids, np.zeros(len(sizes), np.uint32), nthreads=2)
    for i, size in enumerate(HUGE_SAMPLED):
        msg = cs.cas_message(cs.synth_reader(int(cids[i])), size)
        assert len(msg) == 57352 and msg[:8] == size.to_bytes(8, "little")
        assert oracle_native.cas_message(int(cids[i]), 0, size) == msg, size
        assert ids[i].tobytes().hex() == cs.generate_cas_id(cs.synth_reader(int(cids[i])), size), size


@pytest.mark.parametrize("level", [1, 2])
def test_c_oracle_simd_multichunk(oracle_native, level):
    # the CPU-baseline hasher (hash_many over chunks and parents) vs the scalar oracle
    if oracle_native.simd_level(level) != level:
        pytest.skip("CPU lacks this SIMD level")
    rng = np.random.default_rng(level)
    for n in [0, 1, 64, 1023, 1024, 1025, 2049, 15 * 1024, 16 * 1024, 17 * 1024 + 3, 57352, 102408, 333333]:
        d = rng.integers(0, 256, n + 64, dtype=np.uint8)
        want = b3.blake3(d[:n].tobytes()) if n < 5000 else oracle_native.blake3(d[:n].tobytes())
        assert oracle_native.checksums_simd(d, [0], [n], simd=level)[0].tobytes() == want, n


@pytest.mark.parametrize("level", [1, 2])
def test_c_oracle_simd_synth_cas_ids(oracle_native, level):
    # the library-scale parity checker (SIMD hasher over generated messages) == scalar
    if oracle_native.simd_level(level) != level:
        pytest.skip("CPU lacks this SIMD level")
    from spacedrive_amd import synth
    sizes, cids, twins = synth.library(0, 4000, 4000)
    want = oracle_native.cas_ids_synth(sizes, cids, twins, nthreads=4)
    got = oracle_native.cas_ids_synth_simd(sizes, cids, twins, nthreads=4, simd=level)
    assert np.array_equal(got, want)


def test_c_oracle_file_backed_reads(oracle_native, tmp_path):
    """The reference's read schedule from files (cas.rs:27-58) equals the staged path;
    missing and short files map to IO_ERROR(ENOENT) and SHORT_READ."""
    from spacedrive_amd import synth
    from spacedrive_amd.device import stage_plan
    sizes = np.array([1, 1016, 1017, 102400, 102401, 555555, (1 << 32) + 1, 3 << 20], np.uint64)
    cids = np.arange(40, 40 + len(sizes), dtype=np.uint64)
    twins = np.zeros(len(sizes), np.uint32)
    twins[-1] = 5
    ext, total = stage_plan(sizes)
    buf = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    paths = synth.write_files(str(tmp_path), sizes, buf, ext)
    want = oracle_native.cas_ids_synth(sizes, cids, twins)
    for simd, nt in ((0, 1), (-1, 3)):
        got, st = oracle_native.cas_ids_files(paths, sizes, nthreads=nt, simd=simd)
        assert (st == 0).all(), st
        assert np.array_equal(got, want)
    got, st = oracle_native.cas_ids_files([str(tmp_path / "missing"), paths[5], paths[5]],
                                          [10, 555555 + 500000, 555555 + 9000])
    assert st[0] & 0xFFFF == 2 and st[0] >> 16 == 2  # ENOENT
    assert st[1] == 3  # the last sample's read_exact runs past EOF
    # planned 9000 B too large, but every sample still fits and the footer is read at the
    # file's real end (SeekFrom::End, cas.rs:54): the reference returns an id
    assert st[2] == 0
    content = open(paths[5], "rb").read()
    assert got[2].tobytes().hex() == oracle_native.blake3(cs.cas_message_file(content, 555555 + 9000))[:8].hex()


# (file length, size passed to generate_cas_id) pairs whose lengths differ, and the
# reference's outcome: the hashed stream (cas_spec.cas_message_file) or its error
LENGTH_MISMATCH_CASES = [
    (5000, 9000),               # whole kind, file shorter than size: fs::read hashes the 5000 bytes
    (9000, 5000),               # whole kind, file longer than size
    (150_000, 1000),            # whole kind, file longer than 100 KiB (message > 102408 B)
    (3 << 20, 100),             # whole kind, message far beyond the whole-file kernels' 128 chunks
    (777, 0),                   # size 0 (non_indexed.rs:168 passes it): le64(0) || the bytes
    (700_000, 300_000),         # sampled, file longer than size: footer at the real EOF
    (700_000, 900_000),         # sampled, file shorter than size, every sample still fits
    (700_000, 1_600_000),       # sampled, a sample runs past EOF: UnexpectedEof
    (5000, 200_000),            # sampled, the header runs past EOF: UnexpectedEof
]


def test_c_oracle_length_differs_from_size(oracle_native, tmp_path):
    """cas.rs on files whose length differs from the size argument: the C restatement's
    read schedule (fs::read to EOF; read_exact; seek(End(-8192))) == the Python
    statement, scalar and SIMD."""
    paths, sizes, want = [], [], []
    for i, (flen, size) in enumerate(LENGTH_MISMATCH_CASES):
        content = cs.synth_bytes(900 + i, 0, 0, flen)
        p = tmp_path / f"m{i}"
        p.write_bytes(content)
        paths.append(str(p))
        sizes.append(size)
        try:
            want.append(oracle_native.blake3(cs.cas_message_file(content, size))[:8].hex())
        except cs.UnexpectedEof:
            want.append(3)
    for simd in (0, -1):
        got, st = oracle_native.cas_ids_files(paths, np.array(sizes, np.uint64), nthreads=2, simd=simd)
        for i, w in enumerate(want):
            if w == 3:
                assert st[i] == 3, i
            else:
                assert st[i] == 0 and got[i].tobytes().hex() == w, (i, LENGTH_MISMATCH_CASES[i])
    # the Python statement itself on small cases, against the pure-Python spec
    content = cs.synth_bytes(5, 0, 0, 3000)
    assert cs.generate_cas_id_file(content, 2000) == b3.blake3(b"\xd0\x07" + bytes(6) + content).hex()[:16]
    with pytest.raises(cs.UnexpectedEof):  # the header fits, the second sample (at 54096) does not
        cs.cas_message_file(bytes(20000), 200_000)
    with pytest.raises(cs.UnexpectedEof):
        cs.cas_message_file(bytes(8000), 200_000)


def test_c_oracle_file_checksum_read_schedule(oracle_native, tmp_path):
    """hash.rs:10-24 from files: 1 MiB read calls until a short one, hashed through a CV
    stack of 1 MiB subtrees (scalar and SIMD) == the one-shot hash of the whole file."""
    MiB = 1 << 20
    sizes = [0, 1, 1024, 1025, MiB - 1, MiB, MiB + 1, 2 * MiB, 3 * MiB + 5, 4 * MiB, 5 * MiB + 77, 8 * MiB + 1]
    paths, datas = [], []
    for i, s in enumerate(sizes):
        d = np.frombuffer(cs.synth_bytes(70 + i, 0, 0, s) if s < 64 else
                          oracle_native.synth_bytes(70 + i, 0, 0, s), np.uint8)
        p = tmp_path / f"k{i}"
        p.write_bytes(d.tobytes())
        paths.append(str(p))
        datas.append(d)
    paths.append(str(tmp_path / "missing"))
    for simd in (0, -1):
        got, st = oracle_native.file_checksums(paths, nthreads=3, simd=simd)
        assert st[-1] & 0xFFFF == 2 and st[-1] >> 16 == 2
        for i, d in enumerate(datas):
            buf = np.concatenate([d, np.zeros(64, np.uint8)])
            assert st[i] == 0
            assert got[i].tobytes() == oracle_native.checksums(buf, [0], [len(d)])[0].tobytes(), sizes[i]


def test_c_oracle_file_checksum_short_read_of_a_pipe(oracle_native, tmp_path):
    """A FIFO reports st_size 0; hash.rs hashes what its first read returns and stops at
    that short read.  One atomic write of 4000 bytes (< PIPE_BUF) makes it deterministic."""
    import os
    import threading
    fifo = str(tmp_path / "fifo")
    os.mkfifo(fifo)
    payload = cs.synth_bytes(99, 0, 0, 4000)

    def writer():
        with open(fifo, "wb", buffering=0) as f:
            f.write(payload)

    t = threading.Thread(target=writer)
    t.start()
    got, st = oracle_native.file_checksums([fifo], nthreads=1, simd=0)
    t.join()
    assert st[0] == 0 and got[0].tobytes() == b3.blake3(payload)


def test_c_oracle_checksum_mt_equals_streaming(oracle_native):
    """The chunk-parallel checker (used for multi-GiB GPU parity) equals the streaming
    restatement of hash.rs:14-20 across block, chunk and 1 MiB window boundaries."""
    for size in [0, 1, 1024, 1025, 2048, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 3 * (1 << 20) + 5, 9_999_999]:
        want = oracle_native.checksums_synth(np.array([size], np.uint64), np.array([9], np.uint64),
                                             np.array([3], np.uint32))[0].tobytes()
        for nt in (1, 3):
            assert oracle_native.checksum_synth_mt(size, 9, 3, nthreads=nt) == want, (size, nt)


def test_checksum_mt_over_memory_equals_simd(oracle_native):
    # the chunk-parallel in-memory checker (used for multi-GiB files in the GPU tests)
    # agrees with the per-message SIMD restatement at the block and chunk boundaries
    rng = np.random.default_rng(17)
    for n in (0, 1, 1024, 1025, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, (3 << 20) + 777):
        d = rng.integers(0, 256, n + 64, dtype=np.uint8)
        want = oracle_native.checksums_simd(d, [0], [n], nthreads=1)[0].tobytes()
        assert oracle_native.checksum_mt(d, n, nthreads=3) == want, n


def test_stage_synth_threaded_equals_serial(oracle_native):
    # the CPU baseline stages its shard with several threads: the bytes (and the prefix the
    # legs hash) are the same as one thread's
    from spacedrive_amd import synth
    from spacedrive_amd.device import stage_plan
    sizes, cids, twins = synth.library(3, 6000, 6000)
    ext, total = stage_plan(sizes)
    one = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total)
    many = oracle_native.stage_synth(sizes, cids, twins, ext["msg_offset"], total, nthreads=5)
    assert np.array_equal(one, many)
    e2, t2 = stage_plan(sizes[:2500])
    assert np.array_equal(e2, ext[:2500])
    part = oracle_native.stage_synth(sizes[:2500], cids[:2500], twins[:2500], e2["msg_offset"], t2)
    assert np.array_equal(part[:t2], one[:t2])
